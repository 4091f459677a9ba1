// d1c.hpp -- kernel 3 of the fused step (delta1 + gW2/gB2 + gW1/gB1) in the
// cooperative-chunk form, for the reference default net (n1 = 64, n2 = 32).
// Included by train_fused.hip inside namespace srcnn::fused.
//
// Same mathematics as d1_grad12_kernel (layer_deltas.cl:42-127 with f = 1,
// backpropagate.cl:56-114 for layers 1 and 2), different work split: the four
// waves of a block work on ONE 32-pixel chunk at a time, wave w owning the
// 16 channels [16w, 16w + 16) of layer 1:
//   delta1[p][c] = sum_n delta2[p][n] W2[c][n]   16x16x4 MFMA, M = pixels
//                  (2 tiles), N = the wave's 16 channels, K = n2; W2 in registers
//   gW2[c][n] += sum_p A1[p][c] delta2[p][n]     M = the wave's 16 channels,
//                  N = n2 (2 tiles), K = the chunk's pixels; gB2 by VALU adds
//   delta1 *= [A1 > 0]                           (relu' of layer 1)
//   gW1[t][c] += sum_p X[p + off(t)] delta1[p][c] M = taps 0..79 (5 tiles),
//                  N = the wave's channels, K = pixels; delta1's accumulator
//                  registers are the B operand as they stand; tap 80 and the
//                  ones row (gB1) by VALU FMAs
// So a wave holds the gradient tiles of 16 channels only (30 accumulators
// instead of 121), which lets 4 blocks (4 waves per SIMD) share a CU, and no
// cross-wave gradient reduction is needed.  Each wave DMAs its own quarter of
// the chunk's A1 (2 KB) and a quarter of its delta2 (4 KB, shared through a
// block barrier per chunk), one work item ahead, double-buffered.
//
// LDS images (16-B LDS-DMA slots; the DMA picks each lane's source quad):
//   delta2 [32 px][8 quads], quad q of pixel p in slot q ^ f(p),
//          f(p) = 4 bit1(p) | bit2(p): the delta1 operand ds_read_b128 (pixel
//          16 pm + lq, quads 2 lg + hf) and the gW2 operand ds_read_b32 (pixel
//          4 s + {0,3,1,2}[lg]) are both bank-conflict free
//   A1     per wave [32 slots][16 channels], pixel p in slot p ^ bit2(p): the
//          gW2 operand and relu' mask reads are conflict free
//   X      the sample tile at row stride kD1cS = 40 (8 mod 32; tiles up to
//          40 px wide).  gW1's tap tiles 0-3 are the 4x4 tap blocks at
//          (dy, dx) = (0,0), (0,4), (4,0), (4,4): lane lq takes tap
//          (dy0 + lq/4, dx0 + lq%4), so a tile's gather is one per-lane base
//          plus a compile-time offset, conflict free (4 rows 8 banks apart);
//          tile 4 holds row 8 and column 8 (rows 0-6), tap (7,8) goes to VALU
//   pixel -> X offset table (ints, one per pixel slot of the sample): the 4
//          offsets of a lane's k-steps are one ds_read_b128 per pixel tile
// M0 is written by the DMA asm only; the compiler sets it itself around its own uses
#pragma clang diagnostic ignored "-Winline-asm"

// 4-wave teams per block, on alternate chunks of a sample (two teams per
// block, 512 slabs instead of 1024: d1 0.4065 vs 0.399 ms)
constexpr int kD1cTeams = 1;
constexpr int kD1cOcc = 4;                           // waves per SIMD (launch bound: 128 VGPRs)
constexpr int kD1cGrid = 256 * kD1cOcc / kD1cTeams;  // all blocks resident
constexpr int kD1cS = 40;       // X tile row stride in LDS (8 mod 32)
constexpr int kD1cMaxPx = 1024; // pixel slots of the X offset table (nch * 32)

__device__ float g_d1c_zero[4] = {0.0f, 0.0f, 0.0f, 0.0f};  // 16-B zero source (delta2 rows past the sample)

// LDS-DMA as inline asm (train_wide.hip, dma16): through the builtin the
// compiler puts an s_waitcnt vmcnt(0) before later LDS reads of the current
// buffer; consumers reach DMA'd data through the explicit wait + barrier.
__device__ __forceinline__ uint32_t d1c_m0(const float* lds_dst) {
  return __builtin_amdgcn_readfirstlane(
      (uint32_t)reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) void*)lds_dst));
}
// 16 B per lane from a 64-bit per-lane address
__device__ __forceinline__ void d1c_dma16v(const float* src, float* lds_dst) {
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off"
               : : "s"(d1c_m0(lds_dst)), "v"(src) : "m0");
}
// 16 B per lane from a wave-uniform base + 32-bit per-lane byte offset
__device__ __forceinline__ void d1c_dma16s(const float* base, uint32_t off, float* lds_dst) {
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2"
               : : "s"(d1c_m0(lds_dst)), "v"(off), "s"(base) : "m0");
}
__device__ __forceinline__ void d1c_dma4s(const float* base, uint32_t off, float* lds_dst) {
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dword %1, %2"
               : : "s"(d1c_m0(lds_dst)), "v"(off), "s"(base) : "m0");
}

inline bool d1c_fits(int w, int h) { return w <= kD1cS && ((w - 8) * (h - 8) + 31) / 32 * 32 <= kD1cMaxPx; }
inline int d1c_xs_floats(int h) { return (kD1cS * h + 63) / 64 * 64; }
inline size_t d1c_lds_bytes(int w, int h) {
  return (size_t)(kD1cTeams * 6144 + 2 * d1c_xs_floats(h) + ((w - 8) * (h - 8) + 31) / 32 * 32) * sizeof(float);
}

template <int F1>
__global__ __launch_bounds__(256 * kD1cTeams, kD1cOcc) void d1c_grad12_kernel(const float* __restrict__ X,
                                                            const float* __restrict__ A1,
                                                            const float* __restrict__ D2,
                                                            const float* __restrict__ W2,
                                                            float* __restrict__ slab, Geom g, int xsf,
                                                            int parts) {
  constexpr int N1 = 64, N2 = 32, S = kD1cS;
  static_assert(F1 == 9, "d1c: the tap tiling is for 9x9 layer-1 filters");
  constexpr int K1 = F1 * F1, NW1 = K1 * N1, NW2 = N1 * N2, P12 = NW1 + N1 + NW2 + N2;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  constexpr int NT = kD1cTeams;
  const int lane = mfma::lane_id(), wv = mfma::wave_id();
  const int team = wv >> 2, wave = wv & 3;  // team t takes chunks t, t + NT, ...
  float* const a1i = smem + team * 6144;         // per team: [2 buffers][4 waves][512]
  float* const d2i = smem + team * 6144 + 4096;  // per team: [2 buffers][1024]
  float* const xsi = smem + NT * 6144;           // [2 samples][xsf]
  int* const xo = reinterpret_cast<int*>(xsi + 2 * xsf);  // [nch * 32] pixel -> X offset

  SRCNN_CLOCK_BEGIN();
  const int lq = lane & 15, lg = lane >> 4;
  const int c0 = 16 * wave;
  const int npx = g.ow * g.oh, nch = (npx + 31) / 32;
  for (int q = threadIdx.x; q < nch * 32; q += blockDim.x) {
    const int qc = min(q, npx - 1), y = qc / g.ow;
    xo[q] = y * S + qc - y * g.ow;
  }

  // delta1 B operand: k-step s, lane group lg <-> n = 8 lg + s
  float w2r[8];
#pragma unroll
  for (int s = 0; s < 8; s++) w2r[s] = W2[(c0 + lq) * N2 + 8 * lg + s];
  // wait for W2 here: left alone, the compiler puts that wait (as vmcnt(0)) at
  // the first use inside the chunk loop, where it also waits out the operand
  // DMA just issued for the next chunk
#pragma unroll
  for (int s = 0; s < 8; s++) asm volatile("" : "+v"(w2r[s]));
  // gW1 A-operand bases: tiles 0-3 at lane tap (lq/4, lq%4) + the block
  // origin (compile-time), tile 4 at its own per-lane tap (row 8, then
  // column 8 rows 0-6); the remaining tap (7, 8) by VALU FMAs
  const int tb = (lq >> 2) * S + (lq & 3);
  const int t4 = lq < 9 ? 8 * S + lq : (lq - 9) * S + 8;
  constexpr int kTileOff[4] = {0, 4, 4 * S, 4 * S + 4};

  f32x4 g1[5], g2[2];
#pragma unroll
  for (int m = 0; m < 5; m++) g1[m] = mfma::zero4();
  g2[0] = g2[1] = mfma::zero4();
  float gv = 0.0f, gvb = 0.0f, gb2[2] = {0.0f, 0.0f};

  // LDS read bases (floats within one buffer)
  const int fq = (((lq >> 1) & 1) << 2) | ((lq >> 2) & 1);  // f(16 pm + lq)
  const int r1b0 = 32 * lq + 4 * ((2 * lg) ^ fq), r1b1 = 32 * lq + 4 * ((2 * lg + 1) ^ fq);
  const int pl = (0x2130 >> (4 * lg)) & 15;  // gW2 pixel 4 s + pl, pl = {0, 3, 1, 2}[lg]
  const int b1 = (pl >> 1) & 1;
  int r2b[2][2], r3b[2];
#pragma unroll
  for (int s1 = 0; s1 < 2; s1++) {
#pragma unroll
    for (int u = 0; u < 2; u++) r2b[u][s1] = 32 * pl + 16 * (u ^ b1) + 4 * ((lq >> 2) ^ s1) + (lq & 3);
    r3b[s1] = 16 * (pl ^ s1) + lq;
  }
  const int r4e = 64 * lg + lq + 16 * (lg & 1), r4o = 64 * lg + lq - 16 * (lg & 1);

  // DMA source offsets (bytes), fixed per lane: A1 quad j of pixel p in the
  // blocked chunk (l12), delta2 quad q of chunk pixel dp
  uint32_t a1off[2];
#pragma unroll
  for (int k = 0; k < 2; k++) {
    const int Q = 64 * k + lane, sp = Q >> 2, q = Q & 3;
    const int p = sp ^ ((sp >> 2) & 1), j = 4 * wave + q;
    a1off[k] = 4u * ((j >> 1) * 256 + 4 * (p + 32 * (j & 1)));
  }
  const int dp = (64 * wave + lane) >> 3;
  const uint32_t d2off = 4u * (dp * N2 + 4 * ((lane & 7) ^ ((((dp >> 1) & 1) << 2) | ((dp >> 2) & 1))));
  // chunk (smp, c) operands -> buffer b: this wave's A1 quarter (2 instructions),
  // delta2 instruction `wave` of 4
  auto dma_chunk = [&](int smp, int c, int b) {
    const float* a1c = A1 + ((size_t)smp * nch + c) * (32 * N1);
#pragma unroll
    for (int k = 0; k < 2; k++) d1c_dma16s(a1c, a1off[k], a1i + (b * 4 + wave) * 512 + 256 * k);
    const float* d2c = D2 + ((size_t)smp * npx + c * 32) * N2;
    float* dst = d2i + b * 1024 + 256 * wave;
    if (c * 32 + 32 <= npx) {
      d1c_dma16s(d2c, d2off, dst);
    } else {  // the sample's last chunk: rows past it read zeros
      int l_ = lane;
      asm volatile("" : "+v"(l_));
      const int p = (64 * wave + l_) >> 3;
      d1c_dma16v(c * 32 + p < npx ? d2c + d2off / 4 : g_d1c_zero, dst);
    }
  };
  // X tile of sample smp -> dst at row stride S (pad slots read a clamped pixel)
  auto dma_x = [&](int smp, float* dst) {
    const float* xsrc = X + (size_t)smp * g.W * g.H;
    for (int k = wv; 64 * k < S * g.H; k += 4 * NT) {
      int l_ = lane;
      asm volatile("" : "+v"(l_));
      const int f = 64 * k + l_, r = f / S;
      d1c_dma4s(xsrc, 4u * (min(r, g.H - 1) * g.W + min(f - r * S, g.W - 1)), dst + 64 * k);
    }
  };

  // work items: (sample, part), `parts` consecutive chunk ranges per sample
  // (parts > 1 only for small batches, so that every CU keeps its 4 blocks)
  const int cpp = (nch + parts - 1) / parts;  // chunks per part
  const int nitems = g.batch * parts;
  auto first_chunk = [&](int it) { return (it % parts) * cpp; };
  auto end_chunk = [&](int it) { return min(nch, (it % parts) * cpp + cpp); };
  int buf = 0, xbuf = 0;
  if ((int)blockIdx.x < nitems) {
    const int it0 = blockIdx.x;
    dma_x(it0 / parts, xsi);
    if (first_chunk(it0) + team < end_chunk(it0)) dma_chunk(it0 / parts, first_chunk(it0) + team, 0);
  }
  for (int it = blockIdx.x; it < nitems; it += gridDim.x, xbuf ^= 1) {
    const int smp = it / parts, c_beg = first_chunk(it), c_end = end_chunk(it);
    const int nit = it + (int)gridDim.x;  // the next work item
    const float* xs = xsi + xbuf * xsf;
    for (int cc = c_beg; cc < c_end; cc += NT, buf ^= 1) {
      // this chunk's operands (and at cc == c_beg this item's X tile) have
      // landed for every wave; every wave is done with the other buffer
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      const int c = cc + team;
      if (c + NT < c_end)
        dma_chunk(smp, c + NT, buf ^ 1);
      else if (nit < nitems && first_chunk(nit) + team < end_chunk(nit))
        dma_chunk(nit / parts, first_chunk(nit) + team, buf ^ 1);
      if (cc == c_beg && nit < nitems) dma_x(nit / parts, xsi + (xbuf ^ 1) * xsf);
      if (c >= c_end) continue;  // odd chunk count: this team idles on the last step
      const float* d2b = d2i + buf * 1024;
      const float* a1b = a1i + (buf * 4 + wave) * 512;

      // relu' operands of layer 1 first (A1 > 0; register i of d1[pm] below is
      // pixel 16 pm + 4 lg + i), so their LDS latency hides under delta1 and
      // gW2 (read just before the mask, they cost 3% of the kernel)
      float mk[2][4];
#pragma unroll
      for (int pm = 0; pm < 2; pm++)
#pragma unroll
        for (int i = 0; i < 4; i++)
          mk[pm][i] = a1b[256 * pm + 16 * i + ((i & 1) ? r4o : r4e)];
      // delta1 (its operands: two 16-B reads per pixel tile)
      f32x4 av[2][2], d1[2];
#pragma unroll
      for (int pm = 0; pm < 2; pm++) {
        av[pm][0] = *reinterpret_cast<const f32x4*>(d2b + 512 * pm + r1b0);
        av[pm][1] = *reinterpret_cast<const f32x4*>(d2b + 512 * pm + r1b1);
        d1[pm] = mfma::zero4();
      }
      // gW1's pixel -> X-tile offsets of the chunk (k-step k = (pm, i) of
      // lane group lg is pixel 16 pm + 4 lg + i)
      const int4 xb4[2] = {*reinterpret_cast<const int4*>(xo + c * 32 + 4 * lg),
                           *reinterpret_cast<const int4*>(xo + c * 32 + 16 + 4 * lg)};
      // gW2 operands (k-step s: pixel 4 s + pl) in a ring of three register
      // sets, read two k-steps ahead of their MFMAs
      float ga[3], gd[3][2];
      auto gw2_read = [&](int s_) {
        ga[s_ % 3] = a1b[64 * s_ + r3b[s_ & 1]];
#pragma unroll
        for (int u = 0; u < 2; u++) gd[s_ % 3][u] = d2b[128 * s_ + r2b[u][s_ & 1]];
      };
      gw2_read(0);
      gw2_read(1);
      __builtin_amdgcn_sched_barrier(0);  // keep the reads above issued first
      // The MFMA order is pinned (sched_barrier per group): a dependent
      // v_mfma_f32_16x16x4_f32 issues 40 cycles after its predecessor but an
      // independent one after 32 (MI355X_MICROARCH.md constants), and left
      // alone the scheduler chains same-accumulator MFMAs back to back.
      // delta1: the two pixel tiles alternate
#pragma unroll
      for (int s = 0; s < 8; s++) {
#pragma unroll
        for (int pm = 0; pm < 2; pm++) d1[pm] = mfma::mma16(av[pm][s >> 2][s & 3], w2r[s], d1[pm]);
        __builtin_amdgcn_sched_barrier(0);
      }

      // gW1's X gathers: the six values of k-step k (tiles 0-4 and the VALU
      // tap) in a ring of three register sets, two k-steps ahead; the first
      // two are issued under gW2's MFMAs
      float xv[3][6];
      auto gather = [&](int k) {
        const int4 v = xb4[k >> 2];
        const int i = k & 3;
        const float* xl = xs + (i == 0 ? v.x : i == 1 ? v.y : i == 2 ? v.z : v.w);
        float* dst = xv[k % 3];
#pragma unroll
        for (int m = 0; m < 4; m++) dst[m] = xl[tb + kTileOff[m]];
        dst[4] = xl[t4];
        dst[5] = xl[7 * S + 8];
      };

      // gW2 += A1^T delta2; the two n2 tiles alternate
#pragma unroll
      for (int s = 0; s < 8; s++) {
        if (s + 2 < 8) gw2_read(s + 2);
        if (s == 4) gather(0);
        if (s == 6) gather(1);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int u = 0; u < 2; u++) g2[u] = mfma::mma16(ga[s % 3], gd[s % 3][u], g2[u]);
        __builtin_amdgcn_sched_barrier(0);
      }
      // gB2 += delta2: wave w sums k-steps 2w, 2w + 1 (balanced; the waves
      // meet at every chunk barrier), the waves' partials are added at the end
#pragma unroll
      for (int u = 0; u < 2; u++)
        gb2[u] += d2b[256 * wave + r2b[u][0]] + d2b[256 * wave + 128 + r2b[u][1]];

      // relu' of layer 1
#pragma unroll
      for (int pm = 0; pm < 2; pm++)
#pragma unroll
        for (int i = 0; i < 4; i++) d1[pm][i] = mk[pm][i] > 0.0f ? d1[pm][i] : 0.0f;

      // gW1 += Xwin^T delta1: k-step k = (pm, i), lane group lg <-> pixel
      // 16 pm + 4 lg + i (pixels past the sample map onto its last one: their
      // delta1 is 0)
#pragma unroll
      for (int k = 0; k < 8; k++) {
        if (k + 2 < 8) gather(k + 2);
        __builtin_amdgcn_sched_barrier(0);
        const float bv = d1[k >> 2][k & 3];
        const float* x = xv[k % 3];
#pragma unroll
        for (int m = 0; m < 5; m++) g1[m] = mfma::mma16(x[m], bv, g1[m]);
        gv = fmaf(x[5], bv, gv);
        gvb += bv;
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  }
  SRCNN_CLOCK_END(g_clk, 2);
  if constexpr (NT == 2) {
    // team 1 parks its partial gradients in LDS, team 0 adds them (fixed order)
    __syncthreads();
    float* red = smem + wave * 32 * 64 + lane;
    if (team == 1) {
#pragma unroll
      for (int m = 0; m < 5; m++)
#pragma unroll
        for (int i = 0; i < 4; i++) red[(4 * m + i) * 64] = g1[m][i];
#pragma unroll
      for (int u = 0; u < 2; u++)
#pragma unroll
        for (int i = 0; i < 4; i++) red[(20 + 4 * u + i) * 64] = g2[u][i];
      red[28 * 64] = gv;
      red[29 * 64] = gvb;
      red[30 * 64] = gb2[0];
      red[31 * 64] = gb2[1];
    }
    __syncthreads();
#pragma unroll
    for (int m = 0; m < 5; m++)
#pragma unroll
      for (int i = 0; i < 4; i++) g1[m][i] += red[(4 * m + i) * 64];
#pragma unroll
    for (int u = 0; u < 2; u++)
#pragma unroll
      for (int i = 0; i < 4; i++) g2[u][i] += red[(20 + 4 * u + i) * 64];
    gv += red[28 * 64];
    gvb += red[29 * 64];
    gb2[0] += red[30 * 64];
    gb2[1] += red[31 * 64];
  }

  // slab of this block: [gW1 | gB1 | gW2 | gB2]; every wave writes its channels.
  // Row 4 lg + i of tile m is the A-operand lane lq' = 4 lg + i, i.e. tap
  // (dy0 + lg, dx0 + i) for tiles 0-3.
  float* out = slab + (size_t)blockIdx.x * P12;
  // (two teams: team 0 holds the sums)
  const bool writer = team == 0;
  if (writer)
#pragma unroll
  for (int m = 0; m < 4; m++)
#pragma unroll
    for (int i = 0; i < 4; i++) {
      const int tap = (4 * (m >> 1) + lg) * F1 + 4 * (m & 1) + i;
      out[tap * N1 + c0 + lq] = g1[m][i];
    }
  if (writer)
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const int l4 = 4 * lg + i;
    const int tap = l4 < 9 ? 8 * F1 + l4 : (l4 - 9) * F1 + 8;
    out[tap * N1 + c0 + lq] = g1[4][i];
  }
  auto lg_sum = [](float v) {  // fixed-order sum over the 4 lane groups (same value in all)
    v += __shfl_xor(v, 16, 64);
    return v + __shfl_xor(v, 32, 64);
  };
  {
    const float v = lg_sum(gv), vb = lg_sum(gvb);
    if (writer && lg == 0) {
      out[(7 * F1 + 8) * N1 + c0 + lq] = v;
      out[NW1 + c0 + lq] = vb;
    }
  }
  if (writer)
#pragma unroll
  for (int u = 0; u < 2; u++)
#pragma unroll
    for (int i = 0; i < 4; i++) out[NW1 + N1 + (c0 + 4 * lg + i) * N2 + 16 * u + lq] = g2[u][i];
  // gB2: the waves' partials in wave order (LDS past the two-team exchange area)
  float* const red2 = smem + (NT == 2 ? 8192 : 0);
  __syncthreads();
#pragma unroll
  for (int u = 0; u < 2; u++) {
    const float v = lg_sum(gb2[u]);
    if (writer && lg == 0) red2[(wave * 2 + u) * 16 + lq] = v;
  }
  __syncthreads();
  if (writer && wave == 0 && lg == 0)
#pragma unroll
    for (int u = 0; u < 2; u++) {
      float v = 0.0f;
#pragma unroll
      for (int w = 0; w < 4; w++) v += red2[(w * 2 + u) * 16 + lq];
      out[NW1 + N1 + NW2 + 16 * u + lq] = v;
    }
}
