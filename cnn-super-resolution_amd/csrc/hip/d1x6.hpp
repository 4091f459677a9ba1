// d1x6.hpp -- kernel 3 of the fused step (delta1 + gW1/gB1 + gW2/gB2) for
// the reference default net (n1 = 64, n2 = 32, f1 = 9) in split-bf16
// products (split.hpp), paired with l12x6 (its A1 layout and pixel order,
// runs.hpp).  Included by train_fused.hip inside namespace srcnn::fused.
// Same mathematics as d1c_grad12_kernel (layer_deltas.cl:42-127 with f = 1,
// backpropagate.cl:56-114 for layers 1 and 2).
//
// One wave per chunk of 32 slots (8 runs of 4 pixels), all 64 channels, on
// v_mfma_f32_32x32x16_bf16 (x6: six part products per 16-slot k-step):
//   delta1[p][c] = sum_n delta2[p][n] W2[c][n]       M = slots, N = channels
//                  (2 tiles), K = n2 (2 k-steps); delta2 rows straight from
//                  HBM (lane = slot), W2 a split image in LDS.  The result
//                  has the CHANNEL on the lane and the slots in registers
//                  (register r of half h = slot crow(r, h)), the layout of
//                  l12x6's transposed A1 loads, so relu'(A1) is elementwise
//   gW2[c][n] += sum_p A1[p][c] delta2[p][n]         K = slots: A = A1^T as
//                  loaded, B = delta2^T through a per-wave LDS transpose
//   gW1[t][c] += sum_p X[p + off(t)] delta1[p][c]    written as gW1^T: M =
//                  channels, N = taps (3 tiles: 81 taps, the ones column of
//                  gB1, zeros), K = slots; A = delta1 as it stands, B = X
//                  windows: the slots of k-step m, half h are runs 4m + h and
//                  4m + 2 + h, each 4 consecutive X values under any tap --
//                  one ds_read2_b32 per run and part from part-interleaved
//                  pair images (row runs: R; column runs: T, column-major)
//   gB2[n] += sum_p delta2[p][n]                     VALU over delta2^T
// Each wave accumulates over its chunks; at the end the four waves' sums are
// added in wave order through LDS and the block writes one slab (summed by
// slab_reduce in block order).  (One slab per wave was 4x the slab traffic:
// 30 MB written and read back per step.)
// One wave per SIMD (512 registers: 128 accumulators + operands).

constexpr int kD6W2 = 2 * 2 * 3 * 512;  // delta1's W2 image, bf16: [t][k][part][lane][8]
constexpr int kD6Sc = 32 * 36;           // per-wave delta2 transpose scratch (floats)

struct D6Lds {
  int st;      // T image column stride (dwords per column, >= 4 cr + 9)
  int tcols;   // T image columns (the column runs' x range + 8)
  int rs;      // R image row stride (pixels): the least >= w with rs = 9 (mod 64)
  int rdw;     // R image dwords (3 parts interleaved)
  int tdw;     // T image dwords
  int xbuf;    // one X buffer (dwords): R then T
  int w2, xb, sc, slots, runs, bytes;  // byte offsets
  __host__ __device__ D6Lds(int w, int h, const RunGeom& rg) {
    st = 4 * rg.cr + 9;
    if (st < h + 1) st = h + 1;
    tcols = rg.b ? rg.b + 8 : 0;
    // a tap (dy, dx) of gW1's X operand sits 3 (dy rs + dx) dwords past its
    // run base, = 3 (9 dy + dx) = 3 tap (mod 64) for rs = 9 (mod 64): the 32
    // taps of a half-wave hit 32 distinct banks (at rs = w = 33 two taps
    // shared a bank: 53% of d1x6's LDS-active cycles were bank conflicts)
    rs = w + ((9 - w) % 64 + 64) % 64;
    rdw = 3 * (rs * h + 1);
    tdw = 3 * tcols * st;
    xbuf = rdw + tdw;
    w2 = 0;
    xb = kD6W2 * 2;
    sc = xb + 2 * xbuf * 4;
    sc = (sc + 15) & ~15;
    slots = sc + 4 * kD6Sc * 4;
    runs = slots + rg.nch * 32 * 4;
    bytes = runs + rg.nch * 8 * 4;
  }
};

inline bool d1x6_fits(int w, int h) {
  const RunGeom rg = run_geom(w - 8, h - 8);
  return w <= 57 && D6Lds(w, h, rg).bytes <= 150 * 1024;
}

__global__ __launch_bounds__(256, 1) void d1x6_grad12_kernel(const float* __restrict__ X,
                                                              const float* __restrict__ A1T,
                                                              const float* __restrict__ D2,
                                                              const float* __restrict__ W2,
                                                              float* __restrict__ slab, Geom g, RunGeom rg) {
  constexpr int N1 = 64, N2 = 32, F1 = 9, K1 = F1 * F1;
  constexpr int NW1 = K1 * N1, NW2 = N1 * N2, P12 = NW1 + N1 + NW2 + N2;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const D6Lds L(g.W, g.H, rg);
  char* const base = reinterpret_cast<char*>(smem);
  __bf16* const w2i = reinterpret_cast<__bf16*>(base + L.w2);
  uint32_t* const xbuf = reinterpret_cast<uint32_t*>(base + L.xb);
  int* const slots = reinterpret_cast<int*>(base + L.slots);
  int* const runs = reinterpret_cast<int*>(base + L.runs);

  SRCNN_CLOCK_BEGIN();
  const int lane = mfma::lane_id(), wave = mfma::wave_id();
  const int h = lane >> 5, li = lane & 31;
  const int W = g.W, xn = g.W * g.H, npx = g.ow * g.oh, nch = rg.nch;
  const int x0col = 4 * rg.a;  // first column of the column runs

  float xr[kL12Regs];
  auto xload = [&](int smp) {
    const float* src = X + (size_t)smp * xn;
#pragma unroll
    for (int k = 0; k < kL12Regs; k++) {
      const int i = threadIdx.x + 256 * k;
      xr[k] = i < xn ? src[i] : 0.0f;
    }
  };
  if ((int)blockIdx.x < g.batch) xload(blockIdx.x);

  // ---- per-block tables and images ----
  for (int i = threadIdx.x; i < nch * 32; i += 256) slots[i] = slot_pixel(rg, i >> 5, i & 31);
  for (int k = threadIdx.x; k < nch * 8; k += 256) {
    int iy, ix;
    bool col;
    run_origin(rg, k < rg.nrun ? k : 0, iy, ix, col);
    runs[k] = col ? ~(L.rdw + 3 * ((ix - x0col) * L.st + iy)) : 3 * (iy * L.rs + ix);
  }
  // T rows past the tile (and the pair partner of the last row), and the R
  // rows' pad columns, stay zero
  for (int i = threadIdx.x; i < L.xbuf; i += 256) {
    xbuf[i] = 0u;
    xbuf[L.xbuf + i] = 0u;
  }
  {
    // delta1's B operand W2^T: tile t, k-step k, lane (c, h), element j <->
    // W2[32 t + c][16 k + 8 h + j]
    constexpr int kIt = 2 * 2 * 64 * 8 / 256;
    float v[kIt];
#pragma unroll
    for (int k = 0; k < kIt; k++) {
      const int e = threadIdx.x + 256 * k;
      const int j = e & 7, L_ = (e >> 3) & 63, kk = (e >> 9) & 1, t = e >> 10;
      v[k] = W2[(32 * t + (L_ & 31)) * N2 + 16 * kk + 8 * (L_ >> 5) + j];
    }
#pragma unroll
    for (int k = 0; k < kIt; k++) {
      const int e = threadIdx.x + 256 * k;
      const int j = e & 7, L_ = (e >> 3) & 63, kk = (e >> 9) & 1, t = e >> 10;
      __bf16 p[3];
      split3(v[k], p[0], p[1], p[2]);
#pragma unroll
      for (int q = 0; q < 3; q++) w2i[((t * 2 + kk) * 3 + q) * 512 + L_ * 8 + j] = p[q];
    }
  }

  // gW1 operand offsets of this lane's tap 32u + li (3 dwords per pair position)
  int offR3[3], offT3[3];
#pragma unroll
  for (int u = 0; u < 3; u++) {
    const int tap = 32 * u + li;
    const int dy = tap < K1 ? tap / F1 : 0, dx = tap < K1 ? tap - dy * F1 : 0;
    offR3[u] = 3 * (dy * L.rs + dx);
    offT3[u] = 3 * (dx * L.st + dy);
  }
  const bool ones = li == K1 - 64;  // tile 2: tap 81 is the ones column (gB1)
  const bool zcol = li > K1 - 64;   // tile 2: taps 82..95 are zero

  f32x16 g1[2][3], g2[2];
#pragma unroll
  for (int t = 0; t < 2; t++) {
    g2[t] = zero16();
#pragma unroll
    for (int u = 0; u < 3; u++) g1[t][u] = zero16();
  }
  float gb2 = 0.0f;

  float* const sc = smem + L.sc / 4 + wave * kD6Sc;
  const uint16_t* const wl2 = reinterpret_cast<const uint16_t*>(w2i) + lane * 8;

  // chunk operands from HBM, one chunk ahead: delta2 rows of this lane's slot
  // (n = 8h .. 8h+7 and 16 + 8h ..), A1^T runs of this lane's channel
  f32x4 d2n[4], a1n[2][4];
  auto load_chunk = [&](int smp, int c) {
    const int pix = slots[c * 32 + li];
    const float* d2 = D2 + ((size_t)smp * npx + (pix >= 0 ? pix : 0)) * N2 + 8 * h;
#pragma unroll
    for (int k = 0; k < 4; k++) {
      d2n[k] = *reinterpret_cast<const f32x4*>(d2 + 16 * (k >> 1) + 4 * (k & 1));
      if (pix < 0) d2n[k] = mfma::zero4();
    }
    const float* a1 = A1T + ((size_t)smp * nch + c) * (64 * 32) + li * 32 + 4 * h;
#pragma unroll
    for (int t = 0; t < 2; t++)
#pragma unroll
      for (int q = 0; q < 4; q++) a1n[t][q] = *reinterpret_cast<const f32x4*>(a1 + t * 32 * 32 + 8 * q);
  };

  // The block's chunks form one stream (sample j of the block = blockIdx.x +
  // j * gridDim.x, chunks 0 .. nch-1 each); wave w takes stream items w,
  // w + 4, ... -- (wj, wc) is its next one
  int wj = 0, wc = wave;
  auto normalize = [&]() {
    while (wc >= nch) {
      wc -= nch;
      wj++;
    }
  };
  normalize();
  __syncthreads();  // tables
  if ((int)blockIdx.x + wj * (int)gridDim.x < g.batch) load_chunk(blockIdx.x + wj * gridDim.x, wc);
  // the current chunk's operands: copied from the prefetch registers at the
  // END of the previous chunk (here for the first), so the copy's wait never
  // covers the next sample's X loads, issued at each sample's top (a copy at
  // the chunk's top waited out those HBM loads once per sample)
  f32x4 d2c[4], a1c[2][4];
  auto take_chunk = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int k = 0; k < 4; k++) d2c[k] = d2n[k];
#pragma unroll
    for (int t = 0; t < 2; t++)
#pragma unroll
      for (int q = 0; q < 4; q++) a1c[t][q] = a1n[t][q];
  };
  take_chunk();
  for (int it = 0; (int)blockIdx.x + it * (int)gridDim.x < g.batch; it++) {
    const int smp = blockIdx.x + it * gridDim.x;
    uint32_t* const xi = xbuf + (it & 1) * L.xbuf;
    // ---- this sample's X pair images (buffer it & 1) ----
    {
      uint16_t* const x16 = reinterpret_cast<uint16_t*>(xi);
#pragma unroll
      for (int k = 0; k < kL12Regs; k++) {
        const int i = threadIdx.x + 256 * k;
        if (i < xn) {
          __bf16 p[3];
          split3(xr[k], p[0], p[1], p[2]);
          const int y = i / W, x = i - y * W, ri = y * L.rs + x;
          const int ti = L.rdw + 3 * ((x - x0col) * L.st + y);
#pragma unroll
          for (int q = 0; q < 3; q++) {
            const uint16_t b = __builtin_bit_cast(uint16_t, p[q]);
            x16[2 * (3 * ri + q)] = b;
            if (ri > 0) x16[2 * (3 * (ri - 1) + q) + 1] = b;
            if (L.tcols && x >= x0col) {
              x16[2 * (ti + q)] = b;
              if (y > 0) x16[2 * (ti - 3 + q) + 1] = b;
            }
          }
        }
      }
    }
    __syncthreads();  // images (and at it == 0 the tables) complete; buffer (it+1)&1 free
    const int nsmp = smp + (int)gridDim.x;
    if (nsmp < g.batch) xload(nsmp);

    while (wj == it) {
      const int c = wc;
      // (this chunk's operands are in d2c / a1c); the next chunk's loads go out now
      wc += 4;
      normalize();
      if ((int)blockIdx.x + wj * (int)gridDim.x < g.batch) load_chunk(blockIdx.x + wj * gridDim.x, wc);

      // delta2 rows -> scratch [slot][n] (row stride 36), read back transposed
#pragma unroll
      for (int k = 0; k < 4; k++)
        *reinterpret_cast<f32x4*>(sc + li * 36 + 16 * (k >> 1) + 8 * h + 4 * (k & 1)) = d2c[k];
      __builtin_amdgcn_wave_barrier();
      float d2t[16];
#pragma unroll
      for (int r = 0; r < 16; r++) d2t[r] = sc[crow(r, h) * 36 + li];

      // ---- delta1 = delta2 . W2^T (lane = channel, registers = slots) ----
      bf16x8 da[2][3];
#pragma unroll
      for (int k = 0; k < 2; k++) {
        float v[8];
#pragma unroll
        for (int j = 0; j < 8; j++) v[j] = d2c[2 * k + (j >> 2)][j & 3];
        split8_pk(v, da[k]);
      }
      f32x16 d1[2];
#pragma unroll
      for (int t = 0; t < 2; t++) {
        d1[t] = zero16();
#pragma unroll
        for (int k = 0; k < 2; k++) {
          bf16x8 b[3];
#pragma unroll
          for (int q = 0; q < 3; q++)
            b[q] = *reinterpret_cast<const bf16x8*>(wl2 + ((t * 2 + k) * 3 + q) * 512);
          d1[t] = mma_x6(da[k], b, d1[t]);
        }
      }

      // ---- gW2 += A1^T . delta2 (k-step m: registers 8m .. 8m+7) ----
      bf16x8 db[2][3];
#pragma unroll
      for (int m = 0; m < 2; m++) {
        float v[8];
#pragma unroll
        for (int j = 0; j < 8; j++) v[j] = d2t[8 * m + j];
        split8_pk(v, db[m]);
      }
#pragma unroll
      for (int r = 0; r < 16; r++) gb2 += d2t[r];
#pragma unroll
      for (int t = 0; t < 2; t++)
#pragma unroll
        for (int m = 0; m < 2; m++) {
          float v[8];
#pragma unroll
          for (int j = 0; j < 8; j++) v[j] = a1c[t][2 * m + (j >> 2)][j & 3];
          bf16x8 a[3];
          split8_pk(v, a);
          g2[t] = mma_x6(a, db[m], g2[t]);
        }

      // relu' of layer 1 (register r of d1[t] and a1c[t] is the same slot)
#pragma unroll
      for (int t = 0; t < 2; t++)
#pragma unroll
        for (int r = 0; r < 16; r++) d1[t][r] = a1c[t][r >> 2][r & 3] > 0.0f ? d1[t][r] : 0.0f;

      // ---- gW1^T += delta1^T . Xwin ----
      // run codes of this lane's half: k-step m takes runs 4m + h, 4m + 2 + h
      int rc4[2][2];
#pragma unroll
      for (int m = 0; m < 2; m++)
#pragma unroll
        for (int e = 0; e < 2; e++) rc4[m][e] = runs[8 * c + 4 * m + 2 * e + h];
#pragma unroll
      for (int m = 0; m < 2; m++) {
        bf16x8 a1x[2][3];
#pragma unroll
        for (int t = 0; t < 2; t++) {
          float v[8];
#pragma unroll
          for (int j = 0; j < 8; j++) v[j] = d1[t][8 * m + j];
          split8_pk(v, a1x[t]);
        }
#pragma unroll
        for (int u = 0; u < 3; u++) {
          u32x4 d[3];
#pragma unroll
          for (int e = 0; e < 2; e++) {
            const int code = rc4[m][e];
            const uint32_t* p = xi + (code >= 0 ? code + offR3[u] : ~code + offT3[u]);
#pragma unroll
            for (int q = 0; q < 3; q++) {
              d[q][2 * e] = p[q];
              d[q][2 * e + 1] = p[q + 6];
            }
          }
          bf16x8 b[3];
#pragma unroll
          for (int q = 0; q < 3; q++) {
            if (u == 2) {
              const uint32_t one = q == 0 ? 0x3F803F80u : 0u;
#pragma unroll
              for (int e = 0; e < 4; e++) d[q][e] = ones ? one : zcol ? 0u : d[q][e];
            }
            b[q] = __builtin_bit_cast(bf16x8, d[q]);
          }
#pragma unroll
          for (int t = 0; t < 2; t++) g1[t][u] = mma_x6(a1x[t], b, g1[t][u]);
        }
      }
      take_chunk();  // the next chunk's operands (loaded under this chunk)
    }
  }
  SRCNN_CLOCK_END(g_clk, 2);

  // ---- block reduction: waves 1-3 hand their accumulators to wave 0 one
  // 16-register tile at a time, added in wave order (fixed, deterministic) ----
  __syncthreads();  // every wave is done with the LDS images
  float* const red = smem;  // [3 waves][16 registers][64 lanes]
  auto reduce_tile = [&](f32x16& acc) {
    if (wave > 0) {
#pragma unroll
      for (int r = 0; r < 16; r++) red[((wave - 1) * 16 + r) * 64 + lane] = acc[r];
    }
    __syncthreads();
    if (wave == 0) {
#pragma unroll
      for (int w = 0; w < 3; w++)
#pragma unroll
        for (int r = 0; r < 16; r++) acc[r] += red[(w * 16 + r) * 64 + lane];
    }
    __syncthreads();
  };
#pragma unroll
  for (int t = 0; t < 2; t++) {
#pragma unroll
    for (int u = 0; u < 3; u++) reduce_tile(g1[t][u]);
    reduce_tile(g2[t]);
  }
  if (wave > 0) red[(wave - 1) * 64 + lane] = gb2;
  __syncthreads();
  if (wave == 0) {
#pragma unroll
    for (int w = 0; w < 3; w++) gb2 += red[w * 64 + lane];
  }
  if (wave != 0) return;

  // ---- the block's slab: [gW1 | gB1 | gW2 | gB2] ----
  float* out = slab + (size_t)blockIdx.x * P12;
#pragma unroll
  for (int t = 0; t < 2; t++)
#pragma unroll
    for (int u = 0; u < 3; u++) {
      const int tap = 32 * u + li;
#pragma unroll
      for (int r = 0; r < 16; r++) {
        const int ch = 32 * t + crow(r, h);
        if (tap < K1)
          out[tap * N1 + ch] = g1[t][u][r];
        else if (tap == K1)
          out[NW1 + ch] = g1[t][u][r];
      }
    }
#pragma unroll
  for (int t = 0; t < 2; t++)
#pragma unroll
    for (int r = 0; r < 16; r++) out[NW1 + N1 + (32 * t + crow(r, h)) * N2 + li] = g2[t][r];
  gb2 += __shfl_xor(gb2, 32, 64);
  if (h == 0) out[NW1 + N1 + NW2 + li] = gb2;
}
