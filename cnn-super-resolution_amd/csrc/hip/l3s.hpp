// l3s.hpp -- fused kernel 2 of train_fused.hip in the two-pass streaming form
// (included inside namespace srcnn::fused, after l3_delta.hpp).  Per sample:
//   pass 1   Q = W3 . A2^T per 16-pixel unit (MFMA, K = channels) into an LDS
//            Q image [tap][pixel]
//   window   A3 = B3 + sum_tap Q[tap][p + off(tap)] (layer_uber_kernel.cl:70-91,
//            SKIP_RELU), last delta with the reference's relu' quirk
//            (last_layer_delta.cl:34-48), squared error (squared_error.cl:60-69),
//            gB3; delta3 into a zero-bordered LDS grid
//   pass 2   delta2 = [A2 > 0] (W3^T * delta3) per unit (layer_deltas.cl:79-123,
//            MFMA over the taps) to HBM, gW3 += delta3-windows^T . A2
//            (backpropagate.cl:89-112, MFMA over the pixels)
//
// Unlike l3_delta_kernel, no A2 image lives in LDS: A2 streams from HBM into
// registers (pass 1, two units ahead; the next sample's first two units
// during pass 2) and again from L2 / MALL in pass 2 (the relu' mask and gW3's
// operand, one unit ahead).  The LDS holds only the Q image and the delta3
// grid (68 KB for 33x33 tiles), so two blocks share a CU and one block's
// barrier-separated phases run under the other's MFMAs; l3_delta (160 KB,
// one block per CU) spent a third of each sample waiting at them.
//
// 4 waves per block, 2 blocks (2 waves per SIMD, 256 registers each) per CU;
// a sample's 16-pixel units are dealt round-robin to the waves (625 pixels:
// 40 units, 10 per wave).  Operands ping-pong between two named register sets
// that are reloaded right after the MFMAs that read them: a register copy of
// an operand still in flight would wait for it.  On gfx9 a store counts in
// vmcnt like a load, and waiting for a load also waits for every store
// issued before it, so every load is issued before the stores that precede
// its use.

// diagnostics builds only (results invalid): 1 pass-1 A2 loads from sample 0
// (L2-resident), 2 pass-2 A2 loads from sample 0, 8 D2 stores into sample
// 0's rows (L2-resident)
#ifdef SRCNN_L3S_DIAG
constexpr int kL3sDiag = SRCNN_L3S_DIAG;
#else
constexpr int kL3sDiag = 0;
#endif
constexpr int kL3sThreads = 256;
constexpr int kL3sMaxPx = 640;  // A2 pixels per sample
constexpr int kL3sMaxOut = 2 * kL3sThreads;  // L3 outputs per sample (2 per thread)

// LDS geometry shared by host and device (floats)
template <int N2, int F3>
struct L3sLds {
  int PL;      // Q plane stride: whole units + 4 (= 4 mod 8: a Q store's two
               // 32-lane halves land 16 banks apart)
  int GW, GH;  // delta3 grid: delta3(y, x) at (y + F3-1) * GW + x + F3-1, zero elsewhere
  int zp;      // a cell past the grid with zero cells for every tap offset below it
  int qf, gf;  // floats of the Q image and of the grid (+ its zero tail)
  __host__ __device__ L3sLds(int w2, int h2) {
    PL = 16 * ((w2 * h2 + 15) / 16) + 4;
    GW = w2 + F3 - 1;
    GH = h2 + F3 - 1;
    zp = GW * GH + (F3 - 1) * (GW + 1);
    qf = F3 * F3 * PL;
    gf = (zp + 1 + 3) & ~3;
  }
  __host__ __device__ size_t bytes() const { return (size_t)(qf + gf) * sizeof(float); }
};

template <int N2, int F3>
__global__ __launch_bounds__(kL3sThreads, 2) void l3s_kernel(
    const float* __restrict__ A2, const float* __restrict__ T, const float* __restrict__ W3,
    const float* __restrict__ B3, float* __restrict__ D2, float* __restrict__ slab3,
    float* __restrict__ sq_slab, float* __restrict__ A3out, L3Geom g) {
  constexpr int K3 = F3 * F3;
  constexpr int TT = (K3 + 15) / 16;  // 16-wide tap tiles
  constexpr int NT = N2 / 16;         // 16-wide channel tiles
  constexpr int KT = (K3 + 3) / 4;    // delta2 k-steps (over taps)
  constexpr int KQ = N2 / 4;          // Q k-steps (over channels)
  constexpr int NW3 = K3 * N2;        // gW3 size; slab row = NW3 + 1 (gB3)
  constexpr int NWV = kL3sThreads / 64;
  constexpr int OPT = kL3sMaxOut / kL3sThreads;  // L3 outputs per thread
  static_assert(N2 % 16 == 0 && N2 <= 32 && K3 <= 32, "l3s: n2 16 or 32, f3 <= 5");
  SRCNN_CLOCK_BEGIN();
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int npx2 = g.w2 * g.h2, nunit = (npx2 + 15) / 16, nout = g.w3 * g.h3;
  const L3sLds<N2, F3> L(g.w2, g.h2);
  float* const qs = smem;          // [K3][PL]
  float* const gd = smem + L.qf;   // [GH][GW] + zero tail
  const int tid = threadIdx.x, lane = mfma::lane_id(), wave = mfma::wave_id();
  const int lq = lane & 15, lg = lane >> 4;
  const int pad = (g.W - g.w3) / 2;  // last_layer_delta.cl:25
  const int GW = L.GW, PL = L.PL;
  // (q + 0.5) / w2 in fp32 is at least 0.5 / w2 away from an integer for
  // q < kL3sMaxPx, so the truncation is the exact row of pixel q
  const float inv_w2 = 1.0f / (float)g.w2;
  for (int i = tid; i < L.gf; i += kL3sThreads) gd[i] = 0.0f;

  // grid cell of A2 pixel q; delta3(q - off(tap)) is gd[gpos(q) - goff(tap)]
  auto gpos = [&](int q) {
    const int y = (int)(((float)q + 0.5f) * inv_w2);
    return q + y * (F3 - 1) + (F3 - 1) * (GW + 1);
  };
  auto goff = [&](int tap) { return tap < K3 ? (tap / F3) * GW + tap % F3 : 0; };

  // Q A operand: W3[tap = 16 tt + lq][c(s)], k-slot (s, lg) <-> channel
  // c(s) = 16 (s >> 2) + 4 lg + (s & 3) (the channels a lane loads as two
  // 16-B quads of its pixel)
  float wq[TT][KQ];
#pragma unroll
  for (int tt = 0; tt < TT; tt++)
#pragma unroll
    for (int s = 0; s < KQ; s++) {
      const int tap = 16 * tt + lq;
      wq[tt][s] = tap < K3 ? W3[tap * N2 + 16 * (s >> 2) + 4 * lg + (s & 3)] : 0.0f;
    }
  // delta2^T k-slot (s, lg) <-> tap (dy, dx) = (s, lg) for s < F3 (a lane's
  // gathers are then one per-lane base - s GW); with F3 = 5 the fifth column
  // follows: (lg, 4) at s = 5, (4, 4) at s = 6 (lane group 0).  Slots without
  // a tap get W3 = 0.  A operand: W3[tap(s, lg)][c = 16 t + lq].
  static_assert((F3 == 5 && KT == 7) || (F3 <= 4 && KT >= F3), "delta2 tap slots");
  float wd[KT][NT];
#pragma unroll
  for (int s = 0; s < KT; s++) {
    const int tap = s < F3 ? (lg < F3 ? s * F3 + lg : -1) : (s == F3 ? lg * F3 + 4 : (lg == 0 ? 4 * F3 + 4 : -1));
#pragma unroll
    for (int t = 0; t < NT; t++) wd[s][t] = tap >= 0 ? W3[tap * N2 + 16 * t + lq] : 0.0f;
  }
  // delta2 gather offsets: slot s < F3 at base - lg - s GW, s = 5 at
  // base - lg GW - 4, s = 6 at base - 4 GW - 4
  const int od5 = lg * GW + 4;
  // gW3 A operand rows: tap 16 tt + lq (rows past K3 read a real cell and are discarded)
  int og[TT];
#pragma unroll
  for (int tt = 0; tt < TT; tt++) og[tt] = goff(16 * tt + lq);
  const float b3 = B3[0];

  f32x4 gacc[TT][NT];
#pragma unroll
  for (int tt = 0; tt < TT; tt++)
#pragma unroll
    for (int t = 0; t < NT; t++) gacc[tt][t] = mfma::zero4();
  float gb3 = 0.0f, sq = 0.0f;

  // this thread's L3 outputs tid, tid + 256 and their ground truth,
  // prefetched one sample ahead
  float tn[OPT];
  auto tload = [&](int smp) {
#pragma unroll
    for (int k = 0; k < OPT; k++) {
      const int o = tid + k * kL3sThreads;
      const int oy = o / g.w3, ox = o - oy * g.w3;
      if (o < nout) tn[k] = T[(size_t)smp * g.W * g.H + (size_t)(oy + pad) * g.W + ox + pad];
    }
  };
  // A2[p = 16u + lq][16 t + 4 lg .. +3]: Q's B operand (pass 1) and the relu'
  // mask of delta2^T's output (pass 2) of unit u
  auto a2load = [&](const float* a2s, int u, f32x4* av) {
    const int pc = min(16 * u + lq, npx2 - 1);
#pragma unroll
    for (int t = 0; t < NT; t++) av[t] = *reinterpret_cast<const f32x4*>(a2s + (size_t)pc * N2 + 16 * t + 4 * lg);
  };
  // gW3 B operands of unit u: A2[p = 16u + 4s + lg][16 t + lq] (pixels past
  // the sample read its last row: their A operands are zero cells)
  auto bload = [&](const float* a2s, int u, float (*bg)[NT]) {
#pragma unroll
    for (int s = 0; s < 4; s++) {
      const int pc = min(16 * u + 4 * s + lg, npx2 - 1);
#pragma unroll
      for (int t = 0; t < NT; t++) bg[s][t] = a2s[(size_t)pc * N2 + 16 * t + lq];
    }
  };
  const int nj = nunit > wave ? (nunit - wave + NWV - 1) / NWV : 0;  // units of this wave

  // pass 1 of one unit: Q[tap = 16 tt + 4 lg + i][p] into the Q image (rows of
  // whole units; pixels past the sample are written, never read)
  auto q_unit = [&](int u, const f32x4* av) {
    f32x4 q[TT];
#pragma unroll
    for (int tt = 0; tt < TT; tt++) q[tt] = mfma::zero4();
#pragma unroll
    for (int s = 0; s < KQ; s++)
#pragma unroll
      for (int tt = 0; tt < TT; tt++) q[tt] = mfma::mma16(wq[tt][s], av[s >> 2][s & 3], q[tt]);
    const int p = 16 * u + lq;
#pragma unroll
    for (int tt = 0; tt < TT; tt++)
#pragma unroll
      for (int i = 0; i < 4; i++) {
        const int tap = 16 * tt + 4 * lg + i;
        if (tap < K3) qs[tap * PL + p] = q[tt][i];
      }
  };
  // pass 2 of one unit: the delta3-window gathers (issued a unit ahead of
  // their MFMAs), then delta2 (masked by mk = A2 > 0) and gW3 += ...
  auto d_gather = [&](int u, float* ad, float (*ag)[TT]) {
    const int u0 = 16 * u;
    const int gp = gpos(min(u0 + lq, npx2 - 1));
#pragma unroll
    for (int s = 0; s < KT; s++) ad[s] = s < F3 ? gd[gp - lg - s * GW] : gd[gp - (s == F3 ? od5 : 4 * GW + 4)];
#pragma unroll
    for (int s = 0; s < 4; s++) {
      const int pq = u0 + 4 * s + lg;
      const int gq = pq < npx2 ? gpos(pq) : L.zp;  // past the sample: zero cells
#pragma unroll
      for (int tt = 0; tt < TT; tt++) ag[s][tt] = gd[gq - og[tt]];
    }
  };
  auto d_unit = [&](const float* ad, const float (*ag)[TT], const f32x4* mk, const float (*bg)[NT], f32x4* dv) {
    // delta2^T[c = 16 t + 4 lg + i][p]: M = channels, N = pixels, K = taps
#pragma unroll
    for (int t = 0; t < NT; t++) dv[t] = mfma::zero4();
#pragma unroll
    for (int s = 0; s < KT; s++)
#pragma unroll
      for (int t = 0; t < NT; t++) dv[t] = mfma::mma16(wd[s][t], ad[s], dv[t]);
    // gW3[tap = 16 tt + 4 lg + i][c = 16 t + lq] += delta3win . A2: K = pixels
#pragma unroll
    for (int s = 0; s < 4; s++)
#pragma unroll
      for (int tt = 0; tt < TT; tt++)
#pragma unroll
        for (int t = 0; t < NT; t++) gacc[tt][t] = mfma::mma16(ag[s][tt], bg[s][t], gacc[tt][t]);
#pragma unroll
    for (int t = 0; t < NT; t++)
#pragma unroll
      for (int i = 0; i < 4; i++) dv[t][i] = mk[t][i] > 0.0f ? dv[t][i] : 0.0f;
  };
  auto d_store = [&](int smp, int u, const f32x4* dv) {
    const int p = 16 * u + lq;
    if (p < npx2) {
      float* dst = D2 + ((size_t)((kL3sDiag & 8) ? 0 : smp) * npx2 + p) * N2 + 4 * lg;
#pragma unroll
      for (int t = 0; t < NT; t++) *reinterpret_cast<f32x4*>(dst + 16 * t) = dv[t];
    }
  };

  f32x4 bufA[NT], bufB[NT];  // pass 1: units j (A) / j + 1 (B)
  if ((int)blockIdx.x < g.batch) {
    const int smp0 = l3_order(blockIdx.x, g.batch);
    tload(smp0);
    const float* a2s0 = A2 + (size_t)smp0 * npx2 * N2;
    if (nj > 0) a2load(a2s0, wave, bufA);
    if (nj > 1) a2load(a2s0, wave + NWV, bufB);
  }
#ifdef SRCNN_L3_TIMING
  // diagnostics build: wave 0's cycles in pass 1, the pass-1 barrier, the
  // window phase + its barrier, pass 2 (g_l3_timing, tools/l3_timing.py)
  unsigned long long tacc[4] = {0, 0, 0, 0}, tlast = clock64();
#define SRCNN_L3S_TICK(PH)                         \
  do {                                             \
    if (threadIdx.x == 0) {                        \
      const unsigned long long now_ = clock64();   \
      tacc[PH] += now_ - tlast;                    \
      tlast = now_;                                \
    }                                              \
  } while (0)
#else
#define SRCNN_L3S_TICK(PH) \
  do {                     \
  } while (0)
#endif
  for (int sample = blockIdx.x; sample < g.batch; sample += gridDim.x) {
    const int smp = l3_order(sample, g.batch);
    const float* a2s = A2 + (size_t)smp * npx2 * N2;
    const float* a2p1 = (kL3sDiag & 1) ? A2 : a2s;
    const float* a2p2 = (kL3sDiag & 2) ? A2 : a2s;
    float tc[OPT];
#pragma unroll
    for (int k = 0; k < OPT; k++) tc[k] = tn[k];
    const int nxt = sample + (int)gridDim.x;
    if (nxt < g.batch) tload(l3_order(nxt, g.batch));
    // the previous sample's readers of the Q image passed the window barrier;
    // of the grid, the barrier below.  (The first sample: the grid's zero
    // cells are written before that barrier too.)

    // ---- pass 1 ----
#pragma unroll 1
    for (int j = 0; j < nj; j += 2) {
      q_unit(wave + NWV * j, bufA);
      if (j + 2 < nj) a2load(a2p1, wave + NWV * (j + 2), bufA);
      if (j + 1 < nj) {
        q_unit(wave + NWV * (j + 1), bufB);
        if (j + 3 < nj) a2load(a2p1, wave + NWV * (j + 3), bufB);
      }
    }
    SRCNN_L3S_TICK(0);
    __syncthreads();
    SRCNN_L3S_TICK(1);
    // pass-2 operands of the first two units (before the A3 stores below)
    f32x4 mA[NT], mB[NT];
    float gA[4][NT], gB[4][NT];
    if (nj > 0) {
      a2load(a2p2, wave, mA);
      bload(a2p2, wave, gA);
    }
    if (nj > 1) {
      a2load(a2p2, wave + NWV, mB);
      bload(a2p2, wave + NWV, gB);
    }

    // ---- A3, last delta, squared error, gB3; delta3 into the grid ----
#pragma unroll
    for (int k = 0; k < OPT; k++) {
      const int o = tid + k * kL3sThreads;
      if (o < nout) {
        const int oy = o / g.w3, ox = o - oy * g.w3;
        const float* q0 = qs + oy * g.w2 + ox;
        float acc = 0.0f;
#pragma unroll
        for (int dy = 0; dy < F3; dy++)
#pragma unroll
          for (int dx = 0; dx < F3; dx++) acc += q0[(dy * F3 + dx) * PL + dy * g.w2 + dx];
        const float a3 = acc + b3;
        A3out[(size_t)smp * nout + o] = a3;  // to the workspace (srcnn_train_activations)
        const float diff = a3 - tc[k];
        const float d3 = diff * (a3 > 0.0f ? 1.0f : 0.0f);
        gd[(oy + F3 - 1) * GW + ox + F3 - 1] = d3;
        gb3 += d3;
        sq += diff * diff;
      }
    }
    __syncthreads();
    SRCNN_L3S_TICK(2);

    // ---- pass 2 ----
    if (nxt < g.batch) {  // the next sample's first two pass-1 units
      const float* a2n = (kL3sDiag & 1) ? A2 : A2 + (size_t)l3_order(nxt, g.batch) * npx2 * N2;
      if (nj > 0) a2load(a2n, wave, bufA);
      if (nj > 1) a2load(a2n, wave + NWV, bufB);
    }
    float adA[KT], agA[4][TT], adB[KT], agB[4][TT];
    if (nj > 0) d_gather(wave, adA, agA);
#pragma unroll 1
    for (int j = 0; j < nj; j += 2) {
      f32x4 dv[NT];
      if (j + 1 < nj) d_gather(wave + NWV * (j + 1), adB, agB);
      d_unit(adA, agA, mA, gA, dv);
      if (j + 2 < nj) {
        a2load(a2p2, wave + NWV * (j + 2), mA);
        bload(a2p2, wave + NWV * (j + 2), gA);
      }
      d_store(smp, wave + NWV * j, dv);
      if (j + 1 < nj) {
        if (j + 2 < nj) d_gather(wave + NWV * (j + 2), adA, agA);
        d_unit(adB, agB, mB, gB, dv);
        if (j + 3 < nj) {
          a2load(a2p2, wave + NWV * (j + 3), mB);
          bload(a2p2, wave + NWV * (j + 3), gB);
        }
        d_store(smp, wave + NWV * (j + 1), dv);
      }
    }
    SRCNN_L3S_TICK(3);
  }
  SRCNN_CLOCK_END(g_clk, 1);
#ifdef SRCNN_L3_TIMING
  if (threadIdx.x == 0 && blockIdx.x < 1024)
    for (int k = 0; k < 4; k++) g_l3_timing[blockIdx.x][k] = tacc[k];
#endif
#undef SRCNN_L3S_TICK

  // ---- block reduction of the partial gradients, waves in order ----
  __syncthreads();
  float* red = smem;
  for (int w = 0; w < NWV; w++) {
    if (wave == w) {
#pragma unroll
      for (int tt = 0; tt < TT; tt++)
#pragma unroll
        for (int t = 0; t < NT; t++)
#pragma unroll
          for (int i = 0; i < 4; i++) {
            float* dst = red + ((tt * NT + t) * 4 + i) * 64 + lane;
            *dst = (w == 0 ? 0.0f : *dst) + gacc[tt][t][i];
          }
    }
    __syncthreads();
  }
  float* out = slab3 + (size_t)blockIdx.x * (NW3 + 1);
  for (int i = tid; i < TT * NT * 4 * 64; i += kL3sThreads) {
    const int k = i >> 8, r = (i >> 6) & 3, l = i & 63;
    const int tt = k / NT, t = k - tt * NT;
    const int tap = 16 * tt + 4 * (l >> 4) + r, c = 16 * t + (l & 15);
    if (tap < K3) out[tap * N2 + c] = red[i];
  }
  // gB3 and squared error: per-wave shuffle trees, then waves in order
  for (int off = 32; off > 0; off >>= 1) {
    gb3 += __shfl_down(gb3, off, 64);
    sq += __shfl_down(sq, off, 64);
  }
  __syncthreads();
  if (lane == 0) {
    red[2 * wave] = gb3;
    red[2 * wave + 1] = sq;
  }
  __syncthreads();
  if (tid == 0) {
    float tb = 0.f, ts = 0.f;
    for (int w = 0; w < NWV; w++) {
      tb += red[2 * w];
      ts += red[2 * w + 1];
    }
    out[NW3] = tb;
    sq_slab[blockIdx.x] = ts;
  }
}

template <int N2, int F3>
static size_t l3s_lds_bytes(int w2, int h2) {
  return L3sLds<N2, F3>(w2, h2).bytes();
}
