// l3_delta.hpp -- fused kernel 2 of train_fused.hip (included inside
// namespace srcnn::fused): per sample, with the A2 tile resident in LDS,
//   L3 forward       layer_uber_kernel.cl:70-91 (SKIP_RELU)
//   last delta       last_layer_delta.cl:34-48 (relu' quirk on a linear layer)
//   squared error    squared_error.cl:60-69 (validation metric)
//   delta2           layer_deltas.cl:79-123, MFMA over the f3*f3 taps
//   gW3 / gB3        backpropagate.cl:89-112, MFMA over the A2 pixels
// 8 waves per block, one block per CU, grid-strided over samples.
//
// L3 forward has one output channel, so it is not a GEMM as written.  It is
// split into a GEMM and a gather ("Q trick"):
//   Q[q][tap] = sum_c A2[q][c] * W3[tap][c]        (MFMA, M = pixels, N = taps, K = channels)
//   A3[p]     = B3 + sum_tap Q[p + off(tap)][tap]  (25 LDS reads per output)
// which moves the 5x5x32 window sums from LDS-bound VALU onto the matrix cores.
//
// LDS holds two tile-sized regions used ping-pong: region `cur` holds this
// sample's A2, the other first holds Q and, once the L3 gather has consumed
// Q, receives the NEXT sample's A2 by LDS-DMA (global_load_lds, no
// registers) while delta2 / gW3 run.  The next sample swaps the roles.
//
// A2 LDS image: rows of N2 floats, 16-byte quads XOR-swizzled by row (quad
// q of row p at q ^ ((p >> 1) & (N2/4 - 1))): the per-pixel column reads of
// the MFMA A operand and the per-channel row reads are at most 2-way bank
// conflicted without padding.  The DMA realises the swizzle by choosing each
// lane's global source quad.
// Sample order: l3 walks the batch from the end.  l12 wrote the last
// samples' A2 last, so they are the ones still in the MALL; and l3's own last
// D2 rows are then the batch head, which d1 (grid-strided from the start)
// reads first.
__device__ __forceinline__ int l3_order(int s, int batch) { return batch - 1 - s; }

struct L3Geom {
  int W, H;     // ground-truth sample (= network input size)
  int w2, h2;   // A2
  int w3, h3;   // A3
  int batch;
};

// (768 / 1024 threads per block measured slower: the three barrier-separated
// phases, not occupancy, set the pace)
constexpr int kL3Threads = 512;
constexpr int kL3TPF = (1024 + kL3Threads - 1) / kL3Threads;  // L3 outputs per thread (w3 * h3 <= 1024)
constexpr int kL3MaxOut = kL3TPF * kL3Threads;

// float index of A2[p][n] in the swizzled LDS image
template <int N2>
__device__ __forceinline__ int a2_at(int p, int n) {
  constexpr int NQ = N2 / 4;
  return p * N2 + 4 * ((n >> 2) ^ ((p >> 1) & (NQ - 1))) + (n & 3);
}

// LDS geometry shared by host and device (floats)
template <int N2, int F3>
struct L3Lds {
  // 16-pixel units per wave of the largest A2 tile whose two regions fit the
  // 160 KB LDS (npx2 * max(N2, F3^2) <= 20480 floats)
  static constexpr int kMaxPx = 20480 / (N2 > F3 * F3 ? N2 : F3 * F3);
  static constexpr int kUnitsPerWave = ((kMaxPx + 15) / 16 + kL3Threads / 64 - 1) / (kL3Threads / 64);
  int region;  // one ping-pong region: max(A2 tile, Q of whole units, reduction scratch)
  int d3off;   // delta3 grid offset (F3-1) * (w2 + 1)
  int nd3;     // delta3 grid size (zero tail covers chunk overrun)
  __host__ __device__ L3Lds(int w2, int h2) {
    const int npx2 = w2 * h2, nch = (npx2 + 31) / 32;
    int r = npx2 * N2;
    const int npad = (npx2 + 15) / 16 * 16;  // Q is written for whole 16-pixel units
    if (npad * F3 * F3 > r) r = npad * F3 * F3;
    if (((N2 + 31) / 32) * 1024 > r) r = ((N2 + 31) / 32) * 1024;
    region = (r + 3) & ~3;
    d3off = (F3 - 1) * (w2 + 1);
    nd3 = nch * 32 + d3off + 4;
  }
  __host__ __device__ size_t bytes() const { return (2 * (size_t)region + nd3) * sizeof(float); }
};

template <int N2, int F3>
__global__ __launch_bounds__(kL3Threads, 1) void l3_delta_kernel(
    const float* __restrict__ A2, const float* __restrict__ T, const float* __restrict__ W3,
    const float* __restrict__ B3, float* __restrict__ D2, float* __restrict__ slab3,
    float* __restrict__ sq_slab, float* __restrict__ A3out, L3Geom g) {
  // All three GEMMs run on v_mfma_f32_16x16x4_f32 over 16-pixel units, so the
  // ceil(npx2 / 16) units of a sample split evenly over the 8 waves (625
  // pixels: 40 units, 5 per wave; 32-pixel chunks would leave 4 waves a third
  // chunk while the other 4 idle).
  constexpr int K3 = F3 * F3;
  constexpr int TT = (K3 + 15) / 16;  // 16-wide tap tiles
  constexpr int NT = N2 / 16;         // 16-wide channel tiles
  constexpr int KT = (K3 + 3) / 4;    // delta2 k-steps (over taps)
  constexpr int KQ = N2 / 4;          // Q k-steps (over channels)
  constexpr int NW3 = K3 * N2;        // gW3 size; slab row = NW3 + 1 (gB3)
  constexpr int NQ = N2 / 4;          // quads per A2 row
  constexpr int kUMax = L3Lds<N2, F3>::kUnitsPerWave;  // unit slots per wave
  static_assert(K3 <= 32, "taps must fit two 16-wide MFMA tiles");
  static_assert(N2 % 16 == 0 && N2 <= 32 && (NQ & (NQ - 1)) == 0, "n2 must be 16 or 32");
  SRCNN_CLOCK_BEGIN();
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int npx2 = g.w2 * g.h2;
  const int nunit = (npx2 + 15) / 16;
  const L3Lds<N2, F3> L(g.w2, g.h2);
  // delta3 on the A2 grid: delta3(y, x) at d3g[(y + F3-1) * w2 + x + F3-1], zero
  // elsewhere (w3 = w2 - (F3-1), so a row's F3-1 leading columns are the zero
  // border of the previous row's wrap).  delta3(y - dy, x - dx) for A2 pixel
  // p = y*w2 + x is then d3g[p + (F3-1)*(w2+1) - (dy*w2 + dx)]: one add.
  const int d3off = L.d3off;
  float* d3g = smem + 2 * L.region;
  float* red = smem;  // end-of-kernel reduction scratch

  const int tid = threadIdx.x;
  const int lane = mfma::lane_id(), wave = mfma::wave_id();
  const int lq = lane & 15, lg = lane >> 4;  // 16x16x4 operand row / k group
  constexpr int nwaves = kL3Threads / 64;
  const int pad = (g.W - g.w3) / 2;  // last_layer_delta.cl:25
  const int nq = npx2 * NQ;          // 16-byte quads per A2 tile
  const int ndma = (nq + 63) / 64;   // DMA instructions per tile (64 quads each)

  // delta3 grid zero; the LDS past this sample's A2 image too, so operand
  // reads of the rows past the sample (last unit) always see finite values
  for (int i = tid; i < L.nd3; i += kL3Threads) d3g[i] = 0.0f;
  for (int i = npx2 * N2 + tid; i < 2 * L.region; i += kL3Threads) smem[i] = 0.0f;

  auto tap_off = [&](int tap) { return tap < K3 ? (tap / F3) * g.w2 + tap % F3 : 0; };
  // B operand of Q: W3[tap = 16t + lq][c = 4s + lg]
  float wq[KQ][TT];
  // A operand of delta2^T: W3[tap = 4s + lg][n = 16t + lq]
  float wd[KT][NT];
#pragma unroll
  for (int s = 0; s < KQ; s++)
#pragma unroll
    for (int t = 0; t < TT; t++) {
      const int tap = 16 * t + lq;
      wq[s][t] = tap < K3 ? W3[tap * N2 + 4 * s + lg] : 0.0f;
    }
#pragma unroll
  for (int s = 0; s < KT; s++)
#pragma unroll
    for (int t = 0; t < NT; t++) {
      const int tap = 4 * s + lg;
      wd[s][t] = tap < K3 ? W3[tap * N2 + 16 * t + lq] : 0.0f;
    }
  const float b3 = B3[0];
  // Per-lane LDS offsets, so that every operand read in the unit loops is
  // one base register + an immediate (units start at multiples of 16
  // pixels, so the A2 swizzle of a unit-relative pixel is unit independent):
  //  qz[s]:     Q A operand A2[u0 + lq][4s + lg]
  //  bsw[t][j]: A2[u0 + 4lg + s][16t + lq] for s >> 1 == j
  //  od[s]:     delta3 window of tap 4s + lg (delta2^T B operand, pixel u0 + lq)
  //  goff[t]:   delta3 window of tap 16t + lq (gW3 A operand; lanes past the
  //             taps read a real window: their gW3 rows are discarded)
  int qz[KQ], bsw[NT][2], od[KT], goff[TT];
#pragma unroll
  for (int s = 0; s < KQ; s++) qz[s] = lq * N2 + 4 * (s ^ ((lq >> 1) & (NQ - 1))) + lg;
#pragma unroll
  for (int t = 0; t < NT; t++)
#pragma unroll
    for (int j = 0; j < 2; j++)
      bsw[t][j] = 4 * ((4 * t + (lq >> 2)) ^ ((2 * lg + j) & (NQ - 1))) + (lq & 3);
#pragma unroll
  for (int s = 0; s < KT; s++) od[s] = d3off - tap_off(4 * s + lg);
#pragma unroll
  for (int t = 0; t < TT; t++) goff[t] = d3off - tap_off(16 * t + lq);
  //  mo[t]:     quad 4t + lg of A2 row u0 + lq (relu' mask of transposed delta2)
  int mo[NT];
#pragma unroll
  for (int t = 0; t < NT; t++) mo[t] = lq * N2 + 4 * ((4 * t + lg) ^ ((lq >> 1) & (NQ - 1)));

  f32x4 gacc[TT][NT];
#pragma unroll
  for (int t3 = 0; t3 < TT; t3++)
#pragma unroll
    for (int t = 0; t < NT; t++) gacc[t3][t] = mfma::zero4();
  float gb3 = 0.0f, sq = 0.0f;

  // A2 tile of SAMPLE -> region DST by LDS-DMA: instruction k writes image
  // quads [64k, 64k + 64); lane j fetches the global quad that the swizzle
  // places at image quad 64k + j.
#define SRCNN_L3_A2_DMA(SAMPLE, DST)                                                     \
  do {                                                                                   \
    const float* src_ = A2 + (size_t)(SAMPLE)*npx2 * N2;                                 \
    int l_ = lane; /* opaque: addresses are formed at the load, never held */            \
    asm volatile("" : "+v"(l_));                                                         \
    for (int k_ = wave; k_ < ndma; k_ += nwaves) {                                       \
      const int f_ = 64 * k_ + l_;                                                       \
      if (f_ < nq) {                                                                     \
        const int p_ = f_ / NQ, j_ = f_ - p_ * NQ;                                       \
        const int q_ = j_ ^ ((p_ >> 1) & (NQ - 1));                                      \
        __builtin_amdgcn_global_load_lds(                                                \
            (const void*)(src_ + p_ * N2 + 4 * q_),                                      \
            (__attribute__((address_space(3))) void*)((DST) + 256 * k_), 16, 0,          \
            (kNtMask & 1) ? 2 : 0);                                                      \
      }                                                                                  \
    }                                                                                    \
  } while (0)

  // ground truth of this thread's L3 outputs, prefetched one sample ahead
  const int nout = g.w3 * g.h3;
  float tpf[kL3TPF];
#define SRCNN_L3_T_PREFETCH(SAMPLE)                                                    \
  do {                                                                                 \
    _Pragma("unroll") for (int k = 0; k < kL3TPF; k++) {                               \
      const int t_ = tid + k * kL3Threads;                                             \
      const int y_ = t_ / g.w3, x_ = t_ - (t_ / g.w3) * g.w3;                          \
      tpf[k] = t_ < nout ? T[(size_t)(SAMPLE)*g.W * g.H + (size_t)(y_ + pad) * g.W + x_ + pad] : 0.f; \
    }                                                                                  \
  } while (0)

  // masked delta2 of this wave's units (slot j = unit wave + 8j), held
  // until the next sample's Q phase; D2 rows past the sample are not stored
  f32x4 d2k[kUMax][NT];
  float* d2dst = D2;
  bool d2pend = false;
#define SRCNN_L3_D2_STORE(J)                                                           \
  do {                                                                                 \
    const int q_ = 16 * (wave + nwaves * (J)) + lq;                                    \
    if (d2pend && q_ < npx2) {                                      \
      float* dst_ = d2dst + (size_t)q_ * N2 + 4 * lg;                                  \
      _Pragma("unroll") for (int t = 0; t < NT; t++)                                   \
        if (kNtMask & 2)                                                               \
          __builtin_nontemporal_store(d2k[J][t], reinterpret_cast<f32x4*>(dst_ + 16 * t)); \
        else                                                                           \
          *reinterpret_cast<f32x4*>(dst_ + 16 * t) = d2k[J][t];                        \
    }                                                                                  \
  } while (0)

  int cur = 0;
  if ((int)blockIdx.x < g.batch) {
    SRCNN_L3_A2_DMA(l3_order(blockIdx.x, g.batch), smem);
    SRCNN_L3_T_PREFETCH(l3_order(blockIdx.x, g.batch));
  }

  for (int sample = blockIdx.x; sample < g.batch; sample += gridDim.x) {
    // this sample's A2 DMA has landed in every wave; the previous sample's
    // readers of both regions and of d3g are done
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const float* a2s = smem + cur * L.region;
    float* other = smem + (cur ^ 1) * L.region;
    float* qs = other;  // [npx2][K3]
    float tcur[kL3TPF];
#pragma unroll
    for (int k = 0; k < kL3TPF; k++) tcur[k] = tpf[k];
    const bool has_next = sample + (int)gridDim.x < g.batch;
    if (has_next) SRCNN_L3_T_PREFETCH(l3_order(sample + gridDim.x, g.batch));

    // ---- Q = A2 . W3^T per 16-pixel unit (rows past npx2 are discarded);
    // the PREVIOUS sample's masked delta2 leaves to HBM under these MFMAs ----
#pragma unroll
    for (int j = 0; j < kUMax; j++) {
      const int u = wave + nwaves * j;
      if (u < nunit) {
        const int u0 = 16 * u;
        const float* a2u = a2s + u0 * N2;
        float av[KQ];
#pragma unroll
        for (int s = 0; s < KQ; s++) av[s] = a2u[qz[s]];
        __builtin_amdgcn_sched_barrier(0);  // all operand reads in flight before the MFMAs
        f32x4 acc[TT];
#pragma unroll
        for (int t = 0; t < TT; t++) acc[t] = mfma::zero4();
#pragma unroll
        for (int s = 0; s < KQ; s++)
#pragma unroll
          for (int t = 0; t < TT; t++) acc[t] = mfma::mma16(av[s], wq[s][t], acc[t]);
        SRCNN_L3_D2_STORE(j);
        // Q[u0 + 4lg + i][tap = 16t + lq] (the region holds whole units: rows
        // past the sample are written too, never read)
#pragma unroll
        for (int t = 0; t < TT; t++) {
          const int tap = 16 * t + lq;
          if (tap < K3) {
            float* qd = qs + (u0 + 4 * lg) * K3 + tap;
#pragma unroll
            for (int i = 0; i < 4; i++) qd[i * K3] = acc[t][i];
          }
        }
      }
    }
    d2pend = false;
    __syncthreads();

    // ---- L3 = B3 + diagonal sums of Q; last delta; squared error ----
#pragma unroll
    for (int k = 0; k < kL3TPF; k++) {
      const int t = tid + k * kL3Threads;
      if (t < nout) {
        const int y = t / g.w3, x = t - y * g.w3;
        const float* qrow = qs + (y * g.w2 + x) * K3;
        float acc = 0.0f;
#pragma unroll
        for (int dy = 0; dy < F3; dy++)
#pragma unroll
          for (int dx = 0; dx < F3; dx++) acc += qrow[(dy * g.w2 + dx) * K3 + dy * F3 + dx];
        const float a3 = acc + b3;
        // A3 to the workspace (srcnn_train_activations; 1% of l3's bytes)
        A3out[(size_t)l3_order(sample, g.batch) * nout + t] = a3;
        const float diff = a3 - tcur[k];
        const float d3 = diff * (a3 > 0.0f ? 1.0f : 0.0f);
        d3g[y * g.w2 + x + d3off] = d3;
        gb3 += d3;
        sq += diff * diff;
      }
    }
    __syncthreads();

    // Q is consumed: the next sample's A2 streams into its region meanwhile
    // (Measured slower: loading the next A2 into registers under the Q MFMAs
    // and writing it here, so its HBM reads leave the delta2 phase.)
    if (has_next) SRCNN_L3_A2_DMA(l3_order(sample + gridDim.x, g.batch), other);

    // ---- per 16-pixel unit: delta2 and gW3 MFMAs ----
    //   delta2[q][n] = [A2 > 0] * sum_tap delta3(q - off(tap)) W3[tap][n]
    //   gW3[tap][n] += sum_p delta3(p - off(tap)) A2[p][n]
    // delta2 runs TRANSPOSED (M = channels, N = pixels): C register i of lane
    // (lq, lg) in tile t is delta2[u0 + lq][16t + 4lg + i], four consecutive
    // channels of one pixel, so a unit leaves as NT 16-B stores per lane; its
    // relu' mask is one 16-B read of the same quad of the A2 image.
    //
    // The masked delta2 stays in registers (d2k) and is stored under the NEXT
    // sample's Q MFMAs: this phase already streams the next A2 tile in by DMA,
    // and with the stores here too it ran at the per-CU HBM rate (ablation:
    // the stores were half of the phase) while the Q phase moved no bytes.
#pragma unroll
    for (int j = 0; j < kUMax; j++) {
      const int u = wave + nwaves * j;
      if (u < nunit) {
        const int u0 = 16 * u;
        float ad[KT], ag[4][TT], bg[4][NT];
        f32x4 mk[NT];
        const float* dcu = d3g + u0 + lq;
#pragma unroll
        for (int s = 0; s < KT; s++) ad[s] = dcu[od[s]];
        const float* gcu = d3g + u0 + 4 * lg;
        const float* a2u = a2s + (u0 + 4 * lg) * N2;
#pragma unroll
        for (int s = 0; s < 4; s++) {
#pragma unroll
          for (int t3 = 0; t3 < TT; t3++) ag[s][t3] = gcu[goff[t3] + s];
#pragma unroll
          for (int t = 0; t < NT; t++) bg[s][t] = a2u[bsw[t][s >> 1] + s * N2];
        }
#pragma unroll
        for (int t = 0; t < NT; t++) mk[t] = *reinterpret_cast<const f32x4*>(a2s + u0 * N2 + mo[t]);
        __builtin_amdgcn_sched_barrier(0);  // all operand reads in flight before the MFMAs
        f32x4 acc[NT];
#pragma unroll
        for (int t = 0; t < NT; t++) acc[t] = mfma::zero4();
#pragma unroll
        for (int s = 0; s < KT; s++)
#pragma unroll
          for (int t = 0; t < NT; t++)
            acc[t] = mfma::mma16(wd[s][t], ad[s], acc[t]);
#pragma unroll
        for (int s = 0; s < 4; s++)
#pragma unroll
          for (int t3 = 0; t3 < TT; t3++)
#pragma unroll
            for (int t = 0; t < NT; t++)
              gacc[t3][t] = mfma::mma16(ag[s][t3], bg[s][t], gacc[t3][t]);
        // held for the next sample's Q phase (stored from the delta2 phase,
        // or only some units deferred: slower)
#pragma unroll
        for (int t = 0; t < NT; t++)
#pragma unroll
          for (int i = 0; i < 4; i++) d2k[j][t][i] = mk[t][i] > 0.0f ? acc[t][i] : 0.0f;
      }
    }
    d2dst = D2 + (size_t)l3_order(sample, g.batch) * npx2 * N2;
    d2pend = true;
    cur ^= 1;
  }
#pragma unroll
  for (int j = 0; j < kUMax; j++) SRCNN_L3_D2_STORE(j);
#undef SRCNN_L3_D2_STORE
#undef SRCNN_L3_A2_DMA
  SRCNN_CLOCK_END(g_clk, 1);
#undef SRCNN_L3_T_PREFETCH

  // ---- block reduction of the partial gradients, waves in order ----
  __syncthreads();
  for (int w = 0; w < nwaves; w++) {
    if (wave == w) {
#pragma unroll
      for (int t3 = 0; t3 < TT; t3++)
#pragma unroll
        for (int t = 0; t < NT; t++)
#pragma unroll
          for (int i = 0; i < 4; i++) {
            float* dst = red + ((t3 * NT + t) * 4 + i) * 64 + lane;
            *dst = (w == 0 ? 0.0f : *dst) + gacc[t3][t][i];
          }
    }
    __syncthreads();
  }
  float* out = slab3 + (size_t)blockIdx.x * (NW3 + 1);
  for (int i = tid; i < TT * NT * 4 * 64; i += kL3Threads) {
    const int k = i >> 8, r = (i >> 6) & 3, l = i & 63;
    const int t3 = k / NT, t = k - t3 * NT;
    const int tap = 16 * t3 + 4 * (l >> 4) + r, n = 16 * t + (l & 15);
    if (tap < K3) out[tap * N2 + n] = red[i];
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
    for (int w = 0; w < nwaves; w++) {
      tb += red[2 * w];
      ts += red[2 * w + 1];
    }
    out[NW3] = tb;
    sq_slab[blockIdx.x] = ts;
  }
}

template <int N2, int F3>
static size_t l3_lds_bytes(int w2, int h2) {
  return L3Lds<N2, F3>(w2, h2).bytes();
}
