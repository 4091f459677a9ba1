// l3_delta.hpp -- fused kernel 2 of train_fused.hip (included inside
// namespace srcnn::fused): per sample, with the A2 tile resident in LDS,
//   L3 forward       layer_uber_kernel.cl:70-91 (SKIP_RELU), VALU
//   last delta       last_layer_delta.cl:34-48 (relu' quirk on a linear layer)
//   squared error    squared_error.cl:60-69 (validation metric)
//   delta2           layer_deltas.cl:79-123, MFMA over the f3*f3 taps
//   gW3 / gB3        backpropagate.cl:89-112, MFMA over the A2 pixels
// 8 waves per block, one block per CU; the next sample's A2 tile is
// prefetched into registers while the current one is processed.
//
// L3 mapping: 8 lanes per output segment, lane c4 owns channels 4c4..4c4+3
// of a 1x4 run of outputs; the 8 channel-group partials are combined with
// lane shuffles.  W3 lives in LDS (read as float4).
struct L3Geom {
  int W, H;     // ground-truth sample (= network input size)
  int w2, h2;   // A2
  int w3, h3;   // A3
  int batch;
  int ablate;   // diagnostics only (env SRCNN_ABLATE_L3): bit0 L3, bit1 delta2, bit2 gW3
};

constexpr int kL3Threads = 512;
constexpr int kL3Seg = 4;  // outputs per L3 work item (one row segment)

template <int N2, int F3>
__host__ __device__ constexpr int l3_prefetch_regs(int npx2) {
  return (npx2 * (N2 / 4) + kL3Threads - 1) / kL3Threads;
}

template <int N2, int F3, int PF>
__global__ __launch_bounds__(kL3Threads, 1) void l3_delta_kernel(
    const float* __restrict__ A2, const float* __restrict__ T, const float* __restrict__ W3,
    const float* __restrict__ B3, float* __restrict__ D2, float* __restrict__ slab3,
    float* __restrict__ sq_slab, L3Geom g) {
  constexpr int K3 = F3 * F3, KS3 = (K3 + 1) / 2, NT2 = (N2 + 31) / 32;
  constexpr int N2S = N2 + 4;       // padded A2 row
  constexpr int NW3 = K3 * N2;      // gW3 size; slab row = NW3 + 1 (gB3)
  constexpr int C4 = N2 / 4;        // channel quads (lanes per L3 work item)
  static_assert(K3 <= 32, "taps must fit one 32-row MFMA tile");
  static_assert(N2 % 4 == 0 && 64 % C4 == 0, "n2 must be a multiple of 4 dividing 256");
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int npx2 = g.w2 * g.h2;
  const int w3p = g.w3 + 2 * (F3 - 1), h3p = g.h3 + 2 * (F3 - 1);
  float* a2s = smem;                                        // [npx2 + 8][N2S]
  float* w3s = smem + (((npx2 + 8) * N2S + 3) & ~3);        // [K3][N2]
  float* d3p = w3s + ((NW3 + 3) & ~3);                      // [h3p][w3p], zero border
  float* red = d3p + ((w3p * h3p + 3) & ~3);                // [NT2*1024] reduction scratch

  const int tid = threadIdx.x;
  const int lane = mfma::lane_id(), wave = mfma::wave_id();
  const int h = lane >> 5, li = lane & 31;
  const int nwaves = kL3Threads / 64;
  const int pad = (g.W - g.w3) / 2;  // last_layer_delta.cl:25

  for (int i = tid; i < w3p * h3p; i += kL3Threads) d3p[i] = 0.0f;
  for (int i = tid; i < NW3; i += kL3Threads) w3s[i] = W3[i];
  for (int i = tid; i < 8 * N2S; i += kL3Threads) a2s[npx2 * N2S + i] = 0.0f;  // overrun rows

  // gW3 A-operand row of this lane: tap li
  const int my_dy = li / F3, my_dx = li - (li / F3) * F3;
  const bool my_tap = li < K3;
  const float b3 = B3[0];

  f32x16 gacc[NT2];
#pragma unroll
  for (int u = 0; u < NT2; u++) gacc[u] = zero16();
  float gb3 = 0.0f, sq = 0.0f;

  // register prefetch of one A2 tile: PF float4 per thread
  float4 pf[PF];
  const int nq = npx2 * C4;
#define SRCNN_L3_PREFETCH(SAMPLE)                                                        \
  do {                                                                                   \
    const float4* src_ = reinterpret_cast<const float4*>(A2 + (size_t)(SAMPLE)*npx2 * N2); \
    _Pragma("unroll") for (int k = 0; k < PF; k++) {                                     \
      const int i_ = tid + k * kL3Threads;                                               \
      pf[k] = i_ < nq ? src_[i_] : make_float4(0.f, 0.f, 0.f, 0.f);                      \
    }                                                                                    \
  } while (0)
  if ((int)blockIdx.x < g.batch) SRCNN_L3_PREFETCH(blockIdx.x);

  const int nseg = (g.w3 + kL3Seg - 1) / kL3Seg;
  const int nitems = g.h3 * nseg;
  const int c4 = tid % C4, item0 = tid / C4;
  const int items_per_pass = kL3Threads / C4;

  for (int sample = blockIdx.x; sample < g.batch; sample += gridDim.x) {
    __syncthreads();  // previous sample fully consumed a2s / d3p
#pragma unroll
    for (int k = 0; k < PF; k++) {
      const int i = tid + k * kL3Threads;
      if (i < nq) {
        const int p = i / C4, q = i - p * C4;
        *reinterpret_cast<float4*>(a2s + p * N2S + 4 * q) = pf[k];
      }
    }
    if (sample + (int)gridDim.x < g.batch) SRCNN_L3_PREFETCH(sample + gridDim.x);
    __syncthreads();

    // ---- L3 forward + last delta + squared error ----
    for (int it = item0; (g.ablate & 1) == 0 && it < nitems; it += items_per_pass) {
      const int y = it / nseg, x0 = (it - y * nseg) * kL3Seg;
      float acc[kL3Seg];
#pragma unroll
      for (int j = 0; j < kL3Seg; j++) acc[j] = 0.0f;
#pragma unroll 1
      for (int dy = 0; dy < F3; dy++) {
        float4 v[kL3Seg + F3 - 1];
        const float* row = a2s + ((y + dy) * g.w2 + x0) * N2S + 4 * c4;
#pragma unroll
        for (int j = 0; j < kL3Seg + F3 - 1; j++) v[j] = *reinterpret_cast<const float4*>(row + j * N2S);
#pragma unroll
        for (int dx = 0; dx < F3; dx++) {
          const float4 w = *reinterpret_cast<const float4*>(w3s + (dy * F3 + dx) * N2 + 4 * c4);
#pragma unroll
          for (int j = 0; j < kL3Seg; j++) {
            const float4 a = v[j + dx];
            acc[j] += a.x * w.x + a.y * w.y + a.z * w.z + a.w * w.w;
          }
        }
      }
      // combine the C4 channel-group partials (lanes c4 = 0..C4-1 are adjacent)
#pragma unroll
      for (int off = 1; off < C4; off <<= 1)
#pragma unroll
        for (int j = 0; j < kL3Seg; j++) acc[j] += __shfl_xor(acc[j], off, 64);
      if (c4 < kL3Seg) {
        float mine = acc[0];
#pragma unroll
        for (int j = 1; j < kL3Seg; j++) mine = c4 == j ? acc[j] : mine;
        const int x = x0 + c4;
        if (x < g.w3) {
          const float a3 = mine + b3;
          const float t = T[(size_t)sample * g.W * g.H + (size_t)(y + pad) * g.W + x + pad];
          const float diff = a3 - t;
          const float d3 = diff * (a3 > 0.0f ? 1.0f : 0.0f);
          d3p[(y + F3 - 1) * w3p + x + F3 - 1] = d3;
          gb3 += d3;
          sq += diff * diff;
        }
      }
    }
    __syncthreads();

    // ---- delta2: per 32-pixel chunk of the A2 grid ----
    const int nch = (npx2 + 31) / 32;
    for (int c = wave; (g.ablate & 2) == 0 && c < nch; c += nwaves) {
      const int p = min(c * 32 + li, npx2 - 1);
      const int y = p / g.w2, x = p - y * g.w2;
      const int base = (y + F3 - 1) * w3p + x + F3 - 1;
      f32x16 acc[NT2];
#pragma unroll
      for (int u = 0; u < NT2; u++) acc[u] = zero16();
#pragma unroll
      for (int s = 0; s < KS3; s++) {
        const int k0 = 2 * s, k1 = 2 * s + 1;
        const int o0 = (k0 / F3) * w3p + (k0 % F3);
        const int o1 = k1 < K3 ? (k1 / F3) * w3p + (k1 % F3) : 0;
        const float a = d3p[base - (h ? o1 : o0)];
        const int tap = h ? k1 : k0;
#pragma unroll
        for (int u = 0; u < NT2; u++) {
          // B operand W3[tap][n = 32u + li] (zero past the taps / channels)
          const int n = 32 * u + li;
          const float b = (tap < K3 && n < N2) ? w3s[tap * N2 + n] : 0.0f;
          acc[u] = mma(a, b, acc[u]);
        }
      }
#pragma unroll
      for (int r = 0; r < 16; r++) {
        const int pr = c * 32 + crow(r, h);
        if (pr < npx2) {
#pragma unroll
          for (int u = 0; u < NT2; u++) {
            const int n = 32 * u + li;
            if (n < N2) {
              const float m = a2s[pr * N2S + n] > 0.0f ? 1.0f : 0.0f;
              D2[((size_t)sample * npx2 + pr) * N2 + n] = acc[u][r] * m;
            }
          }
        }
      }
    }

    // ---- gW3: G[tap][n] += sum_p' d3p[p' - tap] * A2[p'][n] ----
    {
      const int nks = (g.ablate & 4) ? 0 : (npx2 + 1) / 2;
      int pp = 2 * wave + h;
      int yq = pp / g.w2, xq = pp - yq * g.w2;
      const int stride = 2 * nwaves;
      for (int j = wave; j < nks; j += nwaves) {
        const bool v = pp < npx2;
        const float a =
            (v && my_tap) ? d3p[(yq - my_dy + F3 - 1) * w3p + xq - my_dx + F3 - 1] : 0.0f;
#pragma unroll
        for (int u = 0; u < NT2; u++) {
          const int n = 32 * u + li;
          const float b = (v && n < N2) ? a2s[pp * N2S + n] : 0.0f;
          gacc[u] = mma(a, b, gacc[u]);
        }
        pp += stride;
        xq += stride;
        while (xq >= g.w2) {
          xq -= g.w2;
          yq++;
        }
      }
    }
  }

  // ---- block reduction of the partial gradients, waves in order ----
  __syncthreads();
  for (int w = 0; w < nwaves; w++) {
    if (wave == w) {
#pragma unroll
      for (int u = 0; u < NT2; u++)
#pragma unroll
        for (int r = 0; r < 16; r++) {
          float* dst = red + (u * 16 + r) * 64 + lane;
          *dst = (w == 0 ? 0.0f : *dst) + gacc[u][r];
        }
    }
    __syncthreads();
  }
  float* out = slab3 + (size_t)blockIdx.x * (NW3 + 1);
  for (int i = tid; i < NT2 * 16 * 64; i += kL3Threads) {
    const int u = i / 1024, r = (i >> 6) & 15, l = i & 63;
    const int tap = crow(r, l >> 5), n = 32 * u + (l & 31);
    if (tap < K3 && n < N2) out[tap * N2 + n] = red[i];
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
static size_t l3_lds_bytes(int npx2, int w3, int h3) {
  const int w3p = w3 + 2 * (F3 - 1), h3p = h3 + 2 * (F3 - 1);
  const size_t a2 = ((size_t)(npx2 + 8) * (N2 + 4) + 3) & ~size_t(3);
  const size_t w3s = ((size_t)F3 * F3 * N2 + 3) & ~size_t(3);
  const size_t d3 = ((size_t)w3p * h3p + 3) & ~size_t(3);
  const size_t red = (size_t)((N2 + 31) / 32) * 1024;
  return (a2 + w3s + d3 + red) * sizeof(float);
}
