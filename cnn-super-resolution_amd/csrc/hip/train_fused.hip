// train_fused.hip -- gfx950 fused training step for SRCNN nets with a 1x1
// middle layer (f2 == 1), e.g. the reference default n1=64, n2=32, f1=9, f3=5.
//
// The reference runs one OpenCL kernel per op (ConfigBasedDataPipeline.cpp:
// 200-323): 3 forward, last delta, 2 deltas, 3 gradient kernels, every tensor
// round-tripping through global memory and the gradients summed serially per
// weight (backpropagate.cl:89-106).  Here the same mathematics runs as three
// kernels plus a deterministic reduction:
//
//   l12_fwd      L1 (f1 x f1 x 1 -> n1) and L2 (1x1, n1 -> n2) as fp32 MFMA
//                implicit GEMMs per 32-pixel chunk; A1 goes to HBM (needed by
//                backward) and through a per-wave LDS transpose into L2.
//   l3_delta     per sample: A2 tile in LDS; L3 (f3 x f3 x n2 -> 1, MFMA Q trick),
//                last-layer delta with the reference quirk, delta2 (MFMA over
//                the 25 taps), gW3 (MFMA over pixels), gB3, squared error.
//   d1_grad12    delta1 = relu'(A1) * (delta2 . W2^T) (MFMA), then gW2 and gW1
//                consume delta1 / A1 straight from the accumulator registers
//                (mfma.hpp: k-slot <-> pixel pairing), gB1 via a ones row.
//   slab_reduce  per-block partial gradients summed in block order -> grads.
//
// HBM traffic per 33x33 tile: X 4.4 KB + A1 160 KB (write + read) + A2 80 KB
// (write + read) + delta2 80 KB (write + read) ~ 650 KB vs 1.54 MB for the
// layer-by-layer dataflow.  Results are deterministic: the
// sample -> block -> wave assignment is static and every sum has a fixed
// order; no float atomics anywhere.
#include "common.hpp"
#include "mfma.hpp"
#include "ops.hpp"

namespace srcnn {
namespace fused {

using mfma::crow;
using mfma::f32x16;
using mfma::mma;
using mfma::zero16;

constexpr int kXsMax = 1536;  // input sample / region tile (floats) staged in LDS (<= 39x39)

struct Geom {
  int W, H;      // input sample
  int ow, oh;    // L1 (and L2) output
  int rw, rh;    // region of L1 output handled per work item
  int nrx, nry;  // regions per sample
  int batch;
};

// ---------------------------------------------------------------------------
// Kernel 1: L1 (+ L2) forward
// ---------------------------------------------------------------------------
template <int N1, int N2, int F1, bool STORE_A1, bool DO_L2>
__global__ __launch_bounds__(256, 2) void l12_fwd_kernel(
    const float* __restrict__ X, const float* __restrict__ W1, const float* __restrict__ B1,
    const float* __restrict__ W2, const float* __restrict__ B2, float* __restrict__ A1,
    float* __restrict__ A2, Geom g) {
  constexpr int K1 = F1 * F1, KS1 = (K1 + 1) / 2, NT1 = N1 / 32;
  constexpr int NT2 = (N2 + 31) / 32, KS2 = N1 / 2;
  constexpr int TS = N1 + 1;  // padded row of the per-wave A1 transpose
  __shared__ float xs[kXsMax];
  __shared__ float ts[DO_L2 ? 4 : 1][32][DO_L2 ? TS : 1];
  __shared__ int gidx[4][32];

  const int lane = mfma::lane_id(), wave = mfma::wave_id();
  const int h = lane >> 5, li = lane & 31;
  const int tw = g.rw + F1 - 1;  // LDS row stride of the input tile

  // B operands of L1: W1[tap = 2s + h][n = 32t + li]
  float w1f[KS1][NT1];
#pragma unroll
  for (int s = 0; s < KS1; s++)
#pragma unroll
    for (int t = 0; t < NT1; t++) {
      const int tap = 2 * s + h;
      w1f[s][t] = tap < K1 ? W1[tap * N1 + 32 * t + li] : 0.0f;
    }
  float b1v[NT1];
#pragma unroll
  for (int t = 0; t < NT1; t++) b1v[t] = B1[32 * t + li];
  // B operands of L2: W2[c = 2s + h][n = 32u + li]
  float w2f[DO_L2 ? KS2 : 1][NT2];
  float b2v[NT2];
  if constexpr (DO_L2) {
#pragma unroll
    for (int s = 0; s < KS2; s++)
#pragma unroll
      for (int u = 0; u < NT2; u++) {
        const int n = 32 * u + li;
        w2f[s][u] = n < N2 ? W2[(2 * s + h) * N2 + n] : 0.0f;
      }
#pragma unroll
    for (int u = 0; u < NT2; u++) b2v[u] = (32 * u + li) < N2 ? B2[32 * u + li] : 0.0f;
  }

  const int per_sample = g.nry * g.nrx;
  const int n_items = g.batch * per_sample;
  for (int wi = blockIdx.x; wi < n_items; wi += gridDim.x) {
    const int sample = wi / per_sample;
    const int rr = wi - sample * per_sample;
    const int ry = rr / g.nrx, rx = rr - ry * g.nrx;
    const int oy0 = ry * g.rh, ox0 = rx * g.rw;
    const int crh = min(g.rh, g.oh - oy0), crw = min(g.rw, g.ow - ox0);
    const int th = crh + F1 - 1, tww = crw + F1 - 1;

    __syncthreads();  // previous work item's readers are done with xs
    const float* xsrc = X + (size_t)sample * g.W * g.H + (size_t)oy0 * g.W + ox0;
    for (int i = threadIdx.x; i < th * tww; i += blockDim.x) {
      const int iy = i / tww, ix = i - iy * tww;
      xs[iy * tw + ix] = xsrc[(size_t)iy * g.W + ix];
    }
    __syncthreads();

    const int npx = crh * crw;
    const int nch = (npx + 31) / 32;
    for (int c = wave; c < nch; c += 4) {
      // this lane's own pixel (A-operand row li)
      const int p = c * 32 + li;
      const bool valid = p < npx;
      const int pc = valid ? p : npx - 1;
      const int iy = pc / crw, ix = pc - iy * crw;
      const int xb = iy * tw + ix;
      if (h == 0)
        gidx[wave][li] = valid ? (sample * g.oh + oy0 + iy) * g.ow + ox0 + ix : -1;

      f32x16 acc1[NT1];
#pragma unroll
      for (int t = 0; t < NT1; t++) acc1[t] = zero16();
#pragma unroll
      for (int s = 0; s < KS1; s++) {
        constexpr int dummy = 0;
        (void)dummy;
        const int k0 = 2 * s, k1 = 2 * s + 1;
        const int o0 = (k0 / F1) * tw + (k0 % F1);
        const int o1 = k1 < K1 ? (k1 / F1) * tw + (k1 % F1) : 0;
        const float a = xs[xb + (h ? o1 : o0)];
#pragma unroll
        for (int t = 0; t < NT1; t++) acc1[t] = mma(a, w1f[s][t], acc1[t]);
      }

      // epilogue L1: bias + ReLU (layer_uber_kernel.cl:88-95), store A1 (HWC)
#pragma unroll
      for (int r = 0; r < 16; r++) {
        const int gp = gidx[wave][crow(r, h)];
#pragma unroll
        for (int t = 0; t < NT1; t++) {
          const float v = fmaxf(acc1[t][r] + b1v[t], 0.0f);
          if constexpr (STORE_A1) {
            if (gp >= 0) A1[(size_t)gp * N1 + 32 * t + li] = v;
          }
          if constexpr (DO_L2) ts[wave][crow(r, h)][32 * t + li] = v;
        }
      }
      if constexpr (DO_L2) {
        __builtin_amdgcn_wave_barrier();
        f32x16 acc2[NT2];
#pragma unroll
        for (int u = 0; u < NT2; u++) acc2[u] = zero16();
#pragma unroll
        for (int s = 0; s < KS2; s++) {
          const float a = ts[wave][li][2 * s + h];  // A1[pixel li][channel 2s+h]
#pragma unroll
          for (int u = 0; u < NT2; u++) acc2[u] = mma(a, w2f[s][u], acc2[u]);
        }
#pragma unroll
        for (int r = 0; r < 16; r++) {
          const int gp = gidx[wave][crow(r, h)];
#pragma unroll
          for (int u = 0; u < NT2; u++) {
            const int n = 32 * u + li;
            if (gp >= 0 && n < N2) A2[(size_t)gp * N2 + n] = fmaxf(acc2[u][r] + b2v[u], 0.0f);
          }
        }
      }
      __builtin_amdgcn_wave_barrier();
    }
  }
}


#include "l3_delta.hpp"

// ---------------------------------------------------------------------------
// Kernel 3: delta1 + gW2/gB2 + gW1/gB1
// ---------------------------------------------------------------------------
template <int N1, int N2, int F1>
__global__ __launch_bounds__(256, 2) void d1_grad12_kernel(
    const float* __restrict__ X, const float* __restrict__ A1, const float* __restrict__ D2,
    const float* __restrict__ W2, float* __restrict__ slab, Geom g) {
  constexpr int K1 = F1 * F1, NT1 = N1 / 32, NT2 = (N2 + 31) / 32;
  constexpr int MT = (K1 + 1 + 31) / 32;  // tap tiles (+1 ones row -> gB1)
  constexpr int KD = (N2 + 1) / 2;        // delta1 k-steps (over n)
  constexpr int DS = N2 + 1;              // padded delta2 row in LDS
  constexpr int WS = N2 + 1;              // padded W2 row in LDS
  constexpr int NW1 = K1 * N1, NW2 = N1 * N2;
  constexpr int P12 = NW1 + N1 + NW2 + N2;  // [gW1 | gB1 | gW2 | gB2]
  constexpr int RED = (MT * NT1 + NT1 * NT2) * 16 * 64;
  static_assert(N2 % 2 == 0, "n2 must be even");
  constexpr int A1S = 4 * 32 * N1;        // per-wave A1 chunk staging (LDS-DMA target)
  constexpr int LDS_MAIN = A1S + kXsMax + N1 * WS + 4 * 32 * DS;
  constexpr int LDS_TOTAL = LDS_MAIN > RED ? LDS_MAIN : RED;
  __shared__ __attribute__((aligned(16))) float smem[LDS_TOTAL];
  __shared__ int xbt[4][32];
  float* a1s = smem;                   // [4][32][N1], lane-linear DMA image of A1 rows
  float* xs = smem + A1S;
  float* w2s = xs + kXsMax;            // [N1][WS]: W2[c][n]
  float* d2w = w2s + N1 * WS;          // [4][32][DS]

  const int lane = mfma::lane_id(), wave = mfma::wave_id();
  const int h = lane >> 5, li = lane & 31;
  const int npx = g.ow * g.oh;

  for (int i = threadIdx.x; i < N1 * N2; i += blockDim.x) {
    const int c = i / N2, n = i - c * N2;
    w2s[c * WS + n] = W2[i];
  }
  // gW1 A-operand rows of this lane: taps 32m + li (tap K1 = ones -> gB1)
  int toff[MT];
  float tsel_x[MT], tsel_1[MT];  // a = X * tsel_x + tsel_1: X tap / zero row / ones row
#pragma unroll
  for (int m = 0; m < MT; m++) {
    const int tap = 32 * m + li;
    toff[m] = tap < K1 ? (tap / F1) * g.W + (tap % F1) : 0;
    tsel_x[m] = tap < K1 ? 1.0f : 0.0f;
    tsel_1[m] = tap == K1 ? 1.0f : 0.0f;
  }

  f32x16 g1[MT][NT1], g2[NT1][NT2];
#pragma unroll
  for (int m = 0; m < MT; m++)
#pragma unroll
    for (int t = 0; t < NT1; t++) g1[m][t] = zero16();
#pragma unroll
  for (int t = 0; t < NT1; t++)
#pragma unroll
    for (int u = 0; u < NT2; u++) g2[t][u] = zero16();
  float gb2[NT2];
#pragma unroll
  for (int u = 0; u < NT2; u++) gb2[u] = 0.0f;

  float* d2me = d2w + wave * 32 * DS;
  // A1 rows of one chunk -> this wave's LDS image by LDS-DMA (no registers):
  // instruction k moves floats [256k, 256k + 256) of the [32][N1] chunk; rows
  // past the sample re-read its last row (finite, and their delta2 rows are 0)
  float* a1me = a1s + wave * 32 * N1;
#define SRCNN_D1_A1_DMA(SMP, C)                                                   \
  do {                                                                            \
    int lo_ = 4 * lane; /* opaque: keeps the addresses out of the loop preheader */ \
    asm volatile("" : "+v"(lo_));                                                 \
    const float* base_ = A1 + (size_t)(SMP) * npx * N1;                           \
    _Pragma("unroll") for (int k = 0; k < 32 * N1 / 256; k++) {                   \
      const int f_ = k * 256 + lo_;                                               \
      const int row_ = min((C) * 32 + f_ / N1, npx - 1);                          \
      const float* src_ = base_ + (row_ * N1 + (f_ % N1));                        \
      __builtin_amdgcn_global_load_lds(                                           \
          (const void*)src_, (__attribute__((address_space(3))) void*)(a1me + k * 256), 16, 0, 0); \
    }                                                                             \
  } while (0)
  const int nch = (npx + 31) / 32;
  // A1[p][c] of this lane's accumulator slots, read from the LDS image at use
#define SRCNN_D1_A1(T, R) a1me[crow(R, h) * N1 + 32 * (T) + li]

  for (int sample = blockIdx.x; sample < g.batch; sample += gridDim.x) {
    __syncthreads();
    if (wave < nch) SRCNN_D1_A1_DMA(sample, wave);
    {
      const float* src = X + (size_t)sample * g.W * g.H;
      for (int i = threadIdx.x; i < g.W * g.H; i += 256) xs[i] = src[i];
    }
    __syncthreads();

    for (int c = wave; c < nch; c += 4) {
      {  // this lane's own pixel -> X base offset table
        const int p = min(c * 32 + li, npx - 1);
        const int y = p / g.ow, x = p - y * g.ow;
        if (h == 0) xbt[wave][li] = y * g.W + x;
      }
      // stage the delta2 chunk [32 px][N2] (zero rows past the sample)
      const float* dsrc = D2 + ((size_t)sample * npx + c * 32) * N2;
      for (int i = lane; i < 32 * N2 / 4; i += 64) {
        const int row = i / (N2 / 4), q = i - row * (N2 / 4);
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (c * 32 + row < npx) v = reinterpret_cast<const float4*>(dsrc)[i];
        float* d = d2me + row * DS + 4 * q;
        d[0] = v.x;
        d[1] = v.y;
        d[2] = v.z;
        d[3] = v.w;
      }
      // the A1 DMA of this chunk has landed (the delta2 loads above already
      // waited for the older VM ops; keep the wait explicit for the DMA)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_wave_barrier();

      // delta1[p][c] = [A1 > 0] * sum_n delta2[p][n] * W2[c][n]  (layer_deltas.cl, f=1)
      f32x16 d1[NT1];
#pragma unroll
      for (int t = 0; t < NT1; t++) d1[t] = zero16();
#pragma unroll
      for (int s = 0; s < KD; s++) {
        const int n = 2 * s + h;
        const float a = n < N2 ? d2me[li * DS + n] : 0.0f;
#pragma unroll
        for (int t = 0; t < NT1; t++) {
          const float b = n < N2 ? w2s[(32 * t + li) * WS + n] : 0.0f;
          d1[t] = mma(a, b, d1[t]);
        }
      }
#pragma unroll
      for (int t = 0; t < NT1; t++)
#pragma unroll
        for (int r = 0; r < 16; r++) d1[t][r] = SRCNN_D1_A1(t, r) > 0.0f ? d1[t][r] : 0.0f;

      // gW2[c][n] += sum_p A1[p][c] delta2[p][n]; gB2[n] += sum_p delta2[p][n]
#pragma unroll
      for (int s = 0; s < 16; s++) {
        const int pr = crow(s, h);
#pragma unroll
        for (int u = 0; u < NT2; u++) {
          const int n = 32 * u + li;
          const float b = n < N2 ? d2me[pr * DS + n] : 0.0f;
          gb2[u] += b;
#pragma unroll
          for (int t = 0; t < NT1; t++) g2[t][u] = mma(SRCNN_D1_A1(t, s), b, g2[t][u]);
        }
      }

      // next chunk's A1 DMA overlaps the gW1 MFMAs (the image's reads retired)
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      if (c + 4 < nch) SRCNN_D1_A1_DMA(sample, c + 4);

      // gW1[tap][c] += sum_p X[p + tap] delta1[p][c]; ones row -> gB1[c]
#pragma unroll
      for (int s = 0; s < 16; s++) {
        const int xb = xbt[wave][crow(s, h)];
#pragma unroll
        for (int m = 0; m < MT; m++) {
          float a = xs[xb + toff[m]];
          if (32 * m + 31 >= K1) a = tsel_x[m] != 0.0f ? a : tsel_1[m];  // zero rows / ones row
#pragma unroll
          for (int t = 0; t < NT1; t++) g1[m][t] = mma(a, d1[t][s], g1[m][t]);
        }
#ifdef SRCNN_D1_SCHED
        if ((s & (SRCNN_D1_SCHED - 1)) == SRCNN_D1_SCHED - 1) __builtin_amdgcn_sched_barrier(0);
#endif
      }
      __builtin_amdgcn_wave_barrier();
    }
  }
#undef SRCNN_D1_A1_DMA
#undef SRCNN_D1_A1

  // ---- block reduction (waves in order) into LDS, then one slab per block ----
  __syncthreads();
  float* red = smem;
  for (int w = 0; w < 4; w++) {
    if (wave == w) {
      int k = 0;
#pragma unroll
      for (int m = 0; m < MT; m++)
#pragma unroll
        for (int t = 0; t < NT1; t++, k++)
#pragma unroll
          for (int r = 0; r < 16; r++) {
            float* d = red + (k * 16 + r) * 64 + lane;
            *d = (w == 0 ? 0.0f : *d) + g1[m][t][r];
          }
#pragma unroll
      for (int t = 0; t < NT1; t++)
#pragma unroll
        for (int u = 0; u < NT2; u++, k++)
#pragma unroll
          for (int r = 0; r < 16; r++) {
            float* d = red + (k * 16 + r) * 64 + lane;
            *d = (w == 0 ? 0.0f : *d) + g2[t][u][r];
          }
    }
    __syncthreads();
  }
  float* out = slab + (size_t)blockIdx.x * P12;
  for (int i = threadIdx.x; i < RED; i += blockDim.x) {
    const int k = i / 1024, r = (i >> 6) & 15, l = i & 63;
    const int row = crow(r, l >> 5), col = l & 31;
    if (k < MT * NT1) {
      const int m = k / NT1, t = k - m * NT1;
      const int tap = 32 * m + row, ch = 32 * t + col;
      if (tap < K1) out[tap * N1 + ch] = red[i];
      else if (tap == K1) out[NW1 + ch] = red[i];
    } else {
      const int kk = k - MT * NT1;
      const int t = kk / NT2, u = kk - t * NT2;
      const int ch = 32 * t + row, n = 32 * u + col;
      if (n < N2) out[NW1 + N1 + ch * N2 + n] = red[i];
    }
  }
  // gB2: combine the two lane halves, then waves in order
  __syncthreads();
#pragma unroll
  for (int u = 0; u < NT2; u++) {
    const float v = gb2[u] + __shfl_down(gb2[u], 32, 64);
    if (h == 0) red[(wave * NT2 + u) * 32 + li] = v;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < NT2 * 32; i += blockDim.x) {
    const int u = i / 32, n = 32 * u + (i & 31);
    if (n < N2) {
      float v = 0.f;
      for (int w = 0; w < 4; w++) v += red[(w * NT2 + u) * 32 + (i & 31)];
      out[NW1 + N1 + NW2 + n] = v;
    }
  }
}
// ---------------------------------------------------------------------------
// deterministic slab reduction: dst[i] += sum_b slab[b][i]
// block = 64 columns x 16 rows; row r sums slabs r, r+16, ... in order, then
// the 16 row partials are added in row order (a fixed tree: bit-reproducible)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(1024) void slab_reduce_kernel(const float* __restrict__ slab, int nslab,
                                                           int P, float* __restrict__ dst) {
  __shared__ float part[16][65];
  const int col = blockIdx.x * 64 + (threadIdx.x & 63);
  const int row = threadIdx.x >> 6;
  float acc = 0.0f;
  if (col < P)
    for (int b = row; b < nslab; b += 16) acc += slab[(size_t)b * P + col];
  part[row][threadIdx.x & 63] = acc;
  __syncthreads();
  if (row == 0 && col < P) {
    float t = 0.0f;
#pragma unroll
    for (int r = 0; r < 16; r++) t += part[r][threadIdx.x];
    dst[col] += t;
  }
}

static int reduce_slabs(const float* slab, int nslab, int P, float* dst, hipStream_t s) {
  hipLaunchKernelGGL(slab_reduce_kernel, dim3((P + 63) / 64), dim3(1024), 0, s, slab, nslab, P, dst);
  SRCNN_LAUNCH_TRY();
  return SRCNN_OK;
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
template <int N1, int N2, int F1, int F3>
struct Net {
  static constexpr int P12 = F1 * F1 * N1 + N1 + N1 * N2 + N2;
  static constexpr int P3 = F3 * F3 * N2 + 1;
};

static int grid_for_batch(uint32_t batch, int cap) { return (int)std::min<uint32_t>(batch, cap); }

template <int N2, int F3, int PF>
static int launch_l3(const float* A2, const float* T, const float* W3, const float* B3, float* D2,
                     float* slab3, float* sqs, const L3Geom& lg, int grid, size_t lds, hipStream_t s) {
  static bool attr = false;  // the A2 tile exceeds the 64 KiB default dynamic LDS
  if (!attr) {
    hipError_t e = hipFuncSetAttribute((const void*)l3_delta_kernel<N2, F3, PF>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess)
      return fail(SRCNN_ERR_HIP, "hipFuncSetAttribute(l3_delta): %s", hipGetErrorString(e));
    attr = true;
  }
  hipLaunchKernelGGL((l3_delta_kernel<N2, F3, PF>), dim3(grid), dim3(kL3Threads), lds, s, A2, T,
                     W3, B3, D2, slab3, sqs, lg);
  SRCNN_LAUNCH_TRY();
  return SRCNN_OK;
}

// Returns 1 if the shape is specialised (and the step was enqueued), 0 if
// not (caller falls back to the op-by-op path), <0 on error.
template <int N1, int N2, int F1, int F3>
static int run(const float* X, const float* T, uint32_t w, uint32_t h, uint32_t batch,
               const float* params, float* grads, float* sq_err, float* A1, float* A2, float* D2,
               float* slab, size_t slab_bytes, hipStream_t s, bool query_only, size_t* need) {
  using NetT = Net<N1, N2, F1, F3>;
  const int ow = w - F1 + 1, oh = h - F1 + 1;
  const int w3 = ow - F3 + 1, h3 = oh - F3 + 1;
  if ((int)(w * h) > kXsMax || w3 <= 0 || h3 <= 0) return 0;
  const int npx2 = ow * oh;
  const int pf = l3_prefetch_regs<N2, F3>(npx2);
  if (pf > 16) return 0;
  const size_t lds3 = l3_lds_bytes<N2, F3>(npx2, ow);
  if (lds3 > 160 * 1024 || w3 * h3 > kL3MaxOut) return 0;
  const int g12 = grid_for_batch(batch, 1024);
  const int g3 = grid_for_batch(batch, 256);
  const int gd = grid_for_batch(batch, 512);
  const size_t s12 = (size_t)gd * NetT::P12, s3 = (size_t)g3 * NetT::P3;
  const size_t bytes = (s12 + s3 + g3) * sizeof(float);
  if (query_only) {
    *need = bytes;
    return 1;
  }
  if (slab_bytes < bytes)
    return fail(SRCNN_ERR_WORKSPACE, "fused train step: slab workspace %zu B < %zu B", slab_bytes, bytes);
  float* slab12 = slab;
  float* slab3 = slab12 + s12;
  float* sqs = slab3 + s3;
  // flat parameter layout [W1|B1|W2|B2|W3|B3]
  const float* W1 = params;
  const float* B1 = W1 + F1 * F1 * N1;
  const float* W2 = B1 + N1;
  const float* B2 = W2 + N1 * N2;
  const float* W3 = B2 + N2;
  const float* B3 = W3 + F3 * F3 * N2;
  Geom g{(int)w, (int)h, ow, oh, ow, oh, 1, 1, (int)batch};
  {
    SRCNN_PROFILE("l12_fwd_mfma", s);
    hipLaunchKernelGGL((l12_fwd_kernel<N1, N2, F1, true, true>), dim3(g12), dim3(256), 0, s, X, W1,
                       B1, W2, B2, A1, A2, g);
    SRCNN_LAUNCH_TRY();
  }
  L3Geom lg{(int)w, (int)h, ow, oh, w3, h3, (int)batch};
  {
    SRCNN_PROFILE("l3_delta_fused", s);
    int rc = pf <= 10 ? launch_l3<N2, F3, 10>(A2, T, W3, B3, D2, slab3, sqs, lg, g3, lds3, s)
                      : launch_l3<N2, F3, 16>(A2, T, W3, B3, D2, slab3, sqs, lg, g3, lds3, s);
    if (rc) return rc;
  }
  {
    SRCNN_PROFILE("delta1_grad12_fused", s);
    hipLaunchKernelGGL((d1_grad12_kernel<N1, N2, F1>), dim3(gd), dim3(256), 0, s, X, A1, D2, W2,
                       slab12, g);
    SRCNN_LAUNCH_TRY();
  }
  {
    SRCNN_PROFILE("slab_reduce", s);
    int rc = reduce_slabs(slab12, gd, NetT::P12, grads, s);
    if (!rc) rc = reduce_slabs(slab3, g3, NetT::P3, grads + NetT::P12, s);
    if (!rc && sq_err) rc = reduce_slabs(sqs, g3, 1, sq_err, s);
    if (rc) return rc;
  }
  return 1;
}

template <int N1, int N2, int F1, int F3>
static int dispatch_one(const srcnn_net* net, const float* X, const float* T, uint32_t w,
                        uint32_t h, uint32_t batch, const float* params, float* grads,
                        float* sq_err, float* A1, float* A2, float* D2, float* slab,
                        size_t slab_bytes, hipStream_t s, bool query_only, size_t* need) {
  if (net->n1 != (uint32_t)N1 || net->n2 != (uint32_t)N2 || net->f1 != (uint32_t)F1 ||
      net->f2 != 1 || net->f3 != (uint32_t)F3)
    return 0;
  return run<N1, N2, F1, F3>(X, T, w, h, batch, params, grads, sq_err, A1, A2, D2, slab,
                             slab_bytes, s, query_only, need);
}

int train_fwd_bwd(const srcnn_net* net, const float* X, const float* T, uint32_t w, uint32_t h,
                  uint32_t batch, const float* params, float* grads, float* sq_err, float* A1,
                  float* A2, float* D2, float* slab, size_t slab_bytes, hipStream_t s,
                  bool query_only, size_t* need) {
  int rc;
#define SRCNN_FUSED_CASE(n1, n2, f1, f3)                                                         \
  if ((rc = dispatch_one<n1, n2, f1, f3>(net, X, T, w, h, batch, params, grads, sq_err, A1, A2,  \
                                         D2, slab, slab_bytes, s, query_only, need)) != 0)       \
    return rc;
  SRCNN_FUSED_CASE(64, 32, 9, 5)  // reference default (BASELINE.json configs[1])
  SRCNN_FUSED_CASE(32, 16, 9, 5)  // example_config.json
#undef SRCNN_FUSED_CASE
  return 0;
}

}  // namespace fused
}  // namespace srcnn

#ifdef SRCNN_L3_TIMING
extern "C" __attribute__((visibility("default"))) int srcnn_debug_l3_timing(unsigned long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(srcnn::fused::g_l3_timing), sizeof(srcnn::fused::g_l3_timing)) ==
                 hipSuccess
             ? 0
             : -1;
}
#endif
