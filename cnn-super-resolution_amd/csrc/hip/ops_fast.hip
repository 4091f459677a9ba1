// ops_fast.hip -- gfx950 kernels behind the op-level ABI (srcnn_conv_fwd /
// srcnn_conv_delta / srcnn_conv_grad_acc), i.e. the reference's per-layer
// launchers DataPipeline::execute_layer / calculate_deltas / backpropagate
// (src/DataPipeline.cpp:358-410, :522-594, :596-663) as a caller of the C
// ABI drives them: one launch per layer and stage, activations and deltas in
// the reference HWC layout in HBM (src/kernel/layer_uber_kernel.cl:51-56).
//
// Three kernel families cover the SRCNN layer shapes, all fp32 MFMA
// (v_mfma_f32_16x16x4_f32 / 32x32x2_f32, exact fp32 fma chains):
//
//   pointwise (f == 1: the n1 -> n2 middle layer of the default / example
//   nets).  The convolution is per pixel, so the whole batch is one pixel
//   array and any image size works:
//     pw_kernel<fwd>    out^T[n][p] = W^T . in^T      (M = n, N = 16 px, K = n_prev)
//     pw_kernel<delta>  d^T[c][p]  = W . d_next^T, relu'(y) applied on store
//     pw_grad_kernel    gW[k][n]  += in^T . d         (M = k, N = n, K = pixels)
//   The operands come straight from HBM: with the k index of a 16x16x4
//   MFMA being only the lane group, a lane loads 4 consecutive channels of
//   its pixel as one 16-B load and feeds them to 4 consecutive MFMAs (the W
//   operand uses the same channel order), so every load is a 64-B run per
//   pixel and no LDS round trip is needed.
//
//   single input channel (n_prev == 1: layer 1, f1 x f1 x 1 -> n1), per
//   image window (up to (40 - f1 + 1)^2 outputs) with its 40 x 40 input
//   window in LDS, so any image size runs here:
//     l1_fwd_kernel     transposed: M = 32 channels, N = pixels (32), K = taps
//                       (paired), so a lane ends with 4 runs of 4 consecutive
//                       channels of one pixel: 16-B stores
//     l1_grad_kernel    gW1 (+ gB1 through a ones row): M = taps, N = n1, K = px
//
//   the wide middle layer (5x5, n1 = 128 <-> n2 = 64): train_wide.hip's
//   conv_mfma (forward, delta1) and wgrad2 kernels (wide::op_*), on image
//   windows past 31 x 31
//
//   single output channel (n_cur == 1 / n_next == 1: layer 3, f3 x f3 x n2
//   -> 1), per image window (forward: 21 x 21 outputs; delta2 / gW3: 64 x 64
//   A2 pixels):
//     l3_fwd_kernel     Q[q][tap] = A2[q][:] . W3[tap][:] (MFMA, HBM operands),
//                       A3[p] = B3 + sum_tap Q[p + off(tap)][tap] (LDS)
//     l3_delta_kernel   delta2[q][c] = relu'(A2) sum_tap delta3(q - off(tap)) W3[tap][c]
//                       (the window's delta3 neighbourhood with a zero border, LDS)
//     l3_grad_kernel    gW3[tap][c] = sum_q delta3(q - off(tap)) A2[q][c]: M = taps,
//                       N = n2, K = A2 pixels
//
// Gradients are summed deterministically: per-block slabs, then the
// fixed-order slab reduction of train_fused.hip adds them into gW / gB (the
// racy += of backpropagate.cl:110 is not reproduced).  Shapes outside these
// families return 0 and abi.cpp runs ops_generic.hip instead;
// srcnn_last_path() reports which.
#include <algorithm>

#include "common.hpp"
#include "mfma.hpp"
#include "ops.hpp"

namespace srcnn {
namespace fast {

using mfma::crow;
using mfma::f32x16;
using mfma::f32x4;
using mfma::lane_id;
using mfma::mma;
using mfma::mma16;
using mfma::wave_id;
using mfma::zero16;
using mfma::zero4;

namespace {

constexpr int kWaves = 4;  // 256-thread blocks everywhere

uint32_t blocks_for(size_t work, size_t per_block, uint32_t cap) {
  size_t b = (work + per_block - 1) / per_block;
  if (b < 1) b = 1;
  return b > cap ? cap : (uint32_t)b;
}

// ===========================================================================
// pointwise forward / delta
// ===========================================================================
// MODE 0 forward: out[p][n] = act(sum_k in[p][k] W[k][n] + B[n])    W: [CIN][COUT]
// MODE 1 delta:   out[p][c] = [aux[p][c] > 0] sum_k in[p][k] W[c][k] W: [COUT][CIN]
//   (layer_deltas.cl:79-123 with f_next = 1: W_next[0][c][k], c in n_curr)
template <int CIN, int COUT, int MODE>
__global__ __launch_bounds__(256) void pw_kernel(const float* __restrict__ in,
                                                 const float* __restrict__ W,
                                                 const float* __restrict__ aux,
                                                 float* __restrict__ out, long long npx, int relu) {
  constexpr int KJ = CIN / 16, NT = COUT / 16;
  const int lane = lane_id(), lq = lane & 15, lg = lane >> 4;
  // A operand of k-step (j, i): W(k = 16j + 4lg + i, n = 16t + lq)
  float wr[KJ][4][NT];
#pragma unroll
  for (int j = 0; j < KJ; j++)
#pragma unroll
    for (int i = 0; i < 4; i++)
#pragma unroll
      for (int t = 0; t < NT; t++) {
        const int k = 16 * j + 4 * lg + i, n = 16 * t + lq;
        wr[j][i][t] = MODE == 0 ? W[k * COUT + n] : W[n * CIN + k];
      }
  f32x4 bias[NT];
#pragma unroll
  for (int t = 0; t < NT; t++)
#pragma unroll
    for (int i = 0; i < 4; i++) bias[t][i] = MODE == 0 ? aux[16 * t + 4 * lg + i] : 0.0f;

  const long long nunits = (npx + 15) / 16;
  const long long stride = (long long)gridDim.x * kWaves;
  long long u = (long long)blockIdx.x * kWaves + wave_id();
  f32x4 x[KJ];
  auto load = [&](long long uu) {
    const long long p = min(uu * 16 + lq, npx - 1);
    const float* src = in + p * CIN + 4 * lg;
#pragma unroll
    for (int j = 0; j < KJ; j++) x[j] = *reinterpret_cast<const f32x4*>(src + 16 * j);
  };
  if (u < nunits) load(u);
  for (; u < nunits; u += stride) {
    f32x4 cur[KJ];
#pragma unroll
    for (int j = 0; j < KJ; j++) cur[j] = x[j];
    if (u + stride < nunits) load(u + stride);
    f32x4 acc[NT];
#pragma unroll
    for (int t = 0; t < NT; t++) acc[t] = zero4();
#pragma unroll
    for (int j = 0; j < KJ; j++)
#pragma unroll
      for (int i = 0; i < 4; i++)
#pragma unroll
        for (int t = 0; t < NT; t++) acc[t] = mma16(wr[j][i][t], cur[j][i], acc[t]);
    // lane (lq, lg) holds channels 16t + 4lg .. +3 of pixel 16u + lq
    const long long p = u * 16 + lq;
    if (p < npx) {
#pragma unroll
      for (int t = 0; t < NT; t++) {
        const long long o = p * COUT + 16 * t + 4 * lg;
        f32x4 v = acc[t];
        if (MODE == 0) {
#pragma unroll
          for (int i = 0; i < 4; i++) {
            v[i] += bias[t][i];  // the bias after the sum (layer_uber_kernel.cl:88-95)
            if (relu) v[i] = fmaxf(v[i], 0.0f);
          }
        } else {
          const f32x4 m = *reinterpret_cast<const f32x4*>(aux + o);
#pragma unroll
          for (int i = 0; i < 4; i++) v[i] = m[i] > 0.0f ? v[i] : 0.0f;
        }
        *reinterpret_cast<f32x4*>(out + o) = v;
      }
    }
  }
}

// ===========================================================================
// pointwise gradients: gW[k][n] += sum_p in[p][k] d[p][n], gB[n] += sum_p d[p][n]
// (backpropagate.cl:89-112 with f == 1), one slab per block
// ===========================================================================
template <int CIN, int COUT>
__global__ __launch_bounds__(256) void pw_grad_kernel(const float* __restrict__ in,
                                                      const float* __restrict__ d,
                                                      float* __restrict__ slab, long long npx) {
  constexpr int MT = CIN / 16, NT = COUT / 16, P = CIN * COUT + COUT;
  __shared__ float red[MT * NT * 4 * 64 + NT * 64];
  const int lane = lane_id(), wave = wave_id(), lq = lane & 15, lg = lane >> 4;
  f32x4 acc[MT][NT];
#pragma unroll
  for (int m = 0; m < MT; m++)
#pragma unroll
    for (int t = 0; t < NT; t++) acc[m][t] = zero4();
  float gb[NT];
#pragma unroll
  for (int t = 0; t < NT; t++) gb[t] = 0.0f;
  // K = pixels, 4 per step (lane group lg), two steps per iteration
  const long long ngrp = (npx + 7) / 8;
  const long long stride = (long long)gridDim.x * kWaves;
  float a[2][MT], b[2][NT];
  auto load = [&](long long g) {
#pragma unroll
    for (int h = 0; h < 2; h++) {
      const long long p = g * 8 + 4 * h + lg;
      const bool ok = p < npx;
      const long long pc = ok ? p : npx - 1;
#pragma unroll
      for (int m = 0; m < MT; m++) a[h][m] = ok ? in[pc * CIN + 16 * m + lq] : 0.0f;
#pragma unroll
      for (int t = 0; t < NT; t++) b[h][t] = ok ? d[pc * COUT + 16 * t + lq] : 0.0f;
    }
  };
  long long g = (long long)blockIdx.x * kWaves + wave;
  if (g < ngrp) load(g);
  for (; g < ngrp; g += stride) {
    float ca[2][MT], cb[2][NT];
#pragma unroll
    for (int h = 0; h < 2; h++) {
#pragma unroll
      for (int m = 0; m < MT; m++) ca[h][m] = a[h][m];
#pragma unroll
      for (int t = 0; t < NT; t++) cb[h][t] = b[h][t];
    }
    if (g + stride < ngrp) load(g + stride);
#pragma unroll
    for (int h = 0; h < 2; h++)
#pragma unroll
      for (int m = 0; m < MT; m++)
#pragma unroll
        for (int t = 0; t < NT; t++) acc[m][t] = mma16(ca[h][m], cb[h][t], acc[m][t]);
#pragma unroll
    for (int t = 0; t < NT; t++) gb[t] += cb[0][t] + cb[1][t];
  }
  // block reduction, waves in order; lane (lq, lg) reg i holds gW[16m + 4lg + i][16t + lq]
  for (int w = 0; w < kWaves; w++) {
    if (wave == w) {
#pragma unroll
      for (int m = 0; m < MT; m++)
#pragma unroll
        for (int t = 0; t < NT; t++)
#pragma unroll
          for (int i = 0; i < 4; i++) {
            float* dst = red + (((m * NT + t) * 4 + i) * 64 + lane);
            *dst = (w == 0 ? 0.0f : *dst) + acc[m][t][i];
          }
#pragma unroll
      for (int t = 0; t < NT; t++) {
        float* dst = red + MT * NT * 256 + t * 64 + lane;
        *dst = (w == 0 ? 0.0f : *dst) + gb[t];
      }
    }
    __syncthreads();
  }
  float* o = slab + (size_t)blockIdx.x * P;
  for (int e = threadIdx.x; e < MT * NT * 256; e += blockDim.x) {
    const int l = e & 63, i = (e >> 6) & 3, mt = e >> 8;
    const int m = mt / NT, t = mt - m * NT;
    o[(16 * m + 4 * (l >> 4) + i) * COUT + 16 * t + (l & 15)] = red[e];
  }
  for (int n = threadIdx.x; n < COUT; n += blockDim.x) {
    const float* v = red + MT * NT * 256 + (n >> 4) * 64 + (n & 15);
    o[CIN * COUT + n] = ((v[0] + v[16]) + v[32]) + v[48];
  }
}

// ===========================================================================
// layer 1 forward (n_prev == 1): A1 = act(B1 + conv(X, W1)), per work item
// GEMM M = pixels (32-row tiles, two per wave pass), N = 32 channels, K =
// taps; the k-slot pairing gives half h the taps [KP h, KP h + KP), so every
// operand read is a per-half base + an immediate.
// A work item is one window of an image: up to (kXS - F1 + 1)^2 output pixels
// whose kXS x kXS input window sits in LDS, so any image size runs here (a
// 33x33 training tile is one window; a 256x256 image 64 of them).
// ===========================================================================
constexpr int kXS = 40;                    // LDS row stride of an input window
constexpr int kXTile = kXS * (kXS + 1);    // + one zero row read by the padded tap

// window geometry of work item `it` over `batch` images of w x h inputs
struct L1Win {
  int s, x0, y0, ow, oh;  // image, output window origin and size
  __device__ L1Win(long long it, int w1, int h1, int wo) {
    const int nwx = (w1 + wo - 1) / wo, nwin = nwx * ((h1 + wo - 1) / wo);
    s = nwin == 1 ? (int)it : (int)(it / nwin);
    const int wi = (int)(it - (long long)s * nwin), wy = wi / nwx;
    x0 = (wi - wy * nwx) * wo;
    y0 = wy * wo;
    ow = min(wo, w1 - x0);
    oh = min(wo, h1 - y0);
  }
};
__host__ __device__ inline long long l1_items(int w1, int h1, int wo, int batch) {
  return (long long)batch * ((w1 + wo - 1) / wo) * ((h1 + wo - 1) / wo);
}

// pixel p of a window of width ow -> its offset in an image of width wfull
// from the window origin (no division when the window spans the image width,
// as every training tile does)
__device__ __forceinline__ int win_px(int p, int ow, int wfull) {
  if (ow == wfull) return p;
  const int y = p / ow;
  return y * wfull + p - y * ow;
}

// X window of `win` -> xs (rows at stride kXS), and a zero row below it for
// the padded tap; the caller brackets it with barriers
template <int F1>
__device__ void stage_x_window(const float* __restrict__ X, float* xs, const L1Win& win, int w, int h) {
  const int iw = win.ow + F1 - 1, ih = win.oh + F1 - 1;
  const float* src = X + (size_t)win.s * w * h + (size_t)win.y0 * w + win.x0;
  for (int i = threadIdx.x; i < iw * ih; i += blockDim.x) {
    const int y = i / iw;
    xs[y * kXS + i - y * iw] = src[(size_t)y * w + i - y * iw];
  }
  for (int i = threadIdx.x; i < kXS; i += blockDim.x) xs[ih * kXS + i] = 0.0f;
}

template <int N1, int F1>
__global__ __launch_bounds__(256) void l1_fwd_kernel(const float* __restrict__ X,
                                                     const float* __restrict__ W1,
                                                     const float* __restrict__ B1,
                                                     float* __restrict__ A1, int w, int h, int batch,
                                                     int relu) {
  constexpr int K1 = F1 * F1, KP = (K1 + 1) / 2, Q = KP / F1, R = KP % F1;
  constexpr int NTW = N1 / 32;              // channel tiles
  constexpr int MG = kWaves / NTW;          // waves per channel tile (pixel-pair groups)
  static_assert(N1 % 32 == 0 && NTW <= kWaves, "n1 = 32, 64 or 128");
  __shared__ float xs[kXTile];
  const int lane = lane_id(), wave = wave_id(), j = lane & 31, hh = lane >> 5;
  const int nt = wave % NTW, mg = wave / NTW;
  const int n = 32 * nt + j;
  // A operand (transposed GEMM): W1[tap kp + KP hh][channel n]
  float wb[KP];
#pragma unroll
  for (int kp = 0; kp < KP; kp++) {
    const int t = kp + KP * hh;
    wb[kp] = t < K1 ? W1[t * N1 + n] : 0.0f;
  }
  // C register 4g + i of lane (j, hh) is channel 32 nt + 8g + 4hh + i of pixel j
  f32x4 bias[4];
#pragma unroll
  for (int g = 0; g < 4; g++) bias[g] = *reinterpret_cast<const f32x4*>(B1 + 32 * nt + 8 * g + 4 * hh);
  for (int i = threadIdx.x; i < kXTile; i += 256) xs[i] = 0.0f;
  const int w1 = w - F1 + 1, h1 = h - F1 + 1;
  constexpr int WO = kXS - F1 + 1;
  const long long items = l1_items(w1, h1, WO, batch);
  // tap kp + KP (half 1) sits at one of two fixed offsets from tap kp
  const int dA = hh * (Q * kXS + R), dB = hh * ((Q + 1) * kXS + R - F1);
  for (long long it = blockIdx.x; it < items; it += gridDim.x) {
    const L1Win win(it, w1, h1, WO);
    const int npx = win.ow * win.oh, mtiles = (npx + 31) / 32;
    __syncthreads();
    stage_x_window<F1>(X, xs, win, w, h);
    __syncthreads();
    float* dst = A1 + ((size_t)win.s * w1 * h1 + (size_t)win.y0 * w1 + win.x0) * N1 + 32 * nt + 4 * hh;
    for (int m = 2 * mg; m < mtiles; m += 2 * MG) {
      int base[2];
#pragma unroll
      for (int u = 0; u < 2; u++) {
        const int o = min(32 * (m + u) + j, npx - 1), oy = o / win.ow;
        base[u] = oy * kXS + o - oy * win.ow;
      }
      f32x16 acc0 = zero16(), acc1 = zero16();
#pragma unroll
      for (int kp = 0; kp < KP; kp++) {
        const int toff = (kp / F1) * kXS + kp % F1;
        const int dd = (kp % F1 + R < F1) ? dA : dB;
        acc0 = mma(wb[kp], xs[base[0] + dd + toff], acc0);
        acc1 = mma(wb[kp], xs[base[1] + dd + toff], acc1);
      }
      // this lane's pixels of the two tiles, as offsets in the image
      const int p0 = 32 * m + j, p1 = p0 + 32;
      const size_t q0 = (size_t)win_px(p0, win.ow, w1) * N1, q1 = (size_t)win_px(p1, win.ow, w1) * N1;
#pragma unroll
      for (int g = 0; g < 4; g++) {
        f32x4 v0, v1;
#pragma unroll
        for (int i = 0; i < 4; i++) {
          v0[i] = acc0[4 * g + i] + bias[g][i];
          v1[i] = acc1[4 * g + i] + bias[g][i];
          if (relu) {
            v0[i] = fmaxf(v0[i], 0.0f);
            v1[i] = fmaxf(v1[i], 0.0f);
          }
        }
        if (p0 < npx) *reinterpret_cast<f32x4*>(dst + q0 + 8 * g) = v0;
        if (p1 < npx) *reinterpret_cast<f32x4*>(dst + q1 + 8 * g) = v1;
      }
    }
  }
}

// ===========================================================================
// layer 1 gradients (n_prev == 1): gW1[tap][n] += sum_p X[p + off(tap)] d[p][n],
// gB1[n] += sum_p d[p][n] (the ones row, tap index K1), per sample
// GEMM M = taps (16-row tiles), N = 16-channel tiles, K = pixels (4 per step)
// ===========================================================================
template <int N1, int F1>
struct L1Grad {
  static constexpr int K1 = F1 * F1;
  static constexpr int MT = (K1 + 1 + 15) / 16;    // tap tiles incl. the ones row
  static constexpr int NQ = N1 / 16;               // channel tiles
  static constexpr int CT = NQ < 4 ? NQ : (NQ >= 8 ? 2 : 4);  // channel tiles per wave (n1 = 128: 2,
                                                               // for two waves per SIMD)
  static constexpr int NCG = NQ / CT;              // channel groups
  static constexpr int WPG = kWaves / NCG;         // waves per channel group (pixel split)
  static constexpr int P = K1 * N1 + N1;
};

// MASK: D holds delta1 before its ReLU' factor, applied here from A1 (the
// wide step's wd1x6 writes D1 unmasked, so its epilogue loads no A1)
template <int N1, int F1, bool MASK = false>
__global__ __launch_bounds__(256, 1) void l1_grad_kernel(const float* __restrict__ X,
                                                         const float* __restrict__ D,
                                                         float* __restrict__ slab, int w, int h,
                                                         int batch, const float* __restrict__ A1 = nullptr) {
  using G = L1Grad<N1, F1>;
  constexpr int K1 = G::K1, MT = G::MT, CT = G::CT, WPG = G::WPG;
  static_assert(G::NQ % CT == 0 && kWaves % G::NCG == 0, "channel split");
  __shared__ float xs[kXTile + 64];
  __shared__ float red[MT * CT * 4 * 64];
  const int lane = lane_id(), wave = wave_id(), lq = lane & 15, lg = lane >> 4;
  const int cg = wave / WPG, ws = wave % WPG;  // channel group, pixel slice
  const int w1 = w - F1 + 1, h1 = h - F1 + 1;
  constexpr int WO = kXS - F1 + 1;
  const long long items = l1_items(w1, h1, WO, batch);
  // per-lane tap offsets of rows 16m + lq; the ones row / pad rows read fixed slots
  int toff[MT];
#pragma unroll
  for (int m = 0; m < MT; m++) {
    const int tap = 16 * m + lq;
    toff[m] = tap < K1 ? (tap / F1) * kXS + tap % F1 : (tap == K1 ? -1 : -2);
  }
  f32x4 acc[MT][CT];
#pragma unroll
  for (int m = 0; m < MT; m++)
#pragma unroll
    for (int t = 0; t < CT; t++) acc[m][t] = zero4();
  for (long long it = blockIdx.x; it < items; it += gridDim.x) {
    const L1Win win(it, w1, h1, WO);
    const int npx = win.ow * win.oh, ngrp = (npx + 3) / 4;
    __syncthreads();
    stage_x_window<F1>(X, xs, win, w, h);
    __syncthreads();
    const size_t doff = ((size_t)win.s * w1 * h1 + (size_t)win.y0 * w1 + win.x0) * N1 + 16 * CT * cg + lq;
    const float* ds = D + doff;
    float bn[CT], mn[CT];  // the next group's delta operands (HBM), in flight under the MFMAs
    auto load_b = [&](int gq) {
      const int p = 4 * gq + lg;
      const size_t q = win_px(min(p, npx - 1), win.ow, w1);  // window pixel -> image pixel
#pragma unroll
      for (int t = 0; t < CT; t++) {
        bn[t] = p < npx ? ds[q * N1 + 16 * t] : 0.0f;
        if (MASK) mn[t] = A1[doff + q * N1 + 16 * t];
      }
    };
    if (ws < ngrp) load_b(ws);
    // window pixel p = 4gq + lg as (row py, column px), advanced by 4 WPG
    // pixels per step without a division
    int py = (4 * ws + lg) / win.ow, px = 4 * ws + lg - py * win.ow;
    for (int gq = ws; gq < ngrp; gq += WPG) {
      const int p = 4 * gq + lg;
      const bool ok = p < npx;
      const int xb = ok ? py * kXS + px : 0;  // (rows past the window: delta operand 0)
      for (px += 4 * WPG; px >= win.ow; px -= win.ow) ++py;
      float bv[CT];
#pragma unroll
      for (int t = 0; t < CT; t++) bv[t] = MASK ? (mn[t] > 0.0f ? bn[t] : 0.0f) : bn[t];
      if (gq + WPG < ngrp) load_b(gq + WPG);
      float av[MT];
#pragma unroll
      for (int m = 0; m < MT; m++)
        av[m] = toff[m] >= 0 ? xs[xb + toff[m]] : (toff[m] == -1 ? 1.0f : 0.0f);
#pragma unroll
      for (int m = 0; m < MT; m++)
#pragma unroll
        for (int t = 0; t < CT; t++) acc[m][t] = mma16(av[m], bv[t], acc[m][t]);
    }
  }
  // reduce the WPG waves of each channel group in order, then write the slab
  float* o = slab + (size_t)blockIdx.x * G::P;
  for (int g = 0; g < G::NCG; g++) {
    __syncthreads();
    for (int w = 0; w < WPG; w++) {
      if (cg == g && ws == w) {
#pragma unroll
        for (int m = 0; m < MT; m++)
#pragma unroll
          for (int t = 0; t < CT; t++)
#pragma unroll
            for (int i = 0; i < 4; i++) {
              float* dst = red + ((m * CT + t) * 4 + i) * 64 + lane;
              *dst = (w == 0 ? 0.0f : *dst) + acc[m][t][i];
            }
      }
      __syncthreads();
    }
    for (int e = threadIdx.x; e < MT * CT * 256; e += blockDim.x) {
      const int l = e & 63, i = (e >> 6) & 3, mt = e >> 8;
      const int m = mt / CT, t = mt - m * CT;
      const int tap = 16 * m + 4 * (l >> 4) + i, n = 16 * (CT * g + t) + (l & 15);
      if (tap < K1) o[tap * N1 + n] = red[e];
      else if (tap == K1) o[K1 * N1 + n] = red[e];
    }
  }
}

// ===========================================================================
// layer 3 (single output channel), per sample
// ===========================================================================
// Q[q][tap] for the A2 pixels q of a window: M = taps (16-row tiles), N = 16
// pixels, K = channels with 16-B operand loads of the input straight from HBM
// (see pw_kernel).  A work item is a window of up to wo x wo outputs (the
// L1Win geometry over the A3 grid) whose (wo + F3 - 1)^2 A2 pixels' Q rows sit
// in LDS; a training tile is one window, any larger image several.
template <int N2, int F3>
__global__ __launch_bounds__(256) void l3_fwd_kernel(const float* __restrict__ A2,
                                                     const float* __restrict__ W3,
                                                     const float* __restrict__ B3,
                                                     float* __restrict__ A3, int w2, int h2,
                                                     int batch, int relu, int wo) {
  constexpr int K3 = F3 * F3, TT = (K3 + 15) / 16, KJ = N2 / 16;
  extern __shared__ __attribute__((aligned(16))) float qs[];  // [window A2 pixels][K3]
  const int lane = lane_id(), wave = wave_id(), lq = lane & 15, lg = lane >> 4;
  // A operand of k-step (j, i): W3[tap = 16t + lq][c = 16j + 4lg + i]
  float wq[KJ][4][TT];
#pragma unroll
  for (int j = 0; j < KJ; j++)
#pragma unroll
    for (int i = 0; i < 4; i++)
#pragma unroll
      for (int t = 0; t < TT; t++) {
        const int tap = 16 * t + lq;
        wq[j][i][t] = tap < K3 ? W3[tap * N2 + 16 * j + 4 * lg + i] : 0.0f;
      }
  const float b3 = B3[0];
  const int w3 = w2 - F3 + 1, h3 = h2 - F3 + 1;
  const long long items = l1_items(w3, h3, wo, batch);
  for (long long it = blockIdx.x; it < items; it += gridDim.x) {
    const L1Win win(it, w3, h3, wo);
    const int iw = win.ow + F3 - 1, npxw = iw * (win.oh + F3 - 1), nunit = (npxw + 15) / 16;
    const float* src = A2 + ((size_t)win.s * w2 * h2 + (size_t)win.y0 * w2 + win.x0) * N2;
    f32x4 xn[KJ];  // the next unit's operands, in flight under this unit's MFMAs
    auto load_x = [&](int u) {
      const size_t g = win_px(min(16 * u + lq, npxw - 1), iw, w2);  // window pixel -> image pixel
#pragma unroll
      for (int j = 0; j < KJ; j++) xn[j] = *reinterpret_cast<const f32x4*>(src + g * N2 + 16 * j + 4 * lg);
    };
    if (wave < nunit) load_x(wave);
    for (int u = wave; u < nunit; u += kWaves) {
      f32x4 x[KJ];
#pragma unroll
      for (int j = 0; j < KJ; j++) x[j] = xn[j];
      if (u + kWaves < nunit) load_x(u + kWaves);
      f32x4 acc[TT];
#pragma unroll
      for (int t = 0; t < TT; t++) acc[t] = zero4();
#pragma unroll
      for (int j = 0; j < KJ; j++)
#pragma unroll
        for (int i = 0; i < 4; i++)
#pragma unroll
          for (int t = 0; t < TT; t++) acc[t] = mma16(wq[j][i][t], x[j][i], acc[t]);
      // lane (lq, lg) reg i: Q[16u + lq][tap = 16t + 4lg + i]
      if (16 * u + lq < npxw)
#pragma unroll
        for (int t = 0; t < TT; t++)
#pragma unroll
          for (int i = 0; i < 4; i++) {
            const int tap = 16 * t + 4 * lg + i;
            if (tap < K3) qs[(16 * u + lq) * K3 + tap] = acc[t][i];
          }
    }
    __syncthreads();
    float* dst = A3 + (size_t)win.s * w3 * h3 + (size_t)win.y0 * w3 + win.x0;
    for (int p = threadIdx.x; p < win.ow * win.oh; p += blockDim.x) {
      const int y = p / win.ow, x = p - y * win.ow;
      const float* qrow = qs + (y * iw + x) * K3;
      float acc = 0.0f;
#pragma unroll
      for (int dy = 0; dy < F3; dy++)
#pragma unroll
        for (int dx = 0; dx < F3; dx++) acc += qrow[(dy * iw + dx) * K3 + dy * F3 + dx];
      const float v = acc + b3;
      dst[win_px(p, win.ow, w3)] = relu ? fmaxf(v, 0.0f) : v;
    }
    __syncthreads();
  }
}

// The delta2 / gW3 kernels work on windows of up to kD3Win x kD3Win A2 pixels
// (L1Win over the A2 grid; a training tile is one window).  A window's delta3
// neighbourhood is staged with a zero border as the grid G of row stride
// gw = ow + F3 - 1: G[gy][gx] = delta3(y0 - (F3-1) + gy, x0 - (F3-1) + gx), 0
// outside the A3 grid.  For window pixel (py, px) at g = py * gw + px,
// delta3(A2 pixel - off(dy, dx)) is then G[g + d3off - (dy * gw + dx)] with
// d3off = (F3 - 1)(gw + 1): one add per tap.
constexpr int kD3Win = 64;

// gb != nullptr: also add the delta3 values at the window's own A2 pixels
// (gB3: every delta3 pixel is counted by exactly one window)
template <int F3>
__device__ void stage_d3_window(const float* __restrict__ D3, float* G, const L1Win& win, int w2, int h2,
                                float* gb = nullptr) {
  const int w3 = w2 - F3 + 1, h3 = h2 - F3 + 1;
  const int gw = win.ow + F3 - 1, ng = gw * (win.oh + F3 - 1);
  const float* src = D3 + (size_t)win.s * w3 * h3;
  __syncthreads();  // the previous window's readers are done
  for (int i = threadIdx.x; i < ng; i += blockDim.x) {
    const int gy = i / gw, gx = i - gy * gw;
    const int y = win.y0 - (F3 - 1) + gy, x = win.x0 - (F3 - 1) + gx;
    const float v = (y >= 0 && y < h3 && x >= 0 && x < w3) ? src[(size_t)y * w3 + x] : 0.0f;
    G[i] = v;
    if (gb && gy >= F3 - 1 && gx >= F3 - 1) *gb += v;
  }
  __syncthreads();
}

// delta2[q][c] = [A2[q][c] > 0] sum_tap delta3(q - off(tap)) W3[tap][c]
// (layer_deltas.cl:79-123 with n_next = 1); thread item = (pixel, channel quad)
template <int N2, int F3>
__global__ __launch_bounds__(256) void l3_delta_kernel(const float* __restrict__ D3,
                                                       const float* __restrict__ A2,
                                                       const float* __restrict__ W3,
                                                       float* __restrict__ D2, int w2, int h2,
                                                       int batch) {
  constexpr int K3 = F3 * F3, NQ = N2 / 4;
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* w3s = sm;            // [K3][N2]
  float* d3g = sm + K3 * N2;  // delta3 window grid
  for (int i = threadIdx.x; i < K3 * N2; i += blockDim.x) w3s[i] = W3[i];
  const long long items = l1_items(w2, h2, kD3Win, batch);
  for (long long it = blockIdx.x; it < items; it += gridDim.x) {
    const L1Win win(it, w2, h2, kD3Win);
    stage_d3_window<F3>(D3, d3g, win, w2, h2);
    const int gw = win.ow + F3 - 1, d3off = (F3 - 1) * (gw + 1);
    const size_t base = (size_t)win.s * w2 * h2 + (size_t)win.y0 * w2 + win.x0;
    const float* a2 = A2 + base * N2;
    float* d2 = D2 + base * N2;
    for (int e = threadIdx.x; e < win.ow * win.oh * NQ; e += blockDim.x) {
      const int p = e / NQ, cq = e - p * NQ, py = p / win.ow, px = p - py * win.ow;
      const int g = py * gw + px;                 // window grid pixel
      const size_t q = (size_t)py * w2 + px;      // image pixel (from the window origin)
      f32x4 acc = zero4();
#pragma unroll
      for (int dy = 0; dy < F3; dy++)
#pragma unroll
        for (int dx = 0; dx < F3; dx++) {
          const float dv = d3g[g + d3off - (dy * gw + dx)];
          const f32x4 wv = *reinterpret_cast<const f32x4*>(w3s + (dy * F3 + dx) * N2 + 4 * cq);
#pragma unroll
          for (int i = 0; i < 4; i++) acc[i] += dv * wv[i];
        }
      const f32x4 m = *reinterpret_cast<const f32x4*>(a2 + q * N2 + 4 * cq);
#pragma unroll
      for (int i = 0; i < 4; i++) acc[i] = m[i] > 0.0f ? acc[i] : 0.0f;
      *reinterpret_cast<f32x4*>(d2 + q * N2 + 4 * cq) = acc;
    }
  }
}

// gW3[tap][c] += sum_q delta3(q - off(tap)) A2[q][c], gB3 += sum delta3
// (backpropagate.cl:89-112 with n_cur = 1): M = taps, N = channels, K = A2 px
template <int N2, int F3>
__global__ __launch_bounds__(256) void l3_grad_kernel(const float* __restrict__ A2,
                                                      const float* __restrict__ D3,
                                                      float* __restrict__ slab, int w2, int h2,
                                                      int batch) {
  constexpr int K3 = F3 * F3, TT = (K3 + 15) / 16, NT = N2 / 16, P = K3 * N2 + 1;
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* d3g = sm;
  const int lane = lane_id(), wave = wave_id(), lq = lane & 15, lg = lane >> 4;
  f32x4 acc[TT][NT];
#pragma unroll
  for (int t = 0; t < TT; t++)
#pragma unroll
    for (int u = 0; u < NT; u++) acc[t][u] = zero4();
  float gb = 0.0f;
  const long long items = l1_items(w2, h2, kD3Win, batch);
  for (long long it = blockIdx.x; it < items; it += gridDim.x) {
    const L1Win win(it, w2, h2, kD3Win);
    stage_d3_window<F3>(D3, d3g, win, w2, h2, &gb);
    const int gw = win.ow + F3 - 1, d3off = (F3 - 1) * (gw + 1);
    const int npxw = win.ow * win.oh, ngrp = (npxw + 3) / 4;
    int goff[TT];  // window of tap 16t + lq (rows past K3 read a real window, discarded)
#pragma unroll
    for (int t = 0; t < TT; t++) {
      const int tap = min(16 * t + lq, K3 - 1);
      goff[t] = d3off - ((tap / F3) * gw + tap % F3);
    }
    const float* a2 = A2 + ((size_t)win.s * w2 * h2 + (size_t)win.y0 * w2 + win.x0) * N2 + lq;
    // the A2 operands (HBM) of the wave's next pixel group are in flight
    // while this group's MFMAs run
    float bn[NT];
    auto load_b = [&](int g) {
      const size_t qi = win_px(min(4 * g + lg, npxw - 1), win.ow, w2);
#pragma unroll
      for (int u = 0; u < NT; u++) bn[u] = a2[qi * N2 + 16 * u];
    };
    if (wave < ngrp) load_b(wave);
    // window pixel q = 4g + lg as (row qy, column qx), advanced by 4 kWaves
    // pixels per step without a division
    int qy = (4 * wave + lg) / win.ow, qx = 4 * wave + lg - qy * win.ow;
    for (int g = wave; g < ngrp; g += kWaves) {
      const int q = 4 * g + lg;
      const bool ok = q < npxw;
      const int gq = ok ? qy * gw + qx : 0;  // window grid pixel (rows past the window: unused)
      for (qx += 4 * kWaves; qx >= win.ow; qx -= win.ow) ++qy;
      float av[TT], bv[NT];
#pragma unroll
      for (int u = 0; u < NT; u++) bv[u] = bn[u];
      if (g + kWaves < ngrp) load_b(g + kWaves);
#pragma unroll
      for (int t = 0; t < TT; t++) av[t] = ok ? d3g[gq + goff[t]] : 0.0f;
#pragma unroll
      for (int t = 0; t < TT; t++)
#pragma unroll
        for (int u = 0; u < NT; u++) acc[t][u] = mma16(av[t], bv[u], acc[t][u]);
    }
  }
  // block reduction (waves in order) reusing the d3g area
  float* red = sm;
  __syncthreads();
  for (int w = 0; w < kWaves; w++) {
    if (wave == w) {
#pragma unroll
      for (int t = 0; t < TT; t++)
#pragma unroll
        for (int u = 0; u < NT; u++)
#pragma unroll
          for (int i = 0; i < 4; i++) {
            float* dst = red + ((t * NT + u) * 4 + i) * 64 + lane;
            *dst = (w == 0 ? 0.0f : *dst) + acc[t][u][i];
          }
    }
    __syncthreads();
  }
  float* o = slab + (size_t)blockIdx.x * P;
  for (int e = threadIdx.x; e < TT * NT * 256; e += blockDim.x) {
    const int l = e & 63, i = (e >> 6) & 3, k = e >> 8;
    const int t = k / NT, u = k - t * NT;
    const int tap = 16 * t + 4 * (l >> 4) + i, c = 16 * u + (l & 15);
    if (tap < K3) o[tap * N2 + c] = red[e];
  }
  // gB3: per-wave shuffle tree, waves in order
  for (int off = 32; off > 0; off >>= 1) gb += __shfl_down(gb, off, 64);
  __syncthreads();
  if (lane == 0) red[wave] = gb;
  __syncthreads();
  if (threadIdx.x == 0) o[K3 * N2] = ((red[0] + red[1]) + red[2]) + red[3];
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
constexpr uint32_t kGridCap = 2048;   // pointwise kernels: 8 blocks per CU
constexpr uint32_t kSlabCap = 512;    // gradient kernels: slab count (2 blocks per CU)

// per-block slabs [gW (nW) | gB (nB)] -> gW += rows, gB += rows (fixed order)
int reduce_rows(const float* slab, int nslab, int nW, int nB, float* gW, float* gB, hipStream_t s) {
  SRCNN_PROFILE("slab_reduce", s);
  const fused::SlabSeg segs[2] = {{slab, gW, nslab, nW, nW + nB}, {slab + nW, gB, nslab, nB, nW + nB}};
  return fused::reduce_slabs(segs, 2, s);
}

// the shapes of the reference configs (default 64/32, example 32/16, wide
// 128/64) and the sizes between them; n % 16 == 0 throughout
#define SRCNN_PW_SHAPES(X)                                                                       \
  X(64, 32) X(32, 16) X(32, 64) X(16, 32) X(16, 16) X(32, 32) X(64, 64) X(64, 16) X(16, 64)       \
  X(128, 32) X(32, 128)
#define SRCNN_N1_SHAPES(X) X(32, 9) X(64, 9) X(128, 9) X(32, 5) X(64, 5) X(64, 3)
#define SRCNN_N3_SHAPES(X) X(16, 5) X(32, 5) X(64, 5) X(16, 3) X(32, 3) X(64, 3)

// layer-3 forward window: the largest output side wo whose (wo + F3 - 1)^2 Q
// rows fit the default 64 KiB of LDS (21 at F3 = 5: a 33x33 training tile is
// one window), and the LDS its (clipped) window needs
int l3_fwd_wo(int F3) {
  int wo = 1;
  while ((size_t)(wo + F3) * (wo + F3) * F3 * F3 * sizeof(float) <= 64 * 1024) ++wo;
  return wo;
}
size_t l3_fwd_lds(int F3, uint32_t w2, uint32_t h2) {
  const uint32_t side = (uint32_t)(l3_fwd_wo(F3) + F3 - 1);
  return (size_t)std::min(w2, side) * std::min(h2, side) * F3 * F3 * sizeof(float);
}
// delta3 window grid of the delta2 / gW3 kernels
size_t d3_lds(int F3, uint32_t w2, uint32_t h2) {
  return ((size_t)(std::min<uint32_t>(w2, kD3Win) + F3 - 1) * (std::min<uint32_t>(h2, kD3Win) + F3 - 1)) *
         sizeof(float);
}
constexpr size_t kLdsCap = 64 * 1024;   // the default dynamic LDS of a launch

}  // namespace

int try_conv_fwd(const float* in, float* out, const float* W, const float* B, uint32_t in_w,
                 uint32_t in_h, uint32_t n_prev, uint32_t n_cur, uint32_t f, int relu,
                 uint32_t batch, hipStream_t s) {
  if (int rc = wide::op_conv_fwd(in, out, W, B, in_w, in_h, n_prev, n_cur, f, relu, batch, s)) return rc;
  if (f == 1) {  // pointwise: any image size
    const long long npx = (long long)batch * in_w * in_h;
    const uint32_t grid = blocks_for((npx + 15) / 16, kWaves, kGridCap);
#define SRCNN_PW_F(CI, CO)                                                                       \
    if (n_prev == CI && n_cur == CO) {                                                           \
      SRCNN_PROFILE("conv_fwd_pointwise_mfma", s);                                               \
      hipLaunchKernelGGL((pw_kernel<CI, CO, 0>), dim3(grid), dim3(256), 0, s, in, W, B, out, npx, \
                         relu);                                                                  \
      SRCNN_LAUNCH_TRY();                                                                        \
      return 1;                                                                                  \
    }
    SRCNN_PW_SHAPES(SRCNN_PW_F)
#undef SRCNN_PW_F
    return 0;
  }
  if (n_prev == 1 && in_w >= f && in_h >= f) {
    const long long items = l1_items((int)(in_w - f + 1), (int)(in_h - f + 1), kXS - (int)f + 1, (int)batch);
    const uint32_t grid = (uint32_t)std::min<long long>(items, 1024);
#define SRCNN_L1_F(N1, F1)                                                                      \
    if (n_cur == N1 && f == F1) {                                                               \
      SRCNN_PROFILE("conv_fwd_l1_mfma", s);                                                     \
      hipLaunchKernelGGL((l1_fwd_kernel<N1, F1>), dim3(grid), dim3(256), 0, s, in, W, B, out,   \
                         (int)in_w, (int)in_h, (int)batch, relu);                               \
      SRCNN_LAUNCH_TRY();                                                                       \
      return 1;                                                                                 \
    }
    SRCNN_N1_SHAPES(SRCNN_L1_F)
#undef SRCNN_L1_F
    return 0;
  }
  if (n_cur == 1) {  // windowed: any image size
    const int wo = l3_fwd_wo((int)f);
    const long long items = l1_items((int)(in_w - f + 1), (int)(in_h - f + 1), wo, (int)batch);
    const uint32_t grid = (uint32_t)std::min<long long>(items, 1024);
    const size_t lds = l3_fwd_lds(f, in_w, in_h);
#define SRCNN_L3_F(N2, F3)                                                                      \
    if (n_prev == N2 && f == F3) {                                                              \
      SRCNN_PROFILE("conv_fwd_l3_mfma", s);                                                     \
      hipLaunchKernelGGL((l3_fwd_kernel<N2, F3>), dim3(grid), dim3(256), lds, s, in, W, B, out, \
                         (int)in_w, (int)in_h, (int)batch, relu, wo);                           \
      SRCNN_LAUNCH_TRY();                                                                       \
      return 1;                                                                                 \
    }
    SRCNN_N3_SHAPES(SRCNN_L3_F)
#undef SRCNN_L3_F
  }
  return 0;
}

int try_conv_delta(const float* d_next, const float* y_curr, float* d_curr, const float* W_next,
                   uint32_t f_next, uint32_t n_curr, uint32_t n_next, uint32_t curr_w,
                   uint32_t curr_h, uint32_t batch, hipStream_t s) {
  if (int rc = wide::op_conv_delta(d_next, y_curr, d_curr, W_next, f_next, n_curr, n_next, curr_w,
                                   curr_h, batch, s))
    return rc;
  if (f_next == 1) {
    const long long npx = (long long)batch * curr_w * curr_h;
    const uint32_t grid = blocks_for((npx + 15) / 16, kWaves, kGridCap);
#define SRCNN_PW_D(CI, CO)                                                                       \
    if (n_next == CI && n_curr == CO) {                                                          \
      SRCNN_PROFILE("conv_delta_pointwise_mfma", s);                                             \
      hipLaunchKernelGGL((pw_kernel<CI, CO, 1>), dim3(grid), dim3(256), 0, s, d_next, W_next,    \
                         y_curr, d_curr, npx, 0);                                                \
      SRCNN_LAUNCH_TRY();                                                                        \
      return 1;                                                                                  \
    }
    SRCNN_PW_SHAPES(SRCNN_PW_D)
#undef SRCNN_PW_D
    return 0;
  }
  if (n_next == 1) {
    const size_t lds = (size_t)f_next * f_next * n_curr * sizeof(float) + d3_lds(f_next, curr_w, curr_h);
    if (lds > kLdsCap) return 0;
    const uint32_t grid = (uint32_t)std::min<long long>(l1_items((int)curr_w, (int)curr_h, kD3Win, (int)batch), 2048);
#define SRCNN_L3_D(N2, F3)                                                                     \
    if (n_curr == N2 && f_next == F3) {                                                        \
      SRCNN_PROFILE("conv_delta_l3", s);                                                       \
      hipLaunchKernelGGL((l3_delta_kernel<N2, F3>), dim3(grid), dim3(256), lds, s, d_next,     \
                         y_curr, W_next, d_curr, (int)curr_w, (int)curr_h, (int)batch);        \
      SRCNN_LAUNCH_TRY();                                                                      \
      return 1;                                                                                \
    }
    SRCNN_N3_SHAPES(SRCNN_L3_D)
#undef SRCNN_L3_D
  }
  return 0;
}

namespace {
// which gradient kernel serves the shape, and its grid (= slab count)
enum class GradKind { None, Pointwise, L1, L3 };
GradKind grad_kind(uint32_t n_prev, uint32_t n_cur, uint32_t f, uint32_t out_w, uint32_t out_h) {
  if (f == 1) {
#define SRCNN_PW_Q(CI, CO) if (n_prev == CI && n_cur == CO) return GradKind::Pointwise;
    SRCNN_PW_SHAPES(SRCNN_PW_Q)
#undef SRCNN_PW_Q
    return GradKind::None;
  }
  if (n_prev == 1) {  // windowed: any image size
#define SRCNN_L1_Q(N1, F1) if (n_cur == N1 && f == F1) return GradKind::L1;
    SRCNN_N1_SHAPES(SRCNN_L1_Q)
#undef SRCNN_L1_Q
    return GradKind::None;
  }
  if (n_cur == 1 && d3_lds(f, out_w + f - 1, out_h + f - 1) <= kLdsCap) {
#define SRCNN_L3_Q(N2, F3) if (n_prev == N2 && f == F3) return GradKind::L3;
    SRCNN_N3_SHAPES(SRCNN_L3_Q)
#undef SRCNN_L3_Q
  }
  return GradKind::None;
}
uint32_t grad_grid(GradKind k, uint32_t f, uint32_t out_w, uint32_t out_h, uint32_t batch) {
  if (k == GradKind::Pointwise) {
    const long long npx = (long long)batch * out_w * out_h;
    return blocks_for((npx + 7) / 8, 8 * kWaves, kSlabCap);
  }
  // per-window kernels: more resident blocks where registers / LDS allow it
  if (k == GradKind::L1)
    return (uint32_t)std::min<long long>(l1_items((int)out_w, (int)out_h, kXS - (int)f + 1, (int)batch), kSlabCap);
  return (uint32_t)std::min<long long>(
      l1_items((int)(out_w + f - 1), (int)(out_h + f - 1), kD3Win, (int)batch), 4 * kSlabCap);
}
}  // namespace

size_t grad_workspace_bytes(uint32_t n_prev, uint32_t n_cur, uint32_t f, uint32_t out_w,
                            uint32_t out_h, uint32_t batch) {
  if (size_t b = wide::op_grad_workspace_bytes(n_prev, n_cur, f, out_w, out_h, batch)) return b;
  const GradKind k = grad_kind(n_prev, n_cur, f, out_w, out_h);
  if (k == GradKind::None) return 0;
  const size_t P = (size_t)f * f * n_prev * n_cur + n_cur;
  return (size_t)grad_grid(k, f, out_w, out_h, batch) * P * sizeof(float);
}

int try_conv_grad_acc(const float* in, const float* d, float* gW, float* gB, uint32_t n_prev,
                      uint32_t n_cur, uint32_t f, uint32_t out_w, uint32_t out_h, uint32_t batch,
                      void* ws, size_t ws_bytes, hipStream_t s) {
  if (int rc = wide::op_conv_grad_acc(in, d, gW, gB, n_prev, n_cur, f, out_w, out_h, batch, ws,
                                      ws_bytes, s))
    return rc;
  const GradKind k = grad_kind(n_prev, n_cur, f, out_w, out_h);
  if (k == GradKind::None) return 0;
  const uint32_t grid = grad_grid(k, f, out_w, out_h, batch);
  const int nW = (int)(f * f * n_prev * n_cur), nB = (int)n_cur;
  const size_t need = (size_t)grid * (nW + nB) * sizeof(float);
  if (ws_bytes < need)
    return fail(SRCNN_ERR_WORKSPACE, "backpropagate: workspace %zu B < %zu B (srcnn_conv_grad_workspace_bytes)",
                ws_bytes, need);
  float* slab = static_cast<float*>(ws);
  const int in_w = (int)(out_w + f - 1), in_h = (int)(out_h + f - 1);
  bool launched = false;
  if (k == GradKind::Pointwise) {
    const long long npx = (long long)batch * out_w * out_h;
#define SRCNN_PW_G(CI, CO)                                                                     \
    if (!launched && n_prev == CI && n_cur == CO) {                                            \
      SRCNN_PROFILE("grad_pointwise_mfma", s);                                                 \
      hipLaunchKernelGGL((pw_grad_kernel<CI, CO>), dim3(grid), dim3(256), 0, s, in, d, slab, npx); \
      SRCNN_LAUNCH_TRY();                                                                      \
      launched = true;                                                                         \
    }
    SRCNN_PW_SHAPES(SRCNN_PW_G)
#undef SRCNN_PW_G
  } else if (k == GradKind::L1) {
#define SRCNN_L1_G(N1, F1)                                                                     \
    if (!launched && n_cur == N1 && f == F1) {                                                 \
      SRCNN_PROFILE("grad_l1_mfma", s);                                                        \
      hipLaunchKernelGGL((l1_grad_kernel<N1, F1>), dim3(grid), dim3(256), 0, s, in, d, slab,   \
                         in_w, in_h, (int)batch);                                              \
      SRCNN_LAUNCH_TRY();                                                                      \
      launched = true;                                                                         \
    }
    SRCNN_N1_SHAPES(SRCNN_L1_G)
#undef SRCNN_L1_G
  } else {
    const size_t lds = std::max(d3_lds(f, in_w, in_h), (size_t)(2 * 2 * 4 * 64 + 64) * sizeof(float) * 2);
#define SRCNN_L3_G(N2, F3)                                                                     \
    if (!launched && n_prev == N2 && f == F3) {                                                \
      SRCNN_PROFILE("grad_l3_mfma", s);                                                        \
      const size_t l_ = std::max(lds, (size_t)((F3 * F3 + 15) / 16 * (N2 / 16) * 256 + 8) * sizeof(float)); \
      hipLaunchKernelGGL((l3_grad_kernel<N2, F3>), dim3(grid), dim3(256), l_, s, in, d, slab,  \
                         in_w, in_h, (int)batch);                                              \
      SRCNN_LAUNCH_TRY();                                                                      \
      launched = true;                                                                         \
    }
    SRCNN_N3_SHAPES(SRCNN_L3_G)
#undef SRCNN_L3_G
  }
  if (!launched) return 0;
  if (int rc = reduce_rows(slab, (int)grid, nW, nB, gW, gB, s)) return rc;
  return 1;
}

int l1_grad_slabs(const float* X, const float* D1, const float* A1, float* slab, uint32_t n1, uint32_t f1,
                  int w, int h, int batch, int grid, hipStream_t s) {
#define SRCNN_L1_S(N1, F1)                                                                     \
  if (n1 == N1 && f1 == F1) {                                                                  \
    hipLaunchKernelGGL((l1_grad_kernel<N1, F1, true>), dim3(grid), dim3(256), 0, s, X, D1, slab, w, h, batch, A1); \
    SRCNN_LAUNCH_TRY();                                                                        \
    return 1;                                                                                  \
  }
  SRCNN_N1_SHAPES(SRCNN_L1_S)
#undef SRCNN_L1_S
  return 0;
}

}  // namespace fast
}  // namespace srcnn
