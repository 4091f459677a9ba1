// forward_fused.hip -- gfx950 inference (forward only) for SRCNN nets with a
// 1x1 middle layer (f2 == 1), for frames of any size (4K and up).
//
// The reference runs three layer launches with A1 and A2 round-tripping
// through global memory (ConfigBasedDataPipeline.cpp:200-241, kernel
// layer_uber_kernel.cl:36-96).  Here:
//
//   fwd_l123  per 32 x RH region of L1/L2 outputs: L1 (f1 x f1 x 1 -> n1) and
//             L2 (1x1, n1 -> n2) as fp32 MFMA implicit GEMMs, then the L3
//             "Q trick" GEMM  Q[p][tap] = sum_c A2[p][c] * W3[tap][c], and the
//             L3 window sums  sum_tap Q[p + off(tap)][tap]  of every output the
//             region's A2 pixels reach, accumulated in LDS.  Only those partial
//             output sums ((32 + f3 - 1) x (RH + f3 - 1) floats per region)
//             leave the CU -- A1, A2 and Q never reach HBM.
//   fwd_seam  per output pixel: A3 = B3 + the partial sums of the (at most
//             2 x 2) regions whose A2 it reads, in a fixed order (no ReLU:
//             SKIP_RELU), so the result is deterministic.
//
// A region chunk is one region row of 32 pixels.  Rows / columns past the
// frame are computed on zero-padded inputs; they only reach outputs past the
// frame, which are never stored.  Each (tap row dy, partial row) pair of the
// LDS accumulator is written by exactly one chunk, so no atomics are needed.
#include "common.hpp"
#include "mfma.hpp"
#include "ops.hpp"
#include "split.hpp"

namespace srcnn {
namespace fused {

using mfma::crow;
using mfma::f32x16;
using mfma::mma;
using mfma::zero16;

// held-clock probe slot (common.hpp) of fwd_l123
__device__ unsigned long long g_clk_fwd[1][kClockBlocks][2];

namespace {

constexpr int kFwdRW = 32;        // region width (one chunk per region row)
constexpr int kFwdPD = 4;      // L1 X-gather prefetch distance (k-steps), pinned by sched barriers
constexpr int kFwdGrid = 2048;  // grid cap (blocks)

// diagnostics builds only (results invalid): 1 drop the per-chunk L3 window
// sums, 2 drop the per-region partial-sum output, 4 drop the ReLUs, 8 drop the
// next region's register-staged input loads
constexpr int kFwdRhMax = 28;  // region rows (LDS partial-sum accumulator bound)
constexpr int kFwdXs = (kFwdRhMax + 12) * 40;  // input tile floats staged in LDS (f1 <= 9)

struct FwdGeom {
  int W, H;      // input frame
  int ow, oh;    // L1 / L2 output
  int rh;        // region rows
  int nrx, nry;  // regions per frame
  int batch;
};

template <int N1, int N2, int F1, int F3>
__global__ __launch_bounds__(256, 2) void fwd_l123_kernel(
    const float* __restrict__ X, const float* __restrict__ W1, const float* __restrict__ B1,
    const float* __restrict__ W2, const float* __restrict__ B2, const float* __restrict__ W3,
    float* __restrict__ part, FwdGeom g) {
  constexpr int K1 = F1 * F1, KS1 = (K1 + 1) / 2, NT1 = N1 / 32;
  constexpr int K3 = F3 * F3;
  constexpr int TW = kFwdRW + F1 - 1;  // LDS row stride of the input tile
  constexpr int EW = kFwdRW + F3 - 1;  // partial-sum window width
  constexpr int EHM = kFwdRhMax + F3 - 1;
  static_assert(K3 <= 32 && N2 <= 32 && N2 % 2 == 0 && K1 % 2 == 1, "Q tile shape");
  __shared__ float xs[kFwdXs];
  // L2 bias as the accumulator's initial value: register r of half h is
  // channel crow(r, h) (one 16x32 image, read as 4 broadcast 16-B loads)
  // instead of one more MFMA (b2 x 1) per chunk; the same fp32 values
  __shared__ __attribute__((aligned(16))) float b2i[2][16];
  // per-wave Q^T[tap][pixel + F3-1]: F3-1 zero columns either side, so a
  // window sum reads its F3 taps without bounds tests.  Row stride 52 floats
  // (5 x 52 = 4 mod 32): the window-sum items (dy, e) of one ds_read_b32 fall
  // in consecutive banks.  (Round 3 held Q as [pixel][tap] at stride 36 with
  // float4 stores; its window-sum reads were 4-way bank conflicted: same-box
  // A/B, 4 pairs, the frame 0.4-1.0% faster this way, profiles/r04_ab_fwdq.)
  constexpr int QR = kFwdRW + 2 * (F3 - 1);
  constexpr int QTS = 52;
  static_assert(QR <= QTS, "Q^T row");
  __shared__ __attribute__((aligned(16))) float qs[4][32][QTS];
  __shared__ float accs[F3][EHM][EW];  // [dy][partial row][partial col]

  SRCNN_CLOCK_BEGIN();
  const int lane = mfma::lane_id(), wave = mfma::wave_id();
  const int h = lane >> 5, li = lane & 31;
  const int EH = g.rh + F3 - 1;
  for (int i = threadIdx.x; i < 4 * 32 * 2 * (F3 - 1); i += 256) {  // the zero columns (never written again)
    const int w = i / (64 * (F3 - 1)), r = (i / (2 * (F3 - 1))) % 32, col = i % (2 * (F3 - 1));
    qs[w][r][col < F3 - 1 ? col : kFwdRW + col] = 0.0f;
  }
  // L3 window sums: this lane's items k of the F3 x EW (tap row dy, column e)
  // per chunk, as a base into the wave's Q image (taps dx follow at a stride
  // of QS + 1 floats) and into the partial-sum accumulator (+ chunk row c * EW)
  constexpr int kWin = (F3 * EW + 63) / 64;
  int wrb[kWin], wwb[kWin];
#pragma unroll
  for (int k = 0; k < kWin; k++) {
    const int it = min(lane + 64 * k, F3 * EW - 1), dy = it / EW, e = it - dy * EW;
    wrb[k] = (wave * 32 + dy * F3) * QTS + e;
    wwb[k] = (dy * EHM + F3 - 1 - dy) * EW + e;
  }

  // All three GEMMs run TRANSPOSED (rows = channels / taps, cols = the
  // chunk's 32 pixels), so each layer's accumulator registers are the next
  // layer's B operand as they stand (register s of half h is row crow(s, h),
  // mfma.hpp) -- no LDS transposes between L1, L2 and Q:
  //   A operands: W1[tap = 2s+h][ch = 32t+li] (tap K1 = the bias slot, X = 1),
  //               W2[c = 32t + crow(s,h)][n = li] (+ one bias MFMA),
  //               W3[tap = li][c = crow(s,h)]
  float w1f[KS1][NT1];
#pragma unroll
  for (int s = 0; s < KS1; s++)
#pragma unroll
    for (int t = 0; t < NT1; t++) {
      const int tap = 2 * s + h;
      w1f[s][t] = tap < K1 ? W1[tap * N1 + 32 * t + li] : B1[32 * t + li];
    }
  float w2f[NT1][16];
#pragma unroll
  for (int t = 0; t < NT1; t++)
#pragma unroll
    for (int s = 0; s < 16; s++) w2f[t][s] = li < N2 ? W2[(32 * t + crow(s, h)) * N2 + li] : 0.0f;
  if (threadIdx.x < 32) {
    const int c_ = crow(threadIdx.x & 15, threadIdx.x >> 4);
    b2i[threadIdx.x >> 4][threadIdx.x & 15] = c_ < N2 ? B2[c_] : 0.0f;
  }
  float w3f[16];
#pragma unroll
  for (int s = 0; s < 16; s++) {
    const int cc = crow(s, h);
    w3f[s] = (li < K3 && cc < N2) ? W3[li * N2 + cc] : 0.0f;
  }

  const int per_frame = g.nrx * g.nry;
  const int n_items = g.batch * per_frame;
  // The next region's input tile is register-staged while this region's
  // chunks run (its loads retire under the MFMAs instead of stalling the
  // block between regions); rows / columns past the frame read as 0.
  constexpr int kXR = (kFwdXs + 255) / 256;
  float xr[kXR];
  auto xload = [&](int wi) {
    const int n = wi / per_frame, rr = wi - n * per_frame;
    const int ry = rr / g.nrx, rx = rr - ry * g.nrx;
    const int oy0 = ry * g.rh, ox0 = rx * kFwdRW;
    const int th = min(g.rh, g.oh - oy0) + F1 - 1, tw = min(kFwdRW, g.ow - ox0) + F1 - 1;
    const float* xsrc = X + (size_t)n * g.W * g.H + (size_t)oy0 * g.W + ox0;
#pragma unroll
    for (int k = 0; k < kXR; k++) {
      const int i = threadIdx.x + 256 * k;
      const int iy = i / TW, ix = i - iy * TW;
      xr[k] = (i < th * TW && ix < tw) ? xsrc[(size_t)iy * g.W + ix] : 0.0f;
    }
  };
  if ((int)blockIdx.x < n_items) xload(blockIdx.x);
  for (int wi = blockIdx.x; wi < n_items; wi += gridDim.x) {
    const int n = wi / per_frame, rr = wi - n * per_frame;
    const int ry = rr / g.nrx;
    const int oy0 = ry * g.rh;
    const int crh = min(g.rh, g.oh - oy0);

    __syncthreads();  // the previous region's readers are done with xs / accs
#pragma unroll
    for (int k = 0; k < kXR; k++) {
      const int i = threadIdx.x + 256 * k;
      if (i < kFwdXs) xs[i] = xr[k];
    }
    __syncthreads();
    if (wi + (int)gridDim.x < n_items) xload(wi + gridDim.x);

    // The L3 window sums of a chunk run inside this wave's NEXT chunk's L1
    // MFMA stream (its Q^T stays in the wave's scratch until that chunk's own
    // Q overwrites it): read at k-steps kWinS + kWinD k, summed and stored
    // kWinD / 2 steps later.  Issued after the Q MFMAs they were a ~500-cycle
    // LDS / VALU tail per chunk with no MFMA of this wave behind it.
    constexpr int kWinS = 2, kWinD = (KS1 - kWinS - 4) / kWin;
    static_assert(kWinD >= 2 && kWinS + kWinD * kWin + kWinD / 2 < KS1, "window sums fit the L1 stream");
    auto win_read = [&](int k, float* v) {
      const float* qr = &qs[0][0][0] + wrb[k];
#pragma unroll
      for (int dx = 0; dx < F3; dx++) v[dx] = qr[dx * (QTS + 1)];
    };
    auto win_store = [&](int k, const float* v, int pc) {
      if (k < kWin - 1 || lane + 64 * k < F3 * EW) {
        float t = 0.0f;
#pragma unroll
        for (int dx = 0; dx < F3; dx++) t += v[dx];
        (&accs[0][0][0])[wwb[k] + pc * EW] = t;
      }
    };
    int pc = -1;  // this wave's chunk whose window sums are pending (wave-uniform)
    float wv_last[F3];
    for (int c = wave; c < crh; c += 4) {  // chunk = region row c, pixel li
      // tap 2s+1 sits 1 or TW - F1 + 1 floats past tap 2s: two per-half bases,
      // every gather is base + immediate
      const int xbA = c * TW + li + h, xbB = xbA + h * (TW - F1);
      f32x16 acc1[NT1];
#pragma unroll
      for (int t = 0; t < NT1; t++) acc1[t] = zero16();
      // B operand of k-step s (tap K1 = the bias slot)
      auto xg = [&](int s) {
        const int k0 = 2 * s;
        const int o0 = (k0 / F1) * TW + (k0 % F1);
        const float v = xs[((k0 % F1) + 1 < F1 ? xbA : xbB) + o0];
        return s == KS1 - 1 ? (h ? 1.0f : v) : v;
      };
      // gathers run kFwdPD k-steps ahead of their MFMAs, pinned by sched
      // barriers: left alone, the scheduler issues each one just before its
      // MFMA pair and the wave waits out the full LDS latency every step
      float xq[KS1];
      float wv[F3];
#pragma unroll
      for (int s = 0; s < kFwdPD && s < KS1; s++) xq[s] = xg(s);
#pragma unroll
      for (int s = 0; s < KS1; s++) {
        if (s + kFwdPD < KS1) xq[s + kFwdPD] = xg(s + kFwdPD);
        if (pc >= 0 && s >= kWinS && (s - kWinS) % kWinD == 0 && (s - kWinS) / kWinD < kWin)
          win_read((s - kWinS) / kWinD, wv);
        __builtin_amdgcn_sched_barrier(0);
        const float xv = xq[s];
#pragma unroll
        for (int t = 0; t < NT1; t++) acc1[t] = mma(w1f[s][t], xv, acc1[t]);
        if (pc >= 0 && s >= kWinS + kWinD / 2 && (s - kWinS - kWinD / 2) % kWinD == 0 &&
            (s - kWinS - kWinD / 2) / kWinD < kWin)
          win_store((s - kWinS - kWinD / 2) / kWinD, wv, pc);
        __builtin_amdgcn_sched_barrier(0);
      }
      // L1 ReLU (layer_uber_kernel.cl:88-95; bias already in)
#pragma unroll
      for (int t = 0; t < NT1; t++)
#pragma unroll
        for (int r = 0; r < 16; r++)
          acc1[t][r] = fmaxf(acc1[t][r], 0.0f);
      // L2^T: A2^T[n][p] = B2[n] + sum_c W2[c][n] A1^T[c][p], then ReLU
      f32x16 acc2;
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const mfma::f32x4 v_ = *reinterpret_cast<const mfma::f32x4*>(&b2i[h][4 * q]);
#pragma unroll
        for (int e = 0; e < 4; e++) acc2[4 * q + e] = v_[e];
      }
#pragma unroll
      for (int t = 0; t < NT1; t++)
#pragma unroll
        for (int s = 0; s < 16; s++) acc2 = mma(w2f[t][s], acc1[t][s], acc2);
#pragma unroll
      for (int r = 0; r < 16; r++)
        acc2[r] = fmaxf(acc2[r], 0.0f);
      // Q^T[tap][p] = sum_c W3[tap][c] A2^T[c][p]
      f32x16 accq = zero16();
#pragma unroll
      for (int s = 0; s < 16; s++) accq = mma(w3f[s], acc2[s], accq);
      // Q^T[taps crow(r, h)][pixel li]: 16 rows per lane, lanes consecutive
      // (the pending window sums above read the previous Q^T: their values
      // are summed, so those reads have completed)
#pragma unroll
      for (int r = 0; r < 16; r++) qs[wave][crow(r, h)][li + F3 - 1] = accq[r];
      __builtin_amdgcn_wave_barrier();
      pc = c;
    }
    // tap row dy of a chunk feeds partial row c + F3 - 1 - dy:
    //   accs[dy][c + F3-1 - dy][e] = sum_dx Q[e - (F3-1) + dx][dy*F3 + dx]
    //   (Q row e + dx of the padded image is pixel e - (F3-1) + dx)
    // here the window sums of this wave's last chunk
    if (pc >= 0) {
#pragma unroll
      for (int k = 0; k < kWin; k++) {
        win_read(k, wv_last);
        win_store(k, wv_last, pc);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __syncthreads();
    // partial row pr gets tap rows dy whose chunk c = pr - (F3-1) + dy exists
    float* dst = part + (size_t)wi * EH * EW;
    for (int i = threadIdx.x; i < EH * EW; i += 256) {
      const int pr = i / EW, e = i - pr * EW;
      float v = 0.0f;
#pragma unroll
      for (int dy = 0; dy < F3; dy++) {
        const int c = pr - (F3 - 1) + dy;
        if (c >= 0 && c < crh) v += accs[dy][pr][e];
      }
      dst[i] = v;
    }
  }
  SRCNN_CLOCK_END(g_clk_fwd, 0);
}


// ---------------------------------------------------------------------------
// fwd_l123x6: fwd_l123 for the reference default net (64/32/9/5) with its
// three GEMMs in split-bf16 products (split.hpp; l12x6.hpp in
// train_fused.hip has the same L1 / L2 operand scheme):
//   L1^T  80 taps in 5 bf16 k-steps (slot 8h + j of k-step s: tap (2s+h, j)
//         for 2s+h <= 8, tap (j, 8) for the last half-step), B operand from
//         part-interleaved pair images of the region's input tile (rows
//         2s + h: two ds_read2_b32 per part), tap (8, 8) and B1 in one fp32
//         32x32x2 MFMA that starts the accumulator
//   L2^T  the ReLU'd L1 accumulator split in registers against W2 images
//   Q^T   the ReLU'd L2 accumulator split against W3 images (2 k-steps)
// Eight waves share one block (and the 48 KB of split weight images) per
// CU, two per SIMD; a region is 24 rows (3 chunks per wave).
constexpr int kF6Waves = 8;
constexpr int kF6Rh = 24;              // region rows
constexpr int kF6TW = kFwdRW + 8;      // input tile row stride (f1 = 9)
constexpr int kF6XR = kF6Rh + 8;       // input tile rows
constexpr int kF6QS = 41;              // Q^T row stride (32 + 2 (f3 - 1) columns)
constexpr int kF6W1 = 5 * 2 * 3 * 512; // bf16: [s][t][part][lane][8]
constexpr int kF6W2 = 4 * 3 * 512;     // bf16: [m][part][lane][8]
constexpr int kF6W3 = 2 * 3 * 512;     // bf16: [m][part][lane][8]
struct F6Lds {
  static constexpr int w1 = 0, w2 = w1 + kF6W1 * 2, w3 = w2 + kF6W2 * 2, a88 = w3 + kF6W3 * 2,
                       b2 = a88 + 128 * 4, r = b2 + 32 * 4,
                       rn = kF6TW * kF6XR + 1,  // pair-image dwords per part
                       xs = r + 3 * rn * 4, qs = (xs + kF6TW * kF6XR * 4 + 15) & ~15,
                       accs = qs + kF6Waves * 25 * kF6QS * 4, bytes = accs + 5 * (kF6Rh + 4) * (kFwdRW + 4) * 4;
};

__global__ __launch_bounds__(512, 1) void fwd_l123x6_kernel(
    const float* __restrict__ X, const float* __restrict__ W1, const float* __restrict__ B1,
    const float* __restrict__ W2, const float* __restrict__ B2, const float* __restrict__ W3,
    float* __restrict__ part, FwdGeom g) {
  using mfma::bf16x8;
  using mfma::mma_x6;
  using mfma::relu1;
  using mfma::split3;
  using mfma::split8;
  using mfma::u32x4;
  constexpr int N1 = 64, N2 = 32, F1 = 9, F3 = 5, K3 = F3 * F3, NT1 = 2;
  constexpr int TW = kF6TW, EW = kFwdRW + F3 - 1, EHM = kF6Rh + F3 - 1;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  char* const base = reinterpret_cast<char*>(smem);
  __bf16* const w1i = reinterpret_cast<__bf16*>(base + F6Lds::w1);
  __bf16* const w2i = reinterpret_cast<__bf16*>(base + F6Lds::w2);
  __bf16* const w3i = reinterpret_cast<__bf16*>(base + F6Lds::w3);
  float* const a88s = reinterpret_cast<float*>(base + F6Lds::a88);
  float* const b2i = reinterpret_cast<float*>(base + F6Lds::b2);
  uint32_t* const rimg = reinterpret_cast<uint32_t*>(base + F6Lds::r);
  float* const xs = reinterpret_cast<float*>(base + F6Lds::xs);
  float* const qs = reinterpret_cast<float*>(base + F6Lds::qs);
  float* const accs = reinterpret_cast<float*>(base + F6Lds::accs);
  constexpr int rn = F6Lds::rn;

  SRCNN_CLOCK_BEGIN();
  const int lane = mfma::lane_id(), wave = mfma::wave_id();
  const int h = lane >> 5, li = lane & 31;
  const int EH = g.rh + F3 - 1;
  const int per_frame = g.nrx * g.nry;
  const int n_items = g.batch * per_frame;
  constexpr int kXR = (TW * kF6XR + 511) / 512;
  float xr[kXR];
  auto xload = [&](int wi) {
    const int n = wi / per_frame, rr = wi - n * per_frame;
    const int ry = rr / g.nrx, rx = rr - ry * g.nrx;
    const int oy0 = ry * g.rh, ox0 = rx * kFwdRW;
    const int th = min(g.rh, g.oh - oy0) + F1 - 1, tw = min(kFwdRW, g.ow - ox0) + F1 - 1;
    const float* xsrc = X + (size_t)n * g.W * g.H + (size_t)oy0 * g.W + ox0;
#pragma unroll
    for (int k = 0; k < kXR; k++) {
      const int i = threadIdx.x + 512 * k;
      const int iy = i / TW, ix = i - iy * TW;
      xr[k] = (i < th * TW && ix < tw) ? xsrc[(size_t)iy * g.W + ix] : 0.0f;
    }
  };
  if ((int)blockIdx.x < n_items) xload(blockIdx.x);

  // ---- split weight images ----
  for (int e = threadIdx.x; e < 5 * 2 * 64 * 8; e += 512) {
    const int j = e & 7, L_ = (e >> 3) & 63, t = (e >> 9) & 1, s_ = e >> 10;
    const int gg = 2 * s_ + (L_ >> 5);
    const int tap = gg <= 8 ? gg * F1 + j : j * F1 + 8;
    __bf16 p[3];
    split3(W1[tap * N1 + 32 * t + (L_ & 31)], p[0], p[1], p[2]);
#pragma unroll
    for (int q = 0; q < 3; q++) w1i[((s_ * 2 + t) * 3 + q) * 512 + L_ * 8 + j] = p[q];
  }
  for (int e = threadIdx.x; e < 4 * 64 * 8; e += 512) {
    const int j = e & 7, L_ = (e >> 3) & 63, m = e >> 9;
    const int c = 32 * (m >> 1) + crow(8 * (m & 1) + j, L_ >> 5);
    __bf16 p[3];
    split3(W2[c * N2 + (L_ & 31)], p[0], p[1], p[2]);
#pragma unroll
    for (int q = 0; q < 3; q++) w2i[(m * 3 + q) * 512 + L_ * 8 + j] = p[q];
  }
  for (int e = threadIdx.x; e < 2 * 64 * 8; e += 512) {
    // Q^T A operand: lane (tap, h), k-step m, element j <-> channel crow(8m + j, h)
    const int j = e & 7, L_ = (e >> 3) & 63, m = e >> 9;
    const int tap = L_ & 31, c = crow(8 * m + j, L_ >> 5);
    __bf16 p[3];
    split3(tap < K3 ? W3[tap * N2 + c] : 0.0f, p[0], p[1], p[2]);
#pragma unroll
    for (int q = 0; q < 3; q++) w3i[(m * 3 + q) * 512 + L_ * 8 + j] = p[q];
  }
  if (threadIdx.x < 128)
    a88s[threadIdx.x] = threadIdx.x < 64 ? W1[80 * N1 + threadIdx.x] : B1[threadIdx.x - 64];
  else if (threadIdx.x < 160)
    b2i[threadIdx.x - 128] = B2[crow((threadIdx.x - 128) & 15, (threadIdx.x - 128) >> 4)];
  // Q^T zero columns (never written again)
  for (int i = threadIdx.x; i < kF6Waves * 25 * 2 * (F3 - 1); i += 512) {
    const int w = i / (50 * (F3 - 1)), r = (i / (2 * (F3 - 1))) % 25, col = i % (2 * (F3 - 1));
    qs[(w * 25 + r) * kF6QS + (col < F3 - 1 ? col : kFwdRW + col)] = 0.0f;
  }
  __syncthreads();
  float a88r[NT1];
#pragma unroll
  for (int t = 0; t < NT1; t++) a88r[t] = a88s[64 * h + 32 * t + li];

  // L3 window sums (fwd_l123): item k of the F3 x EW (tap row dy, column e) per chunk
  constexpr int kWin = (F3 * EW + 63) / 64;
  int wrb[kWin], wwb[kWin];
#pragma unroll
  for (int k = 0; k < kWin; k++) {
    const int it = min(lane + 64 * k, F3 * EW - 1), dy = it / EW, e = it - dy * EW;
    wrb[k] = (wave * 25 + dy * F3) * kF6QS + e;
    wwb[k] = (dy * EHM + F3 - 1 - dy) * EW + e;
  }
  auto win_read = [&](int k, float* v) {
#pragma unroll
    for (int dx = 0; dx < F3; dx++) v[dx] = qs[wrb[k] + dx * (kF6QS + 1)];
  };
  auto win_store = [&](int k, const float* v, int pc) {
    if (k < kWin - 1 || lane + 64 * k < F3 * EW) {
      float t = 0.0f;
#pragma unroll
      for (int dx = 0; dx < F3; dx++) t += v[dx];
      accs[wwb[k] + pc * EW] = t;
    }
  };

  const uint16_t* const wl1 = reinterpret_cast<const uint16_t*>(w1i) + lane * 8;
  const uint16_t* const wl2 = reinterpret_cast<const uint16_t*>(w2i) + lane * 8;
  const uint16_t* const wl3 = reinterpret_cast<const uint16_t*>(w3i) + lane * 8;
  auto w1op = [&](int s_, int t, bf16x8 (&a)[3]) {
#pragma unroll
    for (int q = 0; q < 3; q++) a[q] = *reinterpret_cast<const bf16x8*>(wl1 + ((s_ * 2 + t) * 3 + q) * 512);
  };

  for (int wi = blockIdx.x; wi < n_items; wi += gridDim.x) {
    const int n = wi / per_frame, rr = wi - n * per_frame;
    const int ry = rr / g.nrx;
    const int oy0 = ry * g.rh;
    const int crh = min(g.rh, g.oh - oy0);

    __syncthreads();  // the previous region's readers are done with the images / accs
    {
      uint16_t* const r16 = reinterpret_cast<uint16_t*>(rimg);
#pragma unroll
      for (int k = 0; k < kXR; k++) {
        const int i = threadIdx.x + 512 * k;
        if (i < TW * kF6XR) {
          xs[i] = xr[k];
          __bf16 p[3];
          split3(xr[k], p[0], p[1], p[2]);
#pragma unroll
          for (int q = 0; q < 3; q++) {
            const uint16_t b = __builtin_bit_cast(uint16_t, p[q]);
            r16[2 * (q * rn + i)] = b;
            if (i > 0) r16[2 * (q * rn + i) - 1] = b;
          }
        }
      }
    }
    __syncthreads();
    if (wi + (int)gridDim.x < n_items) xload(wi + gridDim.x);

    int pc = -1;  // this wave's chunk whose window sums are pending (wave-uniform)
    float wv[F3];
    for (int c = wave; c < crh; c += kF6Waves) {  // chunk = region row c, pixel li
      const int rb = (c + h) * TW + li;
      const int b4 = h ? c * TW + li + 8 : (c + 8) * TW + li, st4 = h ? TW : 1;
      f32x16 acc1[NT1];
      {
        const float bx = h ? 1.0f : xs[(c + 8) * TW + li + 8];
#pragma unroll
        for (int t = 0; t < NT1; t++) acc1[t] = mma(a88r[t], bx, zero16());
      }
      auto xop = [&](int s_, bf16x8 (&b)[3]) {
#pragma unroll
        for (int q = 0; q < 3; q++) {
          const uint32_t* r = rimg + q * rn + rb + 2 * s_ * TW;
          u32x4 d;
          d[0] = r[0];
          d[1] = r[2];
          d[2] = r[4];
          d[3] = r[6];
          b[q] = __builtin_bit_cast(bf16x8, d);
        }
      };
      bf16x8 wa[2][3], xb[2][3];
      float x4[8];
      xop(0, xb[0]);
      w1op(0, 0, wa[0]);
#pragma unroll
      for (int gi = 0; gi < 10; gi++) {
        const int s_ = gi >> 1, t = gi & 1;
        if (gi + 1 < 10) w1op((gi + 1) >> 1, (gi + 1) & 1, wa[(gi + 1) & 1]);
        if (t == 0 && s_ + 1 < 4) xop(s_ + 1, xb[(s_ + 1) & 1]);
        if (gi == 4) {
#pragma unroll
          for (int j = 0; j < 8; j++) x4[j] = xs[b4 + j * st4];
        }
        if (gi == 6) split8(x4, xb[0]);
        // the previous chunk's window sums ride in this stream
        if (pc >= 0 && (gi & 1) && (gi >> 1) < kWin) win_read(gi >> 1, wv);
        __builtin_amdgcn_sched_barrier(0);
        acc1[t] = mma_x6(wa[gi & 1], xb[s_ & 1], acc1[t]);
        if (pc >= 0 && gi >= 2 && !(gi & 1) && (gi >> 1) - 1 < kWin) win_store((gi >> 1) - 1, wv, pc);
        __builtin_amdgcn_sched_barrier(0);
      }
#pragma unroll
      for (int t = 0; t < NT1; t++)
#pragma unroll
        for (int r = 0; r < 16; r++) acc1[t][r] = relu1(acc1[t][r]);
      f32x16 acc2;
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const mfma::f32x4 v_ = *reinterpret_cast<const mfma::f32x4*>(&b2i[16 * h + 4 * q]);
#pragma unroll
        for (int e = 0; e < 4; e++) acc2[4 * q + e] = v_[e];
      }
      auto opsplit = [&](const f32x16& acc, int m, bf16x8 (&b)[3]) {
        float v[8];
#pragma unroll
        for (int j = 0; j < 8; j++) v[j] = acc[8 * (m & 1) + j];
        split8(v, b);
      };
      bf16x8 wb[2][3], bb[2][3];
      auto wop = [&](const uint16_t* wl, int m, bf16x8 (&a)[3]) {
#pragma unroll
        for (int q = 0; q < 3; q++) a[q] = *reinterpret_cast<const bf16x8*>(wl + (m * 3 + q) * 512);
      };
      wop(wl2, 0, wb[0]);
      opsplit(acc1[0], 0, bb[0]);
#pragma unroll
      for (int m = 0; m < 4; m++) {
        if (m + 1 < 4) wop(wl2, m + 1, wb[(m + 1) & 1]);
        __builtin_amdgcn_sched_barrier(0);
        acc2 = mma_x6(wb[m & 1], bb[m & 1], acc2);
        if (m + 1 < 4) opsplit(acc1[(m + 1) >> 1], m + 1, bb[(m + 1) & 1]);
        __builtin_amdgcn_sched_barrier(0);
      }
#pragma unroll
      for (int r = 0; r < 16; r++) acc2[r] = relu1(acc2[r]);
      // Q^T[tap][p] = sum_c W3[tap][c] A2^T[c][p]
      f32x16 accq = zero16();
      wop(wl3, 0, wb[0]);
      opsplit(acc2, 0, bb[0]);
#pragma unroll
      for (int m = 0; m < 2; m++) {
        if (m + 1 < 2) {
          wop(wl3, 1, wb[1]);
          opsplit(acc2, 1, bb[1]);
        }
        accq = mma_x6(wb[m], bb[m], accq);
      }
      // Q^T rows (taps) crow(r, h) < 25 of pixel li (the pending window sums
      // above read the previous Q^T: their values are summed by now)
#pragma unroll
      for (int r = 0; r < 16; r++)
        if (crow(r, h) < K3) qs[(wave * 25 + crow(r, h)) * kF6QS + li + F3 - 1] = accq[r];
      __builtin_amdgcn_wave_barrier();
      pc = c;
    }
    if (pc >= 0) {
#pragma unroll
      for (int k = 0; k < kWin; k++) {
        win_read(k, wv);
        win_store(k, wv, pc);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __syncthreads();
    float* dst = part + (size_t)wi * EH * EW;
    for (int i = threadIdx.x; i < EH * EW; i += 512) {
      const int pr = i / EW, e = i - pr * EW;
      float v = 0.0f;
#pragma unroll
      for (int dy = 0; dy < F3; dy++) {
        const int c = pr - (F3 - 1) + dy;
        if (c >= 0 && c < crh) v += accs[(dy * EHM + pr) * EW + e];
      }
      dst[i] = v;
    }
  }
  SRCNN_CLOCK_END(g_clk_fwd, 0);
}

// A3[y][x] = B3 + the partials of the regions (ry, rx) in {y, y+f3-1}/rh x
// {x, x+f3-1}/32 (ConfigBasedDataPipeline.cpp:224-238, last layer: no ReLU).
// Grid (columns / blockDim.x, rows, frames): the row's region range is block
// uniform, a thread's column range a shift, and consecutive threads read
// consecutive partials (the 64-bit index division of a flat grid-stride loop
// cost more than the memory traffic).
template <int F3>
__global__ __launch_bounds__(256) void fwd_seam_kernel(const float* __restrict__ part,
                                                       const float* __restrict__ B3,
                                                       float* __restrict__ out, FwdGeom g, int rb) {
  constexpr int EW = kFwdRW + F3 - 1;
  const int w3 = g.ow - F3 + 1, h3 = g.oh - F3 + 1;
  const int EH = g.rh + F3 - 1;
  const float b3 = B3[0];
  const int x = blockIdx.x * blockDim.x + threadIdx.x;
  if (x >= w3) return;
  const int rxa = x / kFwdRW, rxb = (x + F3 - 1) / kFwdRW;
  for (int n = blockIdx.z; n < g.batch; n += gridDim.z) {
    // rows [rb * blockIdx.y, +rb), then grid-strided
    for (int y = rb * blockIdx.y; y < h3; y += (y % rb == rb - 1) ? rb * (gridDim.y - 1) + 1 : 1) {
      const int rya = y / g.rh, ryb = (y + F3 - 1) / g.rh;
      const size_t fbase = (size_t)n * g.nry * g.nrx;
      float v = 0.0f;
      for (int ry = rya; ry <= ryb; ry++) {
        const int pr = y - ry * g.rh + F3 - 1;
        for (int rx = rxa; rx <= rxb; rx++) {
          const int e = x - rx * kFwdRW + F3 - 1;
          v += part[((fbase + (size_t)ry * g.nrx + rx) * EH + pr) * EW + e];
        }
      }
      out[((size_t)n * h3 + y) * w3 + x] = v + b3;
    }
  }
}

template <int N1, int N2, int F1, int F3>
int run_forward(const float* X, uint32_t w, uint32_t h, uint32_t batch, const float* params,
                float* out, void* ws, size_t ws_bytes, hipStream_t s, bool query_only,
                size_t* need) {
  const int ow = (int)w - F1 + 1, oh = (int)h - F1 + 1;
  if (ow < F3 || oh < F3) return 0;
  // the default net in split-bf16 products (fwd_l123x6), fixed 24-row regions
  const bool x6 = N1 == 64 && N2 == 32 && F1 == 9 && F3 == 5 && g_arith == 0;
  // region rows: the input tile (32 + f1 - 1) x (rh + f1 - 1) fits the LDS tile,
  // a multiple of the 4 waves
  int rh = x6 ? kF6Rh : std::min((kFwdXs / (kFwdRW + F1 - 1) - (F1 - 1)) / 4 * 4, kFwdRhMax / 4 * 4);
  if (rh < F3) return 0;
  rh = std::min(rh, oh);
  FwdGeom g{(int)w, (int)h, ow, oh, rh, (ow + kFwdRW - 1) / kFwdRW, (oh + rh - 1) / rh, (int)batch};
  const long items = (long)g.batch * g.nrx * g.nry;
  // partial sums of either arithmetic's regions (srcnn_set_arith between the
  // size query and the call needs no new query)
  auto part_bytes = [&](int r) {
    return (size_t)g.batch * g.nrx * ((oh + r - 1) / r) * (r + F3 - 1) * (kFwdRW + F3 - 1) * sizeof(float);
  };
  size_t pbytes = part_bytes(rh);
  if (N1 == 64 && N2 == 32 && F1 == 9 && F3 == 5) {
    const int rh_f32 = std::min(std::min((kFwdXs / (kFwdRW + F1 - 1) - (F1 - 1)) / 4 * 4, kFwdRhMax / 4 * 4), oh);
    pbytes = std::max({pbytes, part_bytes(rh_f32), part_bytes(std::min(kF6Rh, oh))});
  }
  if (query_only) {
    *need = pbytes;
    return 1;
  }
  if (ws_bytes < pbytes)
    return fail(SRCNN_ERR_WORKSPACE, "fused forward: workspace %zu B < %zu B", ws_bytes, pbytes);
  float* part = static_cast<float*>(ws);
  const float* W1 = params;
  const float* B1 = W1 + F1 * F1 * N1;
  const float* W2 = B1 + N1;
  const float* B2 = W2 + N1 * N2;
  const float* W3 = B2 + N2;
  const float* B3 = W3 + F3 * F3 * N2;
  {
    SRCNN_PROFILE("fwd_l123_mfma", s);
    if (x6) {
      hipError_t e = hipFuncSetAttribute((const void*)fwd_l123x6_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                         160 * 1024);
      if (e != hipSuccess) return fail(SRCNN_ERR_HIP, "hipFuncSetAttribute(fwd_l123x6): %s", hipGetErrorString(e));
      hipLaunchKernelGGL(fwd_l123x6_kernel, dim3((unsigned)std::min<long>(items, 256)), dim3(512), F6Lds::bytes, s,
                         X, W1, B1, W2, B2, W3, part, g);
    } else {
      hipLaunchKernelGGL((fwd_l123_kernel<N1, N2, F1, F3>), dim3((unsigned)std::min<long>(items, kFwdGrid)),
                         dim3(256), 0, s, X, W1, B1, W2, B2, W3, part, g);
    }
    SRCNN_LAUNCH_TRY();
  }
  {
    SRCNN_PROFILE("fwd_l3_seam", s);
    const int w3 = ow - F3 + 1, h3 = oh - F3 + 1;
    const int bx = std::min(256, (w3 + 63) / 64 * 64);
    // up to 8 rows per block while the grid keeps >= 4096 blocks (4K frame:
    // 7 rows, 0.0307 -> 0.0267 ms; small frames: 1 row per block)
    const int nbx = (w3 + bx - 1) / bx;
    const int rb = (int)std::max<long>(1, std::min<long>(8, (long)nbx * h3 * batch / 4096));
    const dim3 grid((unsigned)nbx, (unsigned)std::min((h3 + rb - 1) / rb, 65535),
                    (unsigned)std::min<uint32_t>(batch, 65535));
    hipLaunchKernelGGL((fwd_seam_kernel<F3>), grid, dim3(bx), 0, s, part, B3, out, g, rb);
    SRCNN_LAUNCH_TRY();
  }
  return 1;
}

}  // namespace

int forward_clock(double* ghz) {
  unsigned long long a[1][kClockBlocks][2];
  SRCNN_HIP_TRY(hipMemcpyFromSymbol(a, HIP_SYMBOL(g_clk_fwd), sizeof(a)));
  *ghz = clock_ghz(a[0]);
  return SRCNN_OK;
}

int preload_forward(const srcnn_net* net) {
  if (net->f2 != 1) return 0;
#define SRCNN_FWD_CASE(A, B, C, D)                                                        \
  if (net->n1 == A && net->n2 == B && net->f1 == C && net->f3 == D) {                    \
    const void* k[] = {(const void*)fwd_l123_kernel<A, B, C, D>, (const void*)fwd_seam_kernel<D>, \
                       (const void*)fwd_l123x6_kernel};                                  \
    int rc = resolve_kernels(k, A == 64 && B == 32 ? 3 : 2);                             \
    return rc ? rc : 1;                                                                  \
  }
  SRCNN_FWD_CASE(64, 32, 9, 5)
  SRCNN_FWD_CASE(32, 16, 9, 5)
#undef SRCNN_FWD_CASE
  return 0;
}

int forward(const srcnn_net* net, const float* X, uint32_t w, uint32_t h, uint32_t batch,
            const float* params, float* out, void* ws, size_t ws_bytes, hipStream_t s,
            bool query_only, size_t* need) {
  if (net->f2 != 1) return 0;
#define SRCNN_FWD_CASE(A, B, C, D)                                                       \
  if (net->n1 == A && net->n2 == B && net->f1 == C && net->f3 == D)                     \
    return run_forward<A, B, C, D>(X, w, h, batch, params, out, ws, ws_bytes, s, query_only, need);
  SRCNN_FWD_CASE(64, 32, 9, 5)  // reference default
  SRCNN_FWD_CASE(32, 16, 9, 5)  // example_config.json
#undef SRCNN_FWD_CASE
  return 0;
}

}  // namespace fused
}  // namespace srcnn
