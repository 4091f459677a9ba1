// l3_stream.hpp -- kernel 2 of the fused step (l3) as a pipelined stream of
// 16-pixel units, for n2 = 32, f3 = 5 (the reference default net).  Included
// by train_fused.hip inside namespace srcnn::fused, after d1c.hpp.
//
// Same mathematics as l3_delta_kernel (l3_delta.hpp):
//   L3 forward     layer_uber_kernel.cl:70-91 (SKIP_RELU), as Q = A2 . W3^T
//                  (MFMA) + 25 window sums of Q per output
//   last delta     last_layer_delta.cl:34-48 (relu' quirk on a linear layer)
//   squared error  squared_error.cl:60-69
//   delta2         layer_deltas.cl:79-123 (transposed MFMA over the taps)
//   gW3 / gB3      backpropagate.cl:89-112 (MFMA over the A2 pixels)
// but a different schedule.  l3_delta holds a whole 80 KB A2 tile (two, to
// double-buffer), so one block fills a CU and its HBM traffic comes in
// bursts between barrier-separated phases.  Here a block walks its samples
// as one stream of 16-pixel units (a sample is ceil(npx2 / 16) units; its
// pixel slots past npx2 are zeros), and step k of the stream runs
//   Q      of unit k           (needs A2 unit k)
//   A3     of unit k - L1      (needs Q of units k - L1 .. k - 1)
//   delta2 and gW3 of unit k - L2, L2 = L1 + 1 (need delta3 back to
//          (F3 - 1)(w2 + 1) pixels before the unit, written by A3 stages)
// with L1 = 1 + (15 + (F3 - 1)(w2 + 1)) / 16 (8 for 33x33 tiles).  Only
// small rings stay in LDS (A2 16 units, Q 10 units, delta3 and ground truth
// 256 pixel slots each: 52.7 KB), so three blocks share a CU and their
// stages overlap; the A2 units arrive by LDS-DMA kL3sD steps ahead, delta2
// leaves as one 16-B store per lane per step, so the HBM traffic is a
// steady stream instead of alternating phases.
//
// Waves (one step): w0 / w1 Q tap tile 0 / 1 (8 MFMAs) and the A2 DMA (one
// half unit each); w1 also the ground-truth DMA and the A3 window sums, last
// delta and squared error; w2 / w3 delta2 channel tile 0 / 1 (7 MFMAs) and
// its store, w2 also the A3 store; every wave one gW3 tile (tap tile w >> 1,
// channel tile w & 1: 4 MFMAs), whose accumulator is that wave's share of
// the block's slab, so no cross-wave reduction.  One s_barrier per step; the
// two DMA waves wait for their data with fixed vmcnt counts (each issues the
// same DMAs every step, dummies past the stream's end) and issue no stores,
// which would count in the same in-order counter; never vmcnt(0).
//
// LDS images:
//   A2 unit  [16 px][32 ch], quad q of pixel p at slot q ^ (p & 7): the Q
//            operand (two ds_read_b128 per lane), the delta2 relu' mask (one
//            b128) and the gW3 operand (b32, 16 channels of a pixel per lane
//            group) are bank-conflict free
//   Q        [pixel slot][tap] at stride 28 floats
//   delta3   on the A2 grid (zero where no L3 output is), ring of 256 slots
#pragma once

constexpr int kL3sThreads = 256;
constexpr int kL3sRA = 16;   // A2 ring units (16 pixels x 32 channels, 2 KB each)
constexpr int kL3sD = 5;     // A2 unit k is DMA'd at step k - kL3sD
#ifndef SRCNN_L3S_TD
#define SRCNN_L3S_TD 4
#endif
constexpr int kL3sTD = SRCNN_L3S_TD;  // ground truth of unit a is DMA'd at step a + L1 - kL3sTD (<= L1)
constexpr int kL3sRQ = 160;  // Q ring pixel slots (10 units)
constexpr int kL3sSQ = 28;   // Q slot stride (floats): lane groups 16 banks apart
constexpr int kL3sRD = 256;  // delta3 ring slots (power of two)
constexpr int kL3sRT = 128;  // ground-truth ring slots (power of two, > 16 kL3sTD)
constexpr int kL3sR3 = 128;  // A3 ring slots (A3 of unit a is stored one step after it is formed)
static_assert(kL3sRT / 16 > kL3sTD, "ground-truth ring");
constexpr int kL3sLdsFloats = kL3sRA * 512 + kL3sRQ * kL3sSQ + kL3sRD + kL3sRT + kL3sR3;
constexpr int kL3sBlocksPerCU = 3;
constexpr int kL3sGrid = 256 * kL3sBlocksPerCU;  // all blocks resident

// A3 stores of out-of-range stages go here
__device__ __attribute__((aligned(16))) float g_l3s_sink[64];
#ifdef SRCNN_L3_TIMING
// diagnostics build only: per block and wave, cycles in the top-of-step
// wait + barrier and cycles of the whole step loop
__device__ unsigned long long g_l3s_timing[kL3sGrid][8];
#endif

// A3 lag L1 of a geometry, or 0 if the rings cannot hold the pipeline
inline int l3s_lag(int w2, int h2, int F3) {
  const int offmax = (F3 - 1) * (w2 + 1);
  const int L1 = 1 + (15 + offmax) / 16;
  const int L2 = L1 + 1;
  const bool ok = w2 > 0 && h2 > 0 && (w2 * h2 + 15) / 16 > kL3sD &&  // the prologue's units
                  L1 >= kL3sTD && L1 + 1 <= kL3sRQ / 16 &&          // Q ring: L1 + 1 units
                  L2 + kL3sD + 1 <= kL3sRA &&                       // A2 ring
                  offmax + 32 <= kL3sRD && w2 * h2 < 4096;          // delta3 ring; 20-bit p / w2
  return ok ? L1 : 0;
}

// 4 B per lane from a 64-bit per-lane address into M0 + 4 * lane
__device__ __forceinline__ void l3s_dma4v(const float* src, float* lds_dst) {
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dword %1, off"
               : : "s"(d1c_m0(lds_dst)), "v"(src) : "m0");
}
// 16 B per lane, nontemporal (A2 is read once here)
__device__ __forceinline__ void l3s_dma16v_nt(const float* src, float* lds_dst) {
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt"
               : : "s"(d1c_m0(lds_dst)), "v"(src) : "m0");
}

template <int F3>
__global__ __launch_bounds__(kL3sThreads, kL3sBlocksPerCU) void l3s_kernel(
    const float* __restrict__ A2, const float* __restrict__ T, const float* __restrict__ W3,
    const float* __restrict__ B3, float* __restrict__ D2, float* __restrict__ slab3,
    float* __restrict__ sq_slab, float* __restrict__ A3out, L3Geom g, int L1) {
  constexpr int N2 = 32, K3 = F3 * F3, NW3 = K3 * N2;
  static_assert(K3 <= 28, "delta2 runs 7 k-steps of 4 taps; Q and gW3 two 16-tap tiles");
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* const a2r = smem;                       // [kL3sRA][512]
  float* const qr = a2r + kL3sRA * 512;          // [kL3sRQ][kL3sSQ]
  float* const d3r = qr + kL3sRQ * kL3sSQ;       // [kL3sRD]
  float* const tr = d3r + kL3sRD;                // [kL3sRT]
  float* const a3r = tr + kL3sRT;                // [kL3sR3]
  SRCNN_CLOCK_BEGIN();
  const int lane = mfma::lane_id(), wave = mfma::wave_id();
  const int lq = lane & 15, lg = lane >> 4;
  const int w2 = g.w2, npx2 = g.w2 * g.h2, nout = g.w3 * g.h3;
  const int U = (npx2 + 15) / 16;                 // units per sample
  const int L2 = L1 + 1;
  const int pad = (g.W - g.w3) / 2;               // last_layer_delta.cl:25
  const uint32_t rcp = ((1u << 20) + w2 - 1) / w2;  // p / w2 = (p * rcp) >> 20 for p < 4096
  const int ns = (g.batch - (int)blockIdx.x + (int)gridDim.x - 1) / (int)gridDim.x;
  const int total = ns * U;                       // units of this block's stream
  const int nsteps = total + L2;
  auto tap_off = [&](int tap) { return tap < K3 ? (tap / F3) * w2 + tap % F3 : 0; };
  auto sample_of = [&](int j) { return l3_order((int)blockIdx.x + j * (int)gridDim.x, g.batch); };

  // zero delta3 ring: the slots before the first unit are the zero border
  for (int i = threadIdx.x; i < kL3sRD; i += kL3sThreads) d3r[i] = 0.0f;

  // ---- per-wave roles: W3 operands ----
  const bool qrole = wave < 2;        // Q tap tile `wave`
  const int dt = wave - 2;            // delta2 channel tile (waves 2, 3)
  float wop[8];
#pragma unroll
  for (int s = 0; s < 8; s++) {
    if (qrole) {  // Q B operand: W3[tap = 16 wave + lq][c = 8 lg + s]
      const int tap = 16 * wave + lq;
      wop[s] = tap < K3 ? W3[tap * N2 + 8 * lg + s] : 0.0f;
    } else {      // delta2^T A operand: W3[tap = 4 s + lg][c = 16 dt + lq]
      const int tap = 4 * s + lg;
      wop[s] = (s < 7 && tap < K3) ? W3[tap * N2 + 16 * dt + lq] : 0.0f;
    }
  }
  const float b3 = B3[0];
  wait_vm0();

  // LDS offsets (floats) fixed per lane
  const int sw = lq & 7;
  const int rq0 = lq * 32 + 4 * ((2 * lg) ^ sw), rq1 = lq * 32 + 4 * ((2 * lg + 1) ^ sw);  // Q A operand
  const int rmk = lq * 32 + 4 * (((4 * (dt & 1)) + lg) ^ sw);                             // relu' mask quad
  int od[7];  // delta2 B operand: delta3(pixel lq - off(4 s + lg))
#pragma unroll
  for (int s = 0; s < 7; s++) od[s] = lq - tap_off(4 * s + lg);
  const int t3 = wave >> 1, tc = wave & 1;  // this wave's gW3 tile
  const int gofs = 4 * lg - tap_off(16 * t3 + lq);
  int bo[4];  // gW3 B operand: A2[pixel 4 lg + s][c = 16 tc + lq]
#pragma unroll
  for (int s = 0; s < 4; s++) {
    const int p = 4 * lg + s, c = 16 * tc + lq;
    bo[s] = p * 32 + 4 * ((c >> 2) ^ (p & 7)) + (c & 3);
  }
  f32x4 gacc = mfma::zero4();
  float gb3 = 0.0f, sq = 0.0f;

  // stage counters: stream unit a and its (sample j, unit u) position
  struct Ctr {
    int a, j, u;
    __device__ void next(int U_) {
      if (a >= 0 && ++u == U_) {
        u = 0;
        ++j;
      }
      ++a;
    }
  };
  Ctr cA{kL3sD, 0, kL3sD};       // A2 DMA (waves 0, 1): unit k + D (D < U, l3s_lag)
  Ctr cT{kL3sTD - L1, 0, 0};     // ground-truth DMA (wave 1): unit k - L1 + TD, used TD steps later
  Ctr c3{-L1, 0, 0};             // A3 stage (wave 1): unit k - L1
  Ctr cs{-L1 - 1, 0, 0};         // A3 store (wave 2): unit k - L1 - 1
  Ctr cd{-L2, 0, 0};             // delta2 / gW3 stage: unit k - L2

  // A2 unit (sample j, unit u) -> ring slot; this wave's half (pixels 8w ..)
  auto dma_a2 = [&](int a, int j, int u) {
    const int px = 8 * wave + (lane >> 3), q = (lane & 7) ^ (px & 7);
    const int p = 16 * u + px;
    const bool ok = a < total && p < npx2;
    const float* src = ok ? A2 + ((size_t)sample_of(j) * npx2 + p) * N2 + 4 * q : g_d1c_zero;
    l3s_dma16v_nt(src, a2r + (a % kL3sRA) * 512 + 256 * wave);
  };
  if (qrole)
    for (int a = 0; a < kL3sD; a++) dma_a2(a, 0, a);
#ifdef SRCNN_L3_TIMING
  unsigned long long t_wait = 0, t_all = __builtin_amdgcn_s_memtime();
#endif

  // Every wave that waits on vmcnt issues DMAs only (stores would count in
  // the same in-order counter and turn each wait into a store drain):
  //   wave 0  A2 DMA half                        wait: its unit-k DMA
  //   wave 1  A2 DMA half, ground-truth DMA      wait: both (A3 runs here)
  //   wave 2  delta2 store, A3 store (no waits)
  //   wave 3  delta2 store (no waits)
  int qslot = 0;  // (16 k) mod kL3sRQ
  for (int k = 0; k < nsteps; k++) {
#ifdef SRCNN_L3_TIMING
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
#endif
    // ---- the data this step reads has landed (fixed per-wave counts) ----
    if (wave == 0)
      asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(kL3sD - 1) : "memory");
    else if (wave == 1)  // [A2, T] per step: A2 of unit k is 2D - 1 back, T of unit k - L1 2 TD - 2
      asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(2 * kL3sD - 1 < 2 * kL3sTD - 2 ? 2 * kL3sD - 1
                                                                                    : 2 * kL3sTD - 2)
                   : "memory");
    else
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
#ifdef SRCNN_L3_TIMING
    t_wait += __builtin_amdgcn_s_memtime() - t0;
#endif

    // ---- DMAs of later units ----
    if (qrole) {
      dma_a2(cA.a, cA.j, cA.u);
      if (wave == 1 && lane < 16) {
        const int p = 16 * cT.u + lane;
        const int y = (int)(((uint32_t)p * rcp) >> 20), x = p - y * w2;
        const bool ok = cT.a >= 0 && cT.a < total && y < g.h3 && x < g.w3;
        const float* src = ok ? T + (size_t)sample_of(cT.j) * g.W * g.H + (size_t)(y + pad) * g.W + x + pad : T;
        l3s_dma4v(src, tr + 16 * (cT.a & (kL3sRT / 16 - 1)));
      }
    }
    cA.next(U);
    cT.next(U);

    const int d = cd.a;
    const bool dv = d >= 0 && d < total;
    const float* a2d = a2r + ((d + kL3sRA) % kL3sRA) * 512;

    // ---- gW3 of unit d (every wave, one tile): operands ----
    float ag[4], bg[4];
    if (dv) {
#pragma unroll
      for (int s = 0; s < 4; s++) {
        ag[s] = d3r[(16 * d + gofs + s) & (kL3sRD - 1)];
        bg[s] = a2d[bo[s]];
      }
    }

    if (qrole) {
      // ---- A3 of unit a = k - L1 (wave 1): operands first, so their LDS
      // latency runs under the Q MFMAs ----
      const int a = c3.a;
      float qv[K3];
      if (wave == 1 && lane < 16) {
        int base = (16 * a) % kL3sRQ;
        base = (base < 0 ? base + kL3sRQ : base) + lane;
#pragma unroll
        for (int t = 0; t < K3; t++) {
          int idx = base + (t / F3) * w2 + t % F3;
          idx -= idx >= kL3sRQ ? kL3sRQ : 0;
          qv[t] = qr[idx * kL3sSQ + t];
        }
      }
      // ---- Q of unit k: Q[px][tap] = sum_c A2[px][c] W3[tap][c] ----
      if (k < total) {
        const float* a2u = a2r + (k % kL3sRA) * 512;
        const f32x4 q0 = *reinterpret_cast<const f32x4*>(a2u + rq0);
        const f32x4 q1 = *reinterpret_cast<const f32x4*>(a2u + rq1);
        f32x4 acc = mfma::zero4();
#pragma unroll
        for (int s = 0; s < 4; s++) {
          acc = mfma::mma16(q0[s], wop[s], acc);
          if (dv) gacc = mfma::mma16(ag[s], bg[s], gacc);
        }
#pragma unroll
        for (int s = 0; s < 4; s++) acc = mfma::mma16(q1[s], wop[4 + s], acc);
        // acc[i] = Q[pixel 4 lg + i][tap 16 wave + lq]
        const int tap = 16 * wave + lq;
        if (tap < K3) {
          float* qd = qr + (qslot + 4 * lg) * kL3sSQ + tap;
#pragma unroll
          for (int i = 0; i < 4; i++) qd[i * kL3sSQ] = acc[i];
        }
      } else if (dv) {
#pragma unroll
        for (int s = 0; s < 4; s++) gacc = mfma::mma16(ag[s], bg[s], gacc);
      }
      // ---- A3 = B3 + window sums, last delta, squared error (wave 1) ----
      if (wave == 1 && lane < 16) {
        float sum = 0.0f;
#pragma unroll
        for (int t = 0; t < K3; t++) sum += qv[t];
        const int p = 16 * c3.u + lane;
        const int y = (int)(((uint32_t)p * rcp) >> 20), x = p - y * w2;
        const bool ok = a >= 0 && a < total && y < g.h3 && x < g.w3;
        const float a3 = sum + b3;
        const float diff = a3 - tr[(16 * a + lane) & (kL3sRT - 1)];
        const float d3 = ok ? diff * (a3 > 0.0f ? 1.0f : 0.0f) : 0.0f;
        d3r[(16 * a + lane) & (kL3sRD - 1)] = d3;
        a3r[(16 * a + lane) & (kL3sR3 - 1)] = a3;  // stored by wave 2 next step
        if (ok) {
          gb3 += d3;
          sq += diff * diff;
        }
      }
    } else {
      // ---- A3 of unit k - L1 - 1 to the workspace (wave 2; srcnn_train_activations) ----
      if (wave == 2 && lane < 16) {
        const int a = cs.a;
        const int p = 16 * cs.u + lane;
        const int y = (int)(((uint32_t)p * rcp) >> 20), x = p - y * w2;
        const bool ok = a >= 0 && a < total && y < g.h3 && x < g.w3;
        float* dst = ok ? A3out + (size_t)sample_of(cs.j) * nout + y * g.w3 + x : g_l3s_sink + lane;
        *dst = a3r[(16 * a + lane) & (kL3sR3 - 1)];
      }
      // ---- delta2 of unit d: delta2^T[c][q] = relu'(A2) sum_tap W3[tap][c] delta3(q - off(tap)) ----
      f32x4 v = mfma::zero4();
      if (dv) {
        float ad[7];
#pragma unroll
        for (int s = 0; s < 7; s++) ad[s] = d3r[(16 * d + od[s]) & (kL3sRD - 1)];
        const f32x4 mk = *reinterpret_cast<const f32x4*>(a2d + rmk);
        f32x4 acc = mfma::zero4();
#pragma unroll
        for (int s = 0; s < 7; s++) {
          acc = mfma::mma16(wop[s], ad[s], acc);
          if (s < 4) gacc = mfma::mma16(ag[s], bg[s], gacc);
        }
#pragma unroll
        for (int i = 0; i < 4; i++) v[i] = mk[i] > 0.0f ? acc[i] : 0.0f;
      }
      // acc[i] = delta2[pixel lq][channel 16 dt + 4 lg + i]
      const int q = 16 * cd.u + lq;
      if (dv && q < npx2)
        *reinterpret_cast<f32x4*>(D2 + ((size_t)sample_of(cd.j) * npx2 + q) * N2 + 16 * dt + 4 * lg) = v;
    }
    c3.next(U);
    cs.next(U);
    cd.next(U);
    qslot += 16;
    if (qslot == kL3sRQ) qslot = 0;
  }
#ifdef SRCNN_L3_TIMING
  if (lane == 0) {
    g_l3s_timing[blockIdx.x][2 * wave] = t_wait;
    g_l3s_timing[blockIdx.x][2 * wave + 1] = __builtin_amdgcn_s_memtime() - t_all;
  }
#endif
  wait_vm0();  // no LDS-DMA outstanding when the block ends
  SRCNN_CLOCK_END(g_clk, 1);

  // ---- this block's slab: [gW3 | gB3]; each wave writes its tile ----
  float* out = slab3 + (size_t)blockIdx.x * (NW3 + 1);
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const int tap = 16 * t3 + 4 * lg + i;
    if (tap < K3) out[tap * N2 + 16 * tc + lq] = gacc[i];
  }
  if (wave == 1) {  // gB3 and the squared error: wave 1's lanes 0..15, fixed order
    for (int off = 32; off > 0; off >>= 1) {
      gb3 += __shfl_down(gb3, off, 64);
      sq += __shfl_down(sq, off, 64);
    }
    if (lane == 0) {
      out[NW3] = gb3;
      sq_slab[blockIdx.x] = sq;
    }
  }
}

inline size_t l3s_lds_bytes() { return (size_t)kL3sLdsFloats * sizeof(float); }
