// mfma.hpp -- gfx950 fp32 MFMA helpers shared by the fast kernels.
//
// v_mfma_f32_32x32x2_f32 (exact fp32: a k-ordered fma chain, MI355X_MICROARCH.md
// "Matrix cores"), one wave computes D[32x32] += A[32x2] * B[2x32]:
//   A operand: lane l holds A[i = l&31][k = l>>5]
//   B operand: lane l holds B[k = l>>5][j = l&31]
//   C/D:       lane l, register r holds D[crow(r, l>>5)][l&31]
//              crow(r, h) = (r&3) + 8*(r>>2) + 4*h
// Because the k index of one instruction is just the lane half, any fixed
// pairing of "k-slot s, half h" <-> "reduction index" works as long as the A
// and B operands agree on it.  The kernels use that to feed an accumulator
// tile straight back as the next product's operand (register s of half h is
// reduction index crow(s, h)) with no data movement.
#pragma once

#include <hip/hip_runtime.h>

// (l12 / fwd_l123 start the L2 accumulator from B2 instead of one more MFMA
// per 32-pixel chunk: l12 0.3051 -> 0.3040 ms, 3840x2160 frame 1.134 ->
// 1.112 ms, bit-identical; profiles/r04_ab_b2init)

namespace srcnn {
namespace mfma {

typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ f32x16 mma(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

// v_mfma_f32_16x16x4_f32 (same fp32 rate, 32-cycle issue): D[16x16] += A[16x4] * B[4x16]
//   A: lane l holds A[l&15][k = l>>4];  B: B[k = l>>4][l&15]
//   C/D: lane l, register i holds D[4*(l>>4) + i][l&15]
typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x4 mma16(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ f32x4 zero4() {
  f32x4 z;
#pragma unroll
  for (int i = 0; i < 4; i++) z[i] = 0.0f;
  return z;
}

__device__ __forceinline__ constexpr int crow(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

__device__ __forceinline__ f32x16 zero16() {
  f32x16 z;
#pragma unroll
  for (int i = 0; i < 16; i++) z[i] = 0.0f;
  return z;
}

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }
// wave index, provably uniform (SGPR): keeps per-wave LDS bases and DMA M0
// values scalar instead of per-lane VGPRs
__device__ __forceinline__ int wave_id() { return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); }

}  // namespace mfma
}  // namespace srcnn
