// Probe: throughput of the bf16 MFMA shapes on random operands with every
// SIMD of the chip busy (so the held clock is in the number), 2 waves/SIMD,
// 4 independent accumulators per wave.  Prints ns per MFMA per SIMD and the
// fp32-equivalent TF/s of a six-product split scheme on each shape.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

template <int S>
__global__ __launch_bounds__(256) void rate(float* out, int iters, unsigned seed) {
  unsigned x = seed ^ (threadIdx.x * 2654435761u) ^ (blockIdx.x * 40503u);
  auto rnd = [&]() { x = x * 1664525u + 1013904223u; return (float)(x >> 8) * (1.0f / 16777216.0f) - 0.5f; };
  bf16x8 a8[2], b8[2];
  bf16x4 a4[2], b4[2];
  for (int i = 0; i < 2; i++)
    for (int j = 0; j < 8; j++) {
      a8[i][j] = (__bf16)rnd(); b8[i][j] = (__bf16)rnd();
      if (j < 4) { a4[i][j] = (__bf16)rnd(); b4[i][j] = (__bf16)rnd(); }
    }
  f32x16 c16[4];
  f32x4 c4[4];
  for (int c = 0; c < 4; c++) { for (int i = 0; i < 16; i++) c16[c][i] = 0; for (int i = 0; i < 4; i++) c4[c][i] = 0; }
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int k = 0; k < 8; k++)
#pragma unroll
      for (int c = 0; c < 4; c++) {
        if (S == 0) c16[c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a8[k & 1], b8[(k >> 1) & 1], c16[c], 0, 0, 0);
        if (S == 1) c4[c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a8[k & 1], b8[(k >> 1) & 1], c4[c], 0, 0, 0);
        if (S == 2) c4[c] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a4[k & 1], b4[(k >> 1) & 1], c4[c], 0, 0, 0);
        if (S == 3) c16[c] = __builtin_amdgcn_mfma_f32_32x32x8bf16_1k(a4[k & 1], b4[(k >> 1) & 1], c16[c], 0, 0, 0);
      }
  }
  float s = 0;
  for (int c = 0; c < 4; c++) { for (int i = 0; i < 16; i++) s += c16[c][i]; for (int i = 0; i < 4; i++) s += c4[c][i]; }
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
  float* out;
  (void)hipMalloc(&out, 1024 * 256 * 4);
  const char* names[4] = {"32x32x16 bf16", "16x16x32 bf16", "16x16x16 bf16", "32x32x8 bf16"};
  const double flop[4] = {32.0 * 32 * 16 * 2, 16.0 * 16 * 32 * 2, 16.0 * 16 * 16 * 2, 32.0 * 32 * 8 * 2};
  for (int rep = 0; rep < 2; rep++)
    for (int sh = 0; sh < 4; sh++) {
      auto k = sh == 0 ? rate<0> : sh == 1 ? rate<1> : sh == 2 ? rate<2> : rate<3>;
      const int blocks = 512, iters = 6000;  // 2 waves per SIMD
      hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, 200, 7u);
      (void)hipDeviceSynchronize();
      hipEvent_t e0, e1;
      (void)hipEventCreate(&e0);
      (void)hipEventCreate(&e1);
      (void)hipEventRecord(e0);
      hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, iters, 11u);
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      float ms;
      (void)hipEventElapsedTime(&ms, e0, e1);
      const double per_simd = (double)iters * 32 * 2;  // MFMAs per SIMD (2 waves)
      const double tf = per_simd * 1024 * flop[sh] / (ms * 1e-3) / 1e12;
      printf("%s: %.2f ns per MFMA per SIMD, %.0f TF/s bf16, %.0f TF/s fp32-equivalent (x6)\n", names[sh],
             ms * 1e6 / per_simd, tf, tf / 6);
    }
  return 0;
}
