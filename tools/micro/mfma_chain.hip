// Microbenchmark: throughput of fp32 MFMA 32x32x2 with C independent
// accumulator chains per wave (1 or 2 waves per SIMD).  Prints cycles/MFMA.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int C>
__global__ __launch_bounds__(256) void chain(float* out, int iters, long long* cyc) {
  f32x16 acc[C];
  for (int c = 0; c < C; c++)
    for (int i = 0; i < 16; i++) acc[c][i] = 0.0f;
  float a = threadIdx.x * 1e-3f, b = 1.0f + threadIdx.x * 1e-4f;
  long long t0 = clock64();
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int k = 0; k < 32 / C; k++)
#pragma unroll
      for (int c = 0; c < C; c++) acc[c] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[c], 0, 0, 0);
  }
  long long t1 = clock64();
  float s = 0.0f;
  for (int c = 0; c < C; c++)
    for (int i = 0; i < 16; i++) s += acc[c][i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}

template <int C>
void run(int waves_per_simd) {
  float* out;
  long long* cyc;
  hipMalloc(&out, 256 * 4096 * 4);
  hipMalloc(&cyc, 8);
  const int iters = 2000, blocks = 256 * waves_per_simd;
  hipLaunchKernelGGL(chain<C>, dim3(blocks), dim3(256), 0, 0, out, 10, cyc);
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL(chain<C>, dim3(blocks), dim3(256), 0, 0, out, iters, cyc);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  long long c;
  hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
  const double mfma_per_simd = (double)iters * 32 * waves_per_simd;
  printf("chains=%d waves/SIMD=%d: %.1f clock64-cycles per MFMA (wave view), %.2f ns per MFMA per SIMD, %.1f TF\n",
         C, waves_per_simd, (double)c / (iters * 32), ms * 1e6 / mfma_per_simd,
         mfma_per_simd * 1024 * 4096 / (ms * 1e-3) / 1e12);
  hipFree(out);
  hipFree(cyc);
}

int main() {
  for (int w = 1; w <= 2; w++) {
    run<1>(w);
    run<2>(w);
    run<4>(w);
    run<8>(w);
  }
  return 0;
}
