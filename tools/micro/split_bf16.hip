// Probe: fp32 GEMM tiles through split-bf16 MFMAs on gfx950.
//   a = a0 + a1 + a2 (each bf16, round-to-nearest residual split), the same
//   for b; D += sum of the kept part products through v_mfma_f32_32x32x16_bf16.
//   x3: a0b0 a0b1 a1b0      x6: + a0b2 a1b1 a2b0      x9: every product
// against v_mfma_f32_32x32x2_f32 and an fp64 host product.  Prints, per data
// set and K, the normwise and max elementwise relative error of each form,
// then the matrix-pipe rate of the 32x32x16 bf16 and 32x32x2 f32 loops.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ void split3(float a, __bf16& h, __bf16& m, __bf16& l) {
  h = (__bf16)a;
  const float r = a - (float)h;
  m = (__bf16)r;
  l = (__bf16)(r - (float)m);
}

// one wave: D[32][32] = A[32][K] . B[K][32]; mode 0 f32, 3 / 6 / 9 split terms
__global__ void tile_gemm(const float* A, const float* B, float* D, int K, int mode) {
  const int l = threadIdx.x, col = l & 31, hh = l >> 5;
  f32x16 acc;
  for (int i = 0; i < 16; i++) acc[i] = 0.0f;
  if (mode == 0) {
    for (int k = 0; k < K; k += 2)
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(A[col * K + k + hh], B[(k + hh) * 32 + col], acc, 0, 0, 0);
  } else {
    for (int k = 0; k < K; k += 16) {
      bf16x8 a[3], b[3];
      for (int j = 0; j < 8; j++) {
        const int kk = k + 8 * hh + j;
        __bf16 x0, x1, x2;
        split3(A[col * K + kk], x0, x1, x2);
        a[0][j] = x0, a[1][j] = x1, a[2][j] = x2;
        split3(B[kk * 32 + col], x0, x1, x2);
        b[0][j] = x0, b[1][j] = x1, b[2][j] = x2;
      }
      // small terms first
      if (mode >= 9) {
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2], b[2], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[2], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2], b[1], acc, 0, 0, 0);
      }
      if (mode >= 6) {
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2], b[0], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[1], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[2], acc, 0, 0, 0);
      }
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[0], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[1], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[0], acc, 0, 0, 0);
    }
  }
  for (int r = 0; r < 16; r++) {
    const int row = (r & 3) + 8 * (r >> 2) + 4 * hh;
    D[row * 32 + col] = acc[r];
  }
}

// matrix-pipe rate: independent accumulators, operands in registers
template <bool kBf16>
__global__ __launch_bounds__(256) void rate(float* out, int iters) {
  f32x16 acc[4];
  for (int c = 0; c < 4; c++)
    for (int i = 0; i < 16; i++) acc[c][i] = 0.0f;
  const float a = threadIdx.x * 1e-3f, b = 1.0f + threadIdx.x * 1e-4f;
  bf16x8 av, bv;
  for (int j = 0; j < 8; j++) av[j] = (__bf16)(a + j), bv[j] = (__bf16)(b - j);
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int k = 0; k < 8; k++)
#pragma unroll
      for (int c = 0; c < 4; c++)
        acc[c] = kBf16 ? __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, bv, acc[c], 0, 0, 0)
                       : __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[c], 0, 0, 0);
  }
  float s = 0.0f;
  for (int c = 0; c < 4; c++)
    for (int i = 0; i < 16; i++) s += acc[c][i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

static void errors(const char* tag, const std::vector<float>& A, const std::vector<float>& B, int K) {
  std::vector<double> ref(32 * 32);
  double rn = 0.0;
  for (int i = 0; i < 32; i++)
    for (int j = 0; j < 32; j++) {
      double s = 0.0;
      for (int k = 0; k < K; k++) s += (double)A[i * K + k] * B[k * 32 + j];
      ref[i * 32 + j] = s;
      rn += s * s;
    }
  rn = std::sqrt(rn);
  float *dA, *dB, *dD;
  hipMalloc(&dA, A.size() * 4);
  hipMalloc(&dB, B.size() * 4);
  hipMalloc(&dD, 32 * 32 * 4);
  hipMemcpy(dA, A.data(), A.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(dB, B.data(), B.size() * 4, hipMemcpyHostToDevice);
  printf("%-10s K=%4d", tag, K);
  for (int mode : {0, 3, 6, 9}) {
    hipLaunchKernelGGL(tile_gemm, dim3(1), dim3(64), 0, 0, dA, dB, dD, K, mode);
    std::vector<float> D(32 * 32);
    hipMemcpy(D.data(), dD, 32 * 32 * 4, hipMemcpyDeviceToHost);
    double en = 0.0, emax = 0.0;
    for (int i = 0; i < 32 * 32; i++) {
      const double e = D[i] - ref[i];
      en += e * e;
      // elementwise, relative to the row of |a| . |b| (the product scale)
      emax = std::fmax(emax, std::fabs(e) / (std::fabs(ref[i]) + 1e-30));
    }
    printf("  %s norm %.2e max %.2e", mode == 0 ? "f32" : mode == 3 ? "x3" : mode == 6 ? "x6" : "x9",
           std::sqrt(en) / rn, emax);
  }
  printf("\n");
  hipFree(dA);
  hipFree(dB);
  hipFree(dD);
}

int main() {
  std::mt19937 rng(7);
  std::normal_distribution<float> nd(0.f, 1.f);
  std::uniform_real_distribution<float> ud(0.f, 1.f);
  for (int K : {96, 640}) {
    std::vector<float> A(32 * K), B(K * 32);
    for (auto& v : A) v = nd(rng);
    for (auto& v : B) v = nd(rng);
    errors("normal", A, B, K);
    for (auto& v : A) v = 1e-3f * nd(rng);
    for (auto& v : B) v = ud(rng);
    errors("w1e-3*x", A, B, K);
    for (auto& v : A) v = std::ldexp(nd(rng), (int)(ud(rng) * 20) - 10);
    for (auto& v : B) v = std::ldexp(nd(rng), (int)(ud(rng) * 20) - 10);
    errors("wide-exp", A, B, K);
  }
  float* out;
  hipMalloc(&out, 1024 * 256 * 4);
  for (int waves : {1, 2}) {
    const int blocks = 256 * waves, iters = 4000;
    for (int bf : {0, 1}) {
      auto k = bf ? rate<true> : rate<false>;
      hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, 10);
      hipDeviceSynchronize();
      hipEvent_t e0, e1;
      hipEventCreate(&e0);
      hipEventCreate(&e1);
      hipEventRecord(e0);
      hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, iters);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      const double per_simd = (double)iters * 32 * waves;
      printf("%s waves/SIMD=%d: %.2f ns per MFMA per SIMD\n", bf ? "32x32x16 bf16" : "32x32x2 f32 ", waves,
             ms * 1e6 / per_simd);
    }
  }
  return 0;
}
