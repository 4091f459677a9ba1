// common.hpp -- shared helpers of libsrcnn_hip.so (error state, launch math).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstddef>
#include <cstdint>

#include "srcnn.h"

namespace srcnn {

// Records a thread-local message for srcnn_last_error() and returns `code`.
int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
void clear_error();
// the kernels (by variant) of this thread's most recent network-level call,
// comma-separated (srcnn_last_kernels)
void kernels_reset();
void kernels_note(const char* name);
const char* kernels_last();

// hipFuncGetAttributes on each kernel: the runtime's lazy per-device kernel
// setup happens here instead of at the first launch (srcnn_preload)
inline int resolve_kernels(const void* const* fns, int n) {
  for (int i = 0; i < n; i++) {
    hipFuncAttributes a;
    hipError_t e = hipFuncGetAttributes(&a, fns[i]);
    if (e != hipSuccess) return fail(SRCNN_ERR_HIP, "hipFuncGetAttributes: %s", hipGetErrorString(e));
  }
  return SRCNN_OK;
}

inline hipStream_t as_stream(srcnn_stream_t s) { return reinterpret_cast<hipStream_t>(s); }

inline uint32_t grid_for(size_t total, uint32_t block, uint32_t cap = 1u << 20) {
  size_t g = (total + block - 1) / block;
  if (g == 0) g = 1;
  return g > cap ? cap : static_cast<uint32_t>(g);
}

// kernel-path selection (srcnn_set_path): 0 auto, 1 generic only
extern int g_path;
// matrix-core arithmetic (srcnn_set_arith): 0 split bf16, 1 fp32 MFMA only
extern int g_arith;

// Per-launch hipEvent bracketing for srcnn_profile_* (reference profile
// mode, src/opencl/Kernel.cpp:108-116).  A no-op unless profiling is on.
namespace prof {
extern bool g_enabled;
struct Scope {
  Scope(const char* name, hipStream_t s) {
    if (g_enabled) begin(name, s);
  }
  ~Scope() {
    if (start_) end();
  }
  void begin(const char* name, hipStream_t s);
  void end();
  const char* name_ = nullptr;
  hipStream_t stream_ = nullptr;
  hipEvent_t start_ = nullptr, stop_ = nullptr;
};
}  // namespace prof

}  // namespace srcnn

#define SRCNN_HIP_TRY(expr)                                                        \
  do {                                                                             \
    hipError_t e_ = (expr);                                                        \
    if (e_ != hipSuccess)                                                          \
      return ::srcnn::fail(SRCNN_ERR_HIP, "%s failed: %s (%s:%d)", #expr,          \
                           hipGetErrorString(e_), __FILE__, __LINE__);             \
  } while (0)

#define SRCNN_LAUNCH_TRY() SRCNN_HIP_TRY(hipGetLastError())

// bracket the launches that follow in this scope for the profiler
#define SRCNN_PROFILE(name, stream) ::srcnn::prof::Scope srcnn_prof_scope_(name, stream)

// Held-clock probe (MI355X_MICROARCH.md "DVFS give-back", item 6), built
// only into the diagnostic variant (make PROBE=1 -> -DSRCNN_CLOCK_PROBE): the
// first kClockBlocks blocks of a fused kernel record the s_memtime (shader
// clock) and s_memrealtime (100 MHz) deltas over their lifetime into a
// per-kernel slot of a device array; srcnn_profile_clock() reports their
// median ratio.  The production kernels carry no probe.
namespace srcnn {
// s_waitcnt vmcnt(0) that the compiler's wait-count pass sees (expcnt and
// lgkmcnt left at their maxima; gfx9 encoding vmcnt[3:0] | expcnt[6:4] |
// lgkmcnt[11:8] | vmcnt[5:4] << 14).  The kernels issue their LDS-DMA as
// inline asm, which that pass cannot count; after an inline-asm vmcnt(0) it
// still believed older loads outstanding and, at their first use, emitted a
// vmcnt(N) that waited for the DMA just issued.  After this one it knows them
// complete and emits no such wait.
__device__ __forceinline__ void wait_vm0() { __builtin_amdgcn_s_waitcnt(0x0F70); }
constexpr int kClockBlocks = 8;
#ifdef SRCNN_CLOCK_PROBE
constexpr bool kClockProbe = true;
#else
constexpr bool kClockProbe = false;
#endif
}
#ifndef SRCNN_CLOCK_PROBE
#define SRCNN_CLOCK_BEGIN() \
  do {                      \
  } while (0)
#define SRCNN_CLOCK_END(ARR, SLOT) \
  do {                             \
  } while (0)
#else
#define SRCNN_CLOCK_BEGIN()                                                        \
  const unsigned long long srcnn_clk_c0_ = __builtin_amdgcn_s_memtime();           \
  const unsigned long long srcnn_clk_r0_ = __builtin_amdgcn_s_memrealtime()
#define SRCNN_CLOCK_END(ARR, SLOT)                                                 \
  do {                                                                             \
    if (blockIdx.x < (unsigned)::srcnn::kClockBlocks && threadIdx.x == 0) {        \
      const unsigned long long c1_ = __builtin_amdgcn_s_memtime();                 \
      const unsigned long long r1_ = __builtin_amdgcn_s_memrealtime();             \
      (ARR)[SLOT][blockIdx.x][0] = c1_ - srcnn_clk_c0_;                            \
      (ARR)[SLOT][blockIdx.x][1] = r1_ - srcnn_clk_r0_;                            \
    }                                                                              \
  } while (0)
#endif

namespace srcnn {
// median shader clock (GHz) over the probe blocks of one slot; -1 if unset
inline double clock_ghz(const unsigned long long (*a)[2]) {
  double v[kClockBlocks];
  int n = 0;
  for (int b = 0; b < kClockBlocks; b++)
    if (a[b][1] > 0) v[n++] = (double)a[b][0] / (double)a[b][1] * 0.1;
  if (n == 0) return -1.0;
  for (int i = 1; i < n; i++)
    for (int j = i; j > 0 && v[j - 1] > v[j]; j--) {
      const double t = v[j];
      v[j] = v[j - 1];
      v[j - 1] = t;
    }
  return n % 2 ? v[n / 2] : 0.5 * (v[n / 2 - 1] + v[n / 2]);
}
}  // namespace srcnn

#define SRCNN_REQUIRE(cond, ...)                                                   \
  do {                                                                             \
    if (!(cond)) return ::srcnn::fail(SRCNN_ERR_INVALID, __VA_ARGS__);             \
  } while (0)
