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

inline hipStream_t as_stream(srcnn_stream_t s) { return reinterpret_cast<hipStream_t>(s); }

inline uint32_t grid_for(size_t total, uint32_t block, uint32_t cap = 1u << 20) {
  size_t g = (total + block - 1) / block;
  if (g == 0) g = 1;
  return g > cap ? cap : static_cast<uint32_t>(g);
}

// kernel-path selection (srcnn_set_path): 0 auto, 1 generic only
extern int g_path;

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

#define SRCNN_REQUIRE(cond, ...)                                                   \
  do {                                                                             \
    if (!(cond)) return ::srcnn::fail(SRCNN_ERR_INVALID, __VA_ARGS__);             \
  } while (0)
