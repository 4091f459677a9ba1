// runtime.cpp -- device / memory / stream / event entry points of srcnn.h.
// Replaces opencl::Context (reference src/opencl/Context.{hpp,cpp}): one HIP
// stream per caller instead of the single in-order cl_command_queue
// (Context.cpp:70-72); allocations are raw device pointers instead of
// index-addressed MemoryHandles (the C++ cnn_sr::Context keeps the handles).
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "common.hpp"
#include "ops.hpp"

namespace srcnn {

static thread_local std::string t_last_error;
// SRCNN_PATH=generic in the environment starts the library on the generic
// kernels (A/B runs of programs that do not call srcnn_set_path themselves)
static int initial_path() {
  const char* e = getenv("SRCNN_PATH");
  return e && !strcmp(e, "generic") ? 1 : 0;
}
int g_path = initial_path();
// SRCNN_ARITH=f32 starts the library on the fp32-MFMA kernels (srcnn_set_arith)
static int initial_arith() {
  const char* e = getenv("SRCNN_ARITH");
  return e && !strcmp(e, "f32") ? 1 : 0;
}
int g_arith = initial_arith();

int fail(int code, const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  t_last_error.assign(buf);
  return code;
}

void clear_error() { t_last_error.clear(); }

// kernels launched by this thread's most recent network-level call
// (srcnn_last_kernels)
static thread_local std::string t_kernels;
void kernels_reset() { t_kernels.clear(); }
void kernels_note(const char* name) {
  if (!t_kernels.empty()) t_kernels += ',';
  t_kernels += name;
}
const char* kernels_last() { return t_kernels.c_str(); }

const char* last_error() { return t_last_error.c_str(); }

namespace prof {
bool g_enabled = false;

struct Pending {
  std::string name;
  hipEvent_t start, stop;
};
struct Totals {
  uint64_t launches = 0;
  double ms = 0.0;
};
static std::mutex g_mu;
static std::vector<Pending> g_pending;
static std::vector<hipEvent_t> g_free;
static std::map<std::string, Totals> g_totals;

static hipEvent_t take_event() {
  if (!g_free.empty()) {
    hipEvent_t e = g_free.back();
    g_free.pop_back();
    return e;
  }
  // timing-only events: without the system-scope fence the default event
  // record writes back and invalidates the caches, so every profiled kernel
  // started cold (the step ran 3.4% slower with events around each launch)
  hipEvent_t e = nullptr;
  if (hipEventCreateWithFlags(&e, hipEventDisableSystemFence) != hipSuccess) return nullptr;
  return e;
}

void Scope::begin(const char* name, hipStream_t s) {
  // launches captured into a graph (srcnn_graph_begin) are not bracketed:
  // event records inside a capture would become graph nodes
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(s, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return;
  std::lock_guard<std::mutex> lk(g_mu);
  start_ = take_event();
  stop_ = take_event();
  if (!start_ || !stop_) {
    start_ = stop_ = nullptr;
    return;
  }
  name_ = name;
  stream_ = s;
  (void)hipEventRecord(start_, s);
}

void Scope::end() {
  (void)hipEventRecord(stop_, stream_);
  std::lock_guard<std::mutex> lk(g_mu);
  g_pending.push_back({name_, start_, stop_});
}

// fold finished events into the totals (waits for them)
static int flush() {
  std::lock_guard<std::mutex> lk(g_mu);
  for (auto& p : g_pending) {
    hipError_t e = hipEventSynchronize(p.stop);
    float ms = 0.f;
    if (e == hipSuccess) e = hipEventElapsedTime(&ms, p.start, p.stop);
    if (e != hipSuccess)
      return fail(SRCNN_ERR_HIP, "profile: event query failed: %s", hipGetErrorString(e));
    Totals& t = g_totals[p.name];
    t.launches++;
    t.ms += ms;
    g_free.push_back(p.start);
    g_free.push_back(p.stop);
  }
  g_pending.clear();
  return SRCNN_OK;
}
}  // namespace prof

}  // namespace srcnn

using srcnn::as_stream;

extern "C" {

int srcnn_abi_version(void) { return SRCNN_ABI_VERSION; }

const char* srcnn_last_error(void) { return srcnn::last_error(); }

int srcnn_set_path(int path) {
  SRCNN_REQUIRE(path == 0 || path == 1, "srcnn_set_path: path must be 0 (auto) or 1 (generic), got %d", path);
  srcnn::g_path = path;
  return SRCNN_OK;
}

int srcnn_get_path(void) { return srcnn::g_path; }

int srcnn_set_arith(int arith) {
  SRCNN_REQUIRE(arith == 0 || arith == 1, "srcnn_set_arith: arith must be 0 (split bf16) or 1 (fp32 MFMA), got %d",
                arith);
  srcnn::g_arith = arith;
  return SRCNN_OK;
}

int srcnn_get_arith(void) { return srcnn::g_arith; }

int srcnn_profile_enable(int on) {
  srcnn::prof::g_enabled = on != 0;
  return SRCNN_OK;
}

int srcnn_profile_reset(void) {
  if (int rc = srcnn::prof::flush()) return rc;
  std::lock_guard<std::mutex> lk(srcnn::prof::g_mu);
  srcnn::prof::g_totals.clear();
  return SRCNN_OK;
}

int srcnn_profile_count(int* n) {
  SRCNN_REQUIRE(n, "srcnn_profile_count: null out pointer");
  if (int rc = srcnn::prof::flush()) return rc;
  std::lock_guard<std::mutex> lk(srcnn::prof::g_mu);
  *n = (int)srcnn::prof::g_totals.size();
  return SRCNN_OK;
}

int srcnn_profile_get(int index, char* name, size_t name_len, uint64_t* launches,
                      double* total_ms) {
  std::lock_guard<std::mutex> lk(srcnn::prof::g_mu);
  SRCNN_REQUIRE(index >= 0 && index < (int)srcnn::prof::g_totals.size(),
                "srcnn_profile_get: index %d out of range", index);
  auto it = srcnn::prof::g_totals.begin();
  std::advance(it, index);
  if (name && name_len) snprintf(name, name_len, "%s", it->first.c_str());
  if (launches) *launches = it->second.launches;
  if (total_ms) *total_ms = it->second.ms;
  return SRCNN_OK;
}

int srcnn_profile_print(void) {
  if (int rc = srcnn::prof::flush()) return rc;
  std::lock_guard<std::mutex> lk(srcnn::prof::g_mu);
  for (auto& kv : srcnn::prof::g_totals) {
    const double ns = kv.second.ms * 1e6;
    printf("Kernel '%s' total execution time: %.0fns = %.6fs (%llu launches)\n", kv.first.c_str(),
           ns, ns * 1e-9, (unsigned long long)kv.second.launches);
  }
  fflush(stdout);
  return SRCNN_OK;
}

int srcnn_profile_clock(const char* kernel, double* ghz) {
  SRCNN_REQUIRE(kernel && ghz, "srcnn_profile_clock: null argument");
  static const char* const kTrain[] = {"l12_fwd_mfma", "l3_delta_fused", "delta1_grad12_fused"};
  for (int i = 0; i < 3; i++)
    if (!strcmp(kernel, kTrain[i])) return srcnn::fused::train_clock(i, ghz);
  if (!strcmp(kernel, "fwd_l123_mfma")) return srcnn::fused::forward_clock(ghz);
  return srcnn::fail(SRCNN_ERR_INVALID, "srcnn_profile_clock: no clock probe in kernel '%s'", kernel);
}

int srcnn_device_count(int* count) {
  SRCNN_REQUIRE(count, "srcnn_device_count: null count");
  SRCNN_HIP_TRY(hipGetDeviceCount(count));
  return SRCNN_OK;
}

int srcnn_set_device(int device) {
  SRCNN_HIP_TRY(hipSetDevice(device));
  return SRCNN_OK;
}

int srcnn_device_name(char* buf, size_t len) {
  SRCNN_REQUIRE(buf && len > 0, "srcnn_device_name: empty buffer");
  int dev = 0;
  SRCNN_HIP_TRY(hipGetDevice(&dev));
  hipDeviceProp_t prop;
  SRCNN_HIP_TRY(hipGetDeviceProperties(&prop, dev));
  snprintf(buf, len, "%s (%s, %d CUs)", prop.name, prop.gcnArchName, prop.multiProcessorCount);
  return SRCNN_OK;
}

int srcnn_malloc(void** ptr, size_t bytes) {
  SRCNN_REQUIRE(ptr, "srcnn_malloc: null out pointer");
  *ptr = nullptr;
  if (bytes == 0) return SRCNN_OK;
  hipError_t e = hipMalloc(ptr, bytes);
  if (e != hipSuccess)
    return srcnn::fail(SRCNN_ERR_ALLOC, "hipMalloc(%zu) failed: %s", bytes, hipGetErrorString(e));
  return SRCNN_OK;
}

int srcnn_free(void* ptr) {
  if (ptr) SRCNN_HIP_TRY(hipFree(ptr));
  return SRCNN_OK;
}

int srcnn_memcpy_h2d(void* dst, const void* src, size_t bytes, srcnn_stream_t stream) {
  if (bytes == 0) return SRCNN_OK;
  SRCNN_REQUIRE(dst && src, "srcnn_memcpy_h2d: null pointer");
  SRCNN_HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, as_stream(stream)));
  SRCNN_HIP_TRY(hipStreamSynchronize(as_stream(stream)));
  return SRCNN_OK;
}

int srcnn_memcpy_d2h(void* dst, const void* src, size_t bytes, srcnn_stream_t stream) {
  if (bytes == 0) return SRCNN_OK;
  SRCNN_REQUIRE(dst && src, "srcnn_memcpy_d2h: null pointer");
  SRCNN_HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, as_stream(stream)));
  SRCNN_HIP_TRY(hipStreamSynchronize(as_stream(stream)));
  return SRCNN_OK;
}

int srcnn_memcpy_d2d(void* dst, const void* src, size_t bytes, srcnn_stream_t stream) {
  if (bytes == 0) return SRCNN_OK;
  SRCNN_REQUIRE(dst && src, "srcnn_memcpy_d2d: null pointer");
  SRCNN_HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, as_stream(stream)));
  return SRCNN_OK;
}

int srcnn_stream_create(srcnn_stream_t* stream) {
  SRCNN_REQUIRE(stream, "srcnn_stream_create: null out pointer");
  hipStream_t s;
  SRCNN_HIP_TRY(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  *stream = s;
  return SRCNN_OK;
}

int srcnn_stream_destroy(srcnn_stream_t stream) {
  if (stream) SRCNN_HIP_TRY(hipStreamDestroy(as_stream(stream)));
  return SRCNN_OK;
}

int srcnn_stream_sync(srcnn_stream_t stream) {
  SRCNN_HIP_TRY(hipStreamSynchronize(as_stream(stream)));
  return SRCNN_OK;
}

int srcnn_device_sync(void) {
  SRCNN_HIP_TRY(hipDeviceSynchronize());
  return SRCNN_OK;
}

int srcnn_event_create(srcnn_event_t* ev) {
  SRCNN_REQUIRE(ev, "srcnn_event_create: null out pointer");
  hipEvent_t e;
  SRCNN_HIP_TRY(hipEventCreate(&e));
  *ev = e;
  return SRCNN_OK;
}

int srcnn_event_destroy(srcnn_event_t ev) {
  if (ev) SRCNN_HIP_TRY(hipEventDestroy(reinterpret_cast<hipEvent_t>(ev)));
  return SRCNN_OK;
}

int srcnn_event_record(srcnn_event_t ev, srcnn_stream_t stream) {
  SRCNN_REQUIRE(ev, "srcnn_event_record: null event");
  SRCNN_HIP_TRY(hipEventRecord(reinterpret_cast<hipEvent_t>(ev), as_stream(stream)));
  return SRCNN_OK;
}

int srcnn_event_sync(srcnn_event_t ev) {
  SRCNN_REQUIRE(ev, "srcnn_event_sync: null event");
  SRCNN_HIP_TRY(hipEventSynchronize(reinterpret_cast<hipEvent_t>(ev)));
  return SRCNN_OK;
}

int srcnn_graph_begin(srcnn_stream_t stream) {
  SRCNN_REQUIRE(stream, "srcnn_graph_begin: capture needs a created stream, not the NULL stream");
  SRCNN_HIP_TRY(hipStreamBeginCapture(as_stream(stream), hipStreamCaptureModeThreadLocal));
  return SRCNN_OK;
}

int srcnn_graph_end(srcnn_stream_t stream, srcnn_graph_t* graph) {
  SRCNN_REQUIRE(stream && graph, "srcnn_graph_end: null argument");
  *graph = nullptr;
  hipGraph_t g = nullptr;
  SRCNN_HIP_TRY(hipStreamEndCapture(as_stream(stream), &g));
  hipGraphExec_t ex = nullptr;
  const hipError_t e = hipGraphInstantiate(&ex, g, nullptr, nullptr, 0);
  (void)hipGraphDestroy(g);
  if (e != hipSuccess)
    return srcnn::fail(SRCNN_ERR_HIP, "hipGraphInstantiate: %s", hipGetErrorString(e));
  *graph = ex;
  return SRCNN_OK;
}

int srcnn_graph_launch(srcnn_graph_t graph, srcnn_stream_t stream) {
  SRCNN_REQUIRE(graph, "srcnn_graph_launch: null graph");
  SRCNN_HIP_TRY(hipGraphLaunch(reinterpret_cast<hipGraphExec_t>(graph), as_stream(stream)));
  return SRCNN_OK;
}

int srcnn_graph_destroy(srcnn_graph_t graph) {
  if (graph) SRCNN_HIP_TRY(hipGraphExecDestroy(reinterpret_cast<hipGraphExec_t>(graph)));
  return SRCNN_OK;
}

int srcnn_event_elapsed_ms(srcnn_event_t start, srcnn_event_t stop, float* ms) {
  SRCNN_REQUIRE(start && stop && ms, "srcnn_event_elapsed_ms: null argument");
  SRCNN_HIP_TRY(hipEventElapsedTime(ms, reinterpret_cast<hipEvent_t>(start),
                                    reinterpret_cast<hipEvent_t>(stop)));
  return SRCNN_OK;
}

}  // extern "C"
