// srcnn::Context -- the host runtime the cnn_sr pipeline talks to.
//
// Replaces opencl::Context (reference src/opencl/Context.hpp:72-299) with the
// same surface: handle-indexed device allocations, blocking / non-blocking
// buffer reads and writes, fills, copies, "images" (RGBA8 buffers), block(),
// raw_memory(), kernel objects and the profile mode.  Underneath it is one
// in-order HIP stream of libsrcnn_hip.so (include/srcnn.h); there is no
// OpenCL and no compiler at run time: a "kernel" is the descriptor of a
// gfx950 kernel family that the C ABI dispatches on.
#ifndef SRCNN_HOST_CONTEXT_HPP
#define SRCNN_HOST_CONTEXT_HPP

#include <cstddef>
#include <cstdint>
#include <cstring>
#include <ios>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "srcnn.h"

namespace srcnn {

/** Errors of file / JSON handling (reference: IOException, src/pch.hpp:80). */
typedef std::ios_base::failure IOException;

/** Throw std::runtime_error(msg) unless `cond` (reference utils::require). */
void require(bool cond, const std::string& msg);

/** Throw std::runtime_error with the C ABI's message unless rc == SRCNN_OK. */
void check(int rc, const char* what);

/** Index into Context's allocation table (reference: opencl::MemoryHandle). */
typedef size_t MemoryHandle;

/** "Not allocated" (reference: gpu_nullptr, src/DataPipeline.hpp:7). */
const MemoryHandle gpu_nullptr = MemoryHandle(1) << 30;

/** Allocation flags kept for signature compatibility (all memory is HBM). */
enum MemFlags : int { MEM_READ_WRITE = 1, MEM_READ_ONLY = 2, MEM_WRITE_ONLY = 4 };

/**
 * Completion token of an enqueued command.  Everything runs on one in-order
 * stream, so a token only needs to say how far the stream must drain:
 * waiting on any token = Context::wait() (the reference's cl_event waits are
 * all same-queue, src/opencl/Context.cpp:70-72).
 */
struct Event {
  uint64_t seq = 0;
};

/** Host image: w x h pixels of `bpp` bytes (reference opencl::utils::ImageData). */
struct ImageData {
  ImageData() = default;
  ImageData(int w_, int h_, int bpp_, const unsigned char* px = nullptr) : w(w_), h(h_), bpp(bpp_) {
    data.assign(static_cast<size_t>(w) * h * bpp, 0);
    if (px) std::memcpy(data.data(), px, data.size());
  }
  int w = 0, h = 0, bpp = 0;
  std::vector<unsigned char> data;
};

/** One device allocation (reference RawMemoryHandle, Context.hpp:53-68). */
struct RawMemoryHandle {
  void* ptr = nullptr;
  size_t size = 0;
  /** nonzero for images (bytes per pixel) */
  size_t bpp = 0;
  /** sub-range of another allocation: not freed on its own */
  bool is_view = false;
  MemoryHandle parent = gpu_nullptr;

  void release();
  inline bool is_usable() const { return !released; }
  inline bool is_image() const { return bpp != 0; }

 private:
  friend class Context;
  bool released = true;
};

/** Kernel families the pipeline dispatches (the reference's .cl programs). */
enum class KernelKind {
  Layer,        // layer_uber_kernel.cl  -> srcnn_conv_fwd
  Deltas,       // layer_deltas.cl       -> srcnn_conv_delta
  LastDelta,    // last_layer_delta.cl   -> srcnn_last_delta
  Backprop,     // backpropagate.cl      -> srcnn_conv_grad_acc
  Update,       // update_parameters.cl  -> srcnn_sgd_update
  SquaredError, // squared_error.cl      -> srcnn_sq_err
  Sum,          // sum.cl                -> srcnn_sum
  SubFromAll,   // subtract_from_all.cl  -> srcnn_sub_scalar
  Luma,         // extract_luma.cl       -> srcnn_extract_luma
  SwapLuma,     // swap_luma.cl          -> srcnn_swap_luma
  Net,          // (no .cl: fused net-level step) -> srcnn_train_fwd_bwd / srcnn_forward / srcnn_update_all
  AllReduce     // (no reference kernel) -> srcnn_allreduce_grads (RCCL)
};

/**
 * A specialised kernel (reference opencl::Kernel created with -D macros,
 * src/DataPipeline.cpp:161-180): its family plus the compile-time shape the
 * reference baked in (CURRENT_FILTER_COUNT, PREVIOUS_FILTER_COUNT,
 * F_SPATIAL_SIZE, SKIP_RELU).  Launch counts and, in profile mode, device
 * time are accumulated per kernel object.
 */
class Kernel {
 public:
  Kernel(KernelKind kind, std::string name, size_t n_prev = 0, size_t n_cur = 0,
         size_t f = 0, bool skip_relu = false, std::string args = "");
  /** "'gfx950/<name>'[<args>]", the reference's "'<file>'[<-D args>]"
   * (src/opencl/Kernel.cpp:32-36), so profile.py's regex parses the profile
   * lines; args are the specialisation defines ("--" when there are none) */
  std::string get_human_identifier() const;
  /** the -D defines the reference would have compiled this kernel with */
  std::string compile_args() const;
  uint64_t get_total_execution_time() const;  // ns, profile mode only

  const KernelKind kind;
  const std::string name;
  const size_t n_prev, n_cur, f;
  const bool skip_relu;
  const std::string args;

 private:
  friend class Context;
  uint64_t launches_ = 0;
  double total_ms_ = 0.0;
};

class Context {
 public:
  Context();
  ~Context();
  Context(const Context&) = delete;
  Context& operator=(const Context&) = delete;

  /** Bind to HIP device `device` and create the stream (Context::init). */
  void init(bool profile = false, int device = 0);
  bool is_initialized() const { return _initialized; }
  bool is_running_profile_mode() const { return _profiling; }
  std::string device_name() const;
  void display_device_info() const;
  void print_app_memory_usage() const;

  /** Drain the stream (reference Context::block, clFinish). */
  void block();
  /** Wait for `ev` (same stream: drain). */
  void wait(const Event* ev, int count = 1);

  MemoryHandle allocate(int flags, size_t size);
  /** Handle to [offset, offset+size) of `parent` (no new memory). */
  MemoryHandle view(MemoryHandle parent, size_t offset, size_t size);
  /** RGBA8 image of w x h (reference create_image(CL_RGBA, CL_UNSIGNED_INT8)). */
  MemoryHandle create_image(int flags, size_t w, size_t h);
  RawMemoryHandle* raw_memory(MemoryHandle);
  /** Device pointer of a live allocation (throws for gpu_nullptr / released). */
  void* ptr(MemoryHandle);
  float* fptr(MemoryHandle h) { return static_cast<float*>(ptr(h)); }

  Event read_buffer(MemoryHandle, size_t offset, size_t size, void* dst, bool block,
                    const Event* es = nullptr, int event_count = 0);
  Event read_buffer(MemoryHandle, void* dst, bool block, const Event* es = nullptr,
                    int event_count = 0);
  Event write_buffer(MemoryHandle, size_t offset, size_t size, const void* src, bool block,
                     const Event* es = nullptr, int event_count = 0);
  Event write_buffer(MemoryHandle, const void* src, bool block, const Event* es = nullptr,
                     int event_count = 0);
  Event zeros_float(MemoryHandle, bool block, const Event* es = nullptr, int event_count = 0);
  Event fill_float(MemoryHandle, float, bool block, const Event* es = nullptr,
                   int event_count = 0);
  Event copy_buffer(MemoryHandle src, MemoryHandle dst, const Event* es = nullptr,
                    int event_count = 0);
  Event copy_buffer(MemoryHandle src, MemoryHandle dst, size_t dst_offset,
                    const Event* es = nullptr, int event_count = 0);
  Event write_image(MemoryHandle, const ImageData&, bool block, const Event* es = nullptr,
                    int event_count = 0);

  /** Kernel object owned by the context (reference create_kernel). */
  Kernel* create_kernel(KernelKind kind, const std::string& name, size_t n_prev = 0,
                        size_t n_cur = 0, size_t f = 0, bool skip_relu = false,
                        const std::string& args = "");
  /** Bracket one launch of `k` (counts; device time when profiling). */
  class Launch {
   public:
    Launch(Context& ctx, Kernel& k);
    ~Launch();
    Launch(const Launch&) = delete;
    Launch& operator=(const Launch&) = delete;

   private:
    Context& ctx_;
    Kernel& k_;
    srcnn_event_t a_ = nullptr, b_ = nullptr;
  };
  /** Token for the work enqueued so far. */
  Event mark();

  srcnn_stream_t stream() const { return _stream; }

 private:
  void _cleanup();
  void flush_profile();

  bool _initialized = false;
  bool _profiling = false;
  int _device = 0;
  srcnn_stream_t _stream = nullptr;
  uint64_t _seq = 0;
  std::vector<RawMemoryHandle> _allocations;
  std::vector<std::unique_ptr<Kernel>> _kernels;
  struct Pending {
    Kernel* k;
    srcnn_event_t a, b;
  };
  std::vector<Pending> _pending;
};

}  // namespace srcnn

#endif  // SRCNN_HOST_CONTEXT_HPP
