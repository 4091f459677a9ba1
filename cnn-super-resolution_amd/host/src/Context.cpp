// srcnn::Context over the C ABI of libsrcnn_hip.so (see Context.hpp).
#include "Context.hpp"

#include <cstring>
#include <iostream>

namespace srcnn {

void require(bool cond, const std::string& msg) {
  if (!cond) throw std::runtime_error(msg);
}

void check(int rc, const char* what) {
  if (rc == SRCNN_OK) return;
  std::string msg(what);
  msg += ": ";
  const char* e = srcnn_last_error();
  msg += e ? e : "unknown error";
  throw std::runtime_error(msg);
}

void RawMemoryHandle::release() {
  if (released) return;
  if (!is_view && ptr) srcnn_free(ptr);
  ptr = nullptr;
  released = true;
}

Kernel::Kernel(KernelKind k, std::string nm, size_t np, size_t nc, size_t ff, bool sr,
               std::string a)
    : kind(k), name(std::move(nm)), n_prev(np), n_cur(nc), f(ff), skip_relu(sr), args(std::move(a)) {}

std::string Kernel::compile_args() const {
  // the defines of src/DataPipeline.cpp:161-180 (layer / deltas kernels)
  if (kind == KernelKind::Layer && f > 0)
    return "-D CURRENT_FILTER_COUNT=" + std::to_string(n_cur) + " -D PREVIOUS_FILTER_COUNT=" +
           std::to_string(n_prev) + " -D F_SPATIAL_SIZE=" + std::to_string(f) +
           (skip_relu ? " -D SKIP_RELU" : "");
  if (kind == KernelKind::Deltas && n_cur > 0) return "-D CURRENT_FILTER_COUNT=" + std::to_string(n_cur);
  return args.empty() ? "--" : args;
}

std::string Kernel::get_human_identifier() const {
  return "'gfx950/" + name + "'[" + compile_args() + "]";
}

uint64_t Kernel::get_total_execution_time() const {
  return static_cast<uint64_t>(total_ms_ * 1e6);
}

Context::Context() = default;

Context::~Context() {
  try {
    _cleanup();
  } catch (...) {
  }
}

void Context::init(bool profile, int device) {
  if (_initialized) return;
  int n = 0;
  check(srcnn_device_count(&n), "srcnn_device_count");
  require(n > 0, "No HIP device found (expected an MI355X / gfx950)");
  require(device >= 0 && device < n, "Device index out of range");
  check(srcnn_set_device(device), "srcnn_set_device");
  check(srcnn_stream_create(&_stream), "srcnn_stream_create");
  _device = device;
  _profiling = profile;
  _initialized = true;
}

std::string Context::device_name() const {
  char buf[256] = {0};
  check(srcnn_device_name(buf, sizeof(buf)), "srcnn_device_name");
  return buf;
}

void Context::display_device_info() const {
  std::cout << "Device " << _device << ": " << device_name() << std::endl;
}

void Context::print_app_memory_usage() const {
  size_t total = 0, n = 0;
  for (auto& a : _allocations)
    if (a.is_usable() && !a.is_view) {
      total += a.size;
      ++n;
    }
  std::cout << "Device memory in use: " << n << " allocations, " << total << " bytes ("
            << (total >> 20) << " MB)" << std::endl;
}

void Context::_cleanup() {
  if (!_initialized) return;
  block();
  flush_profile();
  if (_profiling) {
    for (auto& k : _kernels) {
      auto ns = k->get_total_execution_time();
      std::cout << "Kernel " << k->get_human_identifier() << " total execution time: " << ns
                << "ns = " << (ns / 1e9) << "s" << std::endl;
    }
  }
  for (auto& a : _allocations) a.release();
  _allocations.clear();
  _kernels.clear();
  if (_stream) srcnn_stream_destroy(_stream);
  _stream = nullptr;
  _initialized = false;
}

void Context::block() {
  require(_initialized, "Context used before init()");
  check(srcnn_stream_sync(_stream), "block");
}

void Context::wait(const Event* ev, int count) {
  if (ev && count > 0) block();
}

Event Context::mark() { return Event{++_seq}; }

MemoryHandle Context::allocate(int, size_t size) {
  require(_initialized, "Context used before init()");
  RawMemoryHandle h;
  check(srcnn_malloc(&h.ptr, size ? size : 4), "allocate");
  h.size = size;
  h.released = false;
  _allocations.push_back(h);
  return _allocations.size() - 1;
}

MemoryHandle Context::view(MemoryHandle parent, size_t offset, size_t size) {
  RawMemoryHandle* p = raw_memory(parent);
  require(p->is_usable(), "view of a released allocation");
  require(offset + size <= p->size, "view out of the parent allocation");
  RawMemoryHandle h;
  h.ptr = static_cast<char*>(p->ptr) + offset;
  h.size = size;
  h.is_view = true;
  h.parent = parent;
  h.released = false;
  _allocations.push_back(h);
  return _allocations.size() - 1;
}

MemoryHandle Context::create_image(int flags, size_t w, size_t h) {
  MemoryHandle m = allocate(flags, w * h * 4);
  _allocations[m].bpp = 4;
  return m;
}

RawMemoryHandle* Context::raw_memory(MemoryHandle h) {
  require(h < _allocations.size(), "Invalid memory handle");
  return &_allocations[h];
}

void* Context::ptr(MemoryHandle h) {
  RawMemoryHandle* r = raw_memory(h);
  require(r->is_usable(), "Memory handle was released");
  return r->ptr;
}

Event Context::read_buffer(MemoryHandle h, size_t offset, size_t size, void* dst, bool blk,
                           const Event* es, int n) {
  wait(es, n);
  RawMemoryHandle* r = raw_memory(h);
  require(offset + size <= r->size, "read_buffer out of bounds");
  // the C ABI's device->host copy is blocking (pageable host memory)
  check(srcnn_memcpy_d2h(dst, static_cast<char*>(ptr(h)) + offset, size, _stream), "read_buffer");
  (void)blk;
  return mark();
}

Event Context::read_buffer(MemoryHandle h, void* dst, bool blk, const Event* es, int n) {
  return read_buffer(h, 0, raw_memory(h)->size, dst, blk, es, n);
}

Event Context::write_buffer(MemoryHandle h, size_t offset, size_t size, const void* src,
                            bool blk, const Event* es, int n) {
  wait(es, n);
  RawMemoryHandle* r = raw_memory(h);
  require(offset + size <= r->size, "write_buffer out of bounds");
  check(srcnn_memcpy_h2d(static_cast<char*>(ptr(h)) + offset, src, size, _stream), "write_buffer");
  (void)blk;
  return mark();
}

Event Context::write_buffer(MemoryHandle h, const void* src, bool blk, const Event* es, int n) {
  return write_buffer(h, 0, raw_memory(h)->size, src, blk, es, n);
}

Event Context::zeros_float(MemoryHandle h, bool blk, const Event* es, int n) {
  return fill_float(h, 0.0f, blk, es, n);
}

Event Context::fill_float(MemoryHandle h, float v, bool blk, const Event* es, int n) {
  wait(es, n);
  check(srcnn_fill_f32(fptr(h), v, raw_memory(h)->size / sizeof(float), _stream), "fill_float");
  if (blk) block();
  return mark();
}

Event Context::copy_buffer(MemoryHandle src, MemoryHandle dst, const Event* es, int n) {
  return copy_buffer(src, dst, 0, es, n);
}

Event Context::copy_buffer(MemoryHandle src, MemoryHandle dst, size_t dst_offset, const Event* es,
                           int n) {
  wait(es, n);
  size_t bytes = raw_memory(src)->size;
  require(dst_offset + bytes <= raw_memory(dst)->size,
          "copy_buffer: destination smaller than offset + source size");
  check(srcnn_memcpy_d2d(static_cast<char*>(ptr(dst)) + dst_offset, ptr(src), bytes, _stream),
        "copy_buffer");
  return mark();
}

Event Context::write_image(MemoryHandle h, const ImageData& img, bool blk, const Event* es,
                           int n) {
  require(img.w > 0 && img.h > 0, "write_image: empty image");
  require(raw_memory(h)->size >= size_t(img.w) * img.h * 4, "write_image: image too small");
  if (img.bpp == 4) return write_buffer(h, 0, size_t(img.w) * img.h * 4, img.data.data(), blk, es, n);
  require(img.bpp == 3 || img.bpp == 1, "write_image: expected 1, 3 or 4 channels");
  std::vector<unsigned char> rgba(size_t(img.w) * img.h * 4);
  for (size_t i = 0, np = size_t(img.w) * img.h; i < np; ++i) {
    for (int c = 0; c < 3; ++c) rgba[4 * i + c] = img.data[i * img.bpp + (img.bpp == 3 ? c : 0)];
    rgba[4 * i + 3] = 255;
  }
  return write_buffer(h, 0, rgba.size(), rgba.data(), true, es, n);
}

Kernel* Context::create_kernel(KernelKind kind, const std::string& name, size_t n_prev,
                               size_t n_cur, size_t f, bool skip_relu, const std::string& args) {
  _kernels.emplace_back(new Kernel(kind, name, n_prev, n_cur, f, skip_relu, args));
  return _kernels.back().get();
}

Context::Launch::Launch(Context& ctx, Kernel& k) : ctx_(ctx), k_(k) {
  ++k_.launches_;
  if (!ctx_._profiling) return;
  check(srcnn_event_create(&a_), "event_create");
  check(srcnn_event_create(&b_), "event_create");
  check(srcnn_event_record(a_, ctx_._stream), "event_record");
}

Context::Launch::~Launch() {
  if (!a_) return;
  srcnn_event_record(b_, ctx_._stream);
  ctx_._pending.push_back({&k_, a_, b_});
  if (ctx_._pending.size() > 4096) ctx_.flush_profile();
}

void Context::flush_profile() {
  for (auto& p : _pending) {
    float ms = 0.f;
    if (srcnn_event_sync(p.b) == SRCNN_OK && srcnn_event_elapsed_ms(p.a, p.b, &ms) == SRCNN_OK)
      p.k->total_ms_ += ms;
    srcnn_event_destroy(p.a);
    srcnn_event_destroy(p.b);
  }
  _pending.clear();
}

}  // namespace srcnn
