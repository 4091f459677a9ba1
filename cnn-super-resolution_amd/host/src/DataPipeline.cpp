#include "DataPipeline.hpp"

#include <iomanip>
#include <iostream>
#include <string>
#include <vector>

namespace cnn_sr {

using srcnn::check;
using srcnn::require;

int DataPipeline::LOAD_KERNEL_LUMA = 1;
int DataPipeline::LOAD_KERNEL_LAYERS = 2;
int DataPipeline::LOAD_KERNEL_MISC = 4;
int DataPipeline::LOAD_KERNEL_BACKPROPAGATE = 8;
int DataPipeline::LOAD_KERNEL_NONE = 0;
int DataPipeline::LOAD_KERNEL_ALL = 1 | 2 | 4 | 8;

#define SRCNN_HAS_SIZE(H, BYTES) allocation_has_right_size__((H), (BYTES), __LINE__, #H)

DataPipeline::DataPipeline(srcnn::Context* ctx) : _context(ctx), _initialized(false) {}

void DataPipeline::init(int load_flags) {
  require(_context && _context->is_initialized(), "DataPipeline needs an initialized Context");
  load_kernels(load_flags);
  _initialized = true;
}

srcnn::Context* DataPipeline::context() { return _context; }

void DataPipeline::check_initialized(int flags) {
  if (!_initialized) throw std::runtime_error("Tried to use DataPipeline before it was initialized");
  load_kernels(flags);
}

void DataPipeline::load_kernels(int flags) {
  using srcnn::KernelKind;
  auto& c = *_context;
  if ((flags & LOAD_KERNEL_LUMA) && !_luma_kernel_norm) {
    // names / defines of the reference's kernels (src/DataPipeline.cpp:121-159)
    _luma_kernel_norm = c.create_kernel(KernelKind::Luma, "extract_luma", 0, 0, 0, false, "-D NORMALIZE");
    _luma_kernel_raw = c.create_kernel(KernelKind::Luma, "extract_luma");
    _swap_luma_kernel = c.create_kernel(KernelKind::SwapLuma, "swap_luma");
  }
  if ((flags & LOAD_KERNEL_MISC) && !_sum_kernel) {
    _squared_error_kernel = c.create_kernel(KernelKind::SquaredError, "squared_error");
    _sum_kernel = c.create_kernel(KernelKind::Sum, "sum");
    _sum_squared_kernel = c.create_kernel(KernelKind::Sum, "sum", 0, 0, 0, false, "-D SUM_SQUARED");
    _subtract_from_all_kernel = c.create_kernel(KernelKind::SubFromAll, "subtract_from_all");
  }
  if ((flags & LOAD_KERNEL_BACKPROPAGATE) && !_backpropagate_kernel) {
    _last_layer_delta_kernel = c.create_kernel(KernelKind::LastDelta, "last_layer_delta");
    _update_parameters_kernel = c.create_kernel(KernelKind::Update, "update_parameters");
    _backpropagate_kernel = c.create_kernel(KernelKind::Backprop, "backpropagate");
  }
  _loaded |= flags;
}

bool DataPipeline::allocation_has_right_size__(MemoryHandle h, size_t size, size_t line,
                                               const char* name) {
  if (h == gpu_nullptr) return false;
  auto* raw = _context->raw_memory(h);
  if (raw->is_usable() && raw->size >= size) return true;
  std::cout << "Was forced to reallocate gpu buffer. Set the MemoryHandle to gpu_nullptr to let "
               "DataPipeline allocate it at the right size. Expected: "
            << size << ", got: " << raw->size << ". Code line: " << line << ", variable: '"
            << name << "'" << std::endl;
  throw std::runtime_error("Was forced to realocate gpu buffer due too difference in sizes.");
}

size_t DataPipeline::element_count(MemoryHandle h, size_t el) {
  return _context->raw_memory(h)->size / el;
}

void* DataPipeline::scratch(size_t bytes) {
  bytes = bytes ? bytes : 4;
  if (_scratch != gpu_nullptr && _context->raw_memory(_scratch)->size < bytes) {
    _context->block();
    _context->raw_memory(_scratch)->release();
    _scratch = gpu_nullptr;
  }
  if (_scratch == gpu_nullptr) _scratch = _context->allocate(srcnn::MEM_READ_WRITE, bytes);
  return _context->ptr(_scratch);
}

void* DataPipeline::reduce_scratch(size_t bytes) {
  bytes = bytes ? bytes : 4;
  if (_reduce_scratch != gpu_nullptr && _context->raw_memory(_reduce_scratch)->size < bytes) {
    _context->block();
    _context->raw_memory(_reduce_scratch)->release();
    _reduce_scratch = gpu_nullptr;
  }
  if (_reduce_scratch == gpu_nullptr)
    _reduce_scratch = _context->allocate(srcnn::MEM_READ_WRITE, bytes);
  return _context->ptr(_reduce_scratch);
}

void DataPipeline::print_buffer(MemoryHandle h, const char* name, size_t lines) {
  size_t len = element_count(h, sizeof(float));
  std::vector<float> v(len);
  _context->block();
  _context->read_buffer(h, v.data(), true);
  size_t per = lines ? (len + lines - 1) / lines : len;
  std::cout << name << ": [" << std::endl;
  for (size_t i = 0; i < len; ++i) {
    std::cout << std::setw(9) << std::setprecision(4) << v[i] << ((i + 1) % per ? ", " : ",\n");
  }
  std::cout << "]" << std::endl << std::endl;
}

Kernel* DataPipeline::create_layer_kernel(const LayerData& d, bool skip_relu) {
  return _context->create_kernel(srcnn::KernelKind::Layer, "layer_uber_kernel", d.n_prev_filter_cnt,
                                 d.current_filter_count, d.f_spatial_size, skip_relu);
}

Kernel* DataPipeline::create_deltas_kernel(const LayerData& d) {
  return _context->create_kernel(srcnn::KernelKind::Deltas, "layer_deltas", d.n_prev_filter_cnt,
                                 d.current_filter_count, d.f_spatial_size);
}

// ---------------------------------------------------------------- luma / misc

Event DataPipeline::extract_luma(ImageData& img, MemoryHandle& raw_img, MemoryHandle& luma,
                                 bool normalize, Event* ev) {
  check_initialized(LOAD_KERNEL_LUMA);
  _context->wait(ev);
  size_t px = size_t(img.w) * img.h;
  if (!SRCNN_HAS_SIZE(raw_img, px * 4)) raw_img = _context->create_image(srcnn::MEM_READ_WRITE, img.w, img.h);
  _context->write_image(raw_img, img, true);
  if (!SRCNN_HAS_SIZE(luma, px * sizeof(float)))
    luma = _context->allocate(srcnn::MEM_READ_WRITE, px * sizeof(float));
  Kernel& k = normalize ? *_luma_kernel_norm : *_luma_kernel_raw;
  srcnn::Context::Launch l(*_context, k);
  check(srcnn_extract_luma(static_cast<const uint8_t*>(_context->ptr(raw_img)), _context->fptr(luma),
                           img.w, img.h, normalize ? 1 : 0, _context->stream()),
        "extract_luma");
  return _context->mark();
}

Event DataPipeline::swap_luma(ImageData& img, MemoryHandle& org_img, MemoryHandle new_luma,
                              MemoryHandle& target, size_t luma_w, size_t luma_h, Event* ev) {
  check_initialized(LOAD_KERNEL_LUMA);
  _context->wait(ev);
  size_t px = size_t(img.w) * img.h;
  if (!SRCNN_HAS_SIZE(new_luma, luma_w * luma_h * sizeof(float)))
    throw std::runtime_error("Invalid size of new luma buffer");
  require(luma_w <= size_t(img.w) && luma_h <= size_t(img.h), "new luma bigger than the image");
  if (!SRCNN_HAS_SIZE(target, px * 3)) target = _context->allocate(srcnn::MEM_READ_WRITE, px * 3);
  if (!SRCNN_HAS_SIZE(org_img, px * 4)) org_img = _context->create_image(srcnn::MEM_READ_WRITE, img.w, img.h);
  _context->write_image(org_img, img, true);
  srcnn::Context::Launch l(*_context, *_swap_luma_kernel);
  check(srcnn_swap_luma(static_cast<const uint8_t*>(_context->ptr(org_img)), _context->fptr(new_luma),
                        static_cast<uint8_t*>(_context->ptr(target)), img.w, img.h, luma_w, luma_h,
                        _context->stream()),
        "swap_luma");
  return _context->mark();
}

float DataPipeline::sum(MemoryHandle data, bool squared, Event* ev) {
  check_initialized(LOAD_KERNEL_MISC);
  _context->wait(ev);
  size_t len = element_count(data, sizeof(float));
  if (!SRCNN_HAS_SIZE(_tmp_gpu_float, sizeof(float)))
    _tmp_gpu_float = _context->allocate(srcnn::MEM_READ_WRITE, sizeof(float));
  size_t ws = srcnn_reduce_workspace_bytes(len);
  void* w = reduce_scratch(ws);
  {
    srcnn::Context::Launch l(*_context, squared ? *_sum_squared_kernel : *_sum_kernel);
    check(srcnn_sum(_context->fptr(data), len, squared ? 1 : 0, _context->fptr(_tmp_gpu_float), w, ws,
                    _context->stream()),
          "sum");
  }
  float result = 0.f;
  _context->read_buffer(_tmp_gpu_float, 0, sizeof(float), &result, true);
  return result;
}

Event DataPipeline::subtract_from_all(MemoryHandle data, float v, Event* ev) {
  check_initialized(LOAD_KERNEL_MISC);
  _context->wait(ev);
  srcnn::Context::Launch l(*_context, *_subtract_from_all_kernel);
  check(srcnn_sub_scalar(_context->fptr(data), v, element_count(data, sizeof(float)), _context->stream()),
        "subtract_from_all");
  return _context->mark();
}

Event DataPipeline::subtract_mean(MemoryHandle data, float* mean, Event* ev) {
  check_initialized(LOAD_KERNEL_MISC);
  float s = sum(data, false, ev);  // blocking, as the reference
  float m = s / static_cast<float>(element_count(data, sizeof(float)));
  if (mean) *mean = m;
  return subtract_from_all(data, m);
}

// ---------------------------------------------------------------- forward

void DataPipeline::pre_execute_layer_validation(const LayerData& d, MemoryHandle in, size_t w,
                                                size_t h) {
  LayerData::validate(d);
  require(in != gpu_nullptr, "Layer input buffer is not allocated");
  size_t expected = d.input_size(w, h), cnt = element_count(in, sizeof(float));
  if (expected > cnt) {
    throw std::runtime_error("Declared input_w(" + std::to_string(w) + ")*input_h(" +
                             std::to_string(h) + ")*n_prev_filter_cnt(" +
                             std::to_string(d.n_prev_filter_cnt) + ")=" + std::to_string(expected) +
                             " is bigger then allocated gpu memory (" + std::to_string(cnt) +
                             " elements).");
  }
}

Event DataPipeline::execute_layer(Kernel& kernel, const LayerData& d, LayerAllocationPool& a,
                                  MemoryHandle& in, size_t w, size_t h, size_t n,
                                  MemoryHandle& out, Event* ev) {
  check_initialized(LOAD_KERNEL_LAYERS);
  pre_execute_layer_validation(d, in, w, h);
  require(kernel.kind == srcnn::KernelKind::Layer, "execute_layer needs a layer kernel");
  require(kernel.n_prev == d.n_prev_filter_cnt && kernel.n_cur == d.current_filter_count &&
              kernel.f == d.f_spatial_size,
          "Kernel was created for a different layer shape");
  require(w >= d.f_spatial_size && h >= d.f_spatial_size, "Input smaller than the filter");
  require(d.input_size(w, h) * n <= element_count(in, sizeof(float)),
          "Input buffer smaller than sample_count samples");
  _context->wait(ev);
  size_t od[2];
  d.get_output_dimensions(od, w, h);
  size_t out_bytes = sizeof(float) * od[0] * od[1] * d.current_filter_count * n;
  if (!SRCNN_HAS_SIZE(a.weights, sizeof(float) * d.weight_size())) {
    a.weights = _context->allocate(srcnn::MEM_READ_WRITE, sizeof(float) * d.weight_size());
    _context->write_buffer(a.weights, 0, sizeof(float) * d.weight_size(), d.weights_ptr(), true);
  }
  if (!SRCNN_HAS_SIZE(a.bias, sizeof(float) * d.bias_size())) {
    a.bias = _context->allocate(srcnn::MEM_READ_WRITE, sizeof(float) * d.bias_size());
    _context->write_buffer(a.bias, 0, sizeof(float) * d.bias_size(), d.bias_ptr(), true);
  }
  if (!SRCNN_HAS_SIZE(out, out_bytes)) out = _context->allocate(srcnn::MEM_READ_WRITE, out_bytes);
  srcnn::Context::Launch l(*_context, kernel);
  check(srcnn_conv_fwd(_context->fptr(in), _context->fptr(out), _context->fptr(a.weights),
                       _context->fptr(a.bias), w, h, d.n_prev_filter_cnt, d.current_filter_count,
                       d.f_spatial_size, kernel.skip_relu ? 0 : 1, n, _context->stream()),
        "execute_layer");
  return _context->mark();
}

// ---------------------------------------------------------------- backward

Event DataPipeline::squared_error(MemoryHandle gt, size_t gt_w, size_t gt_h, size_t n,
                                  MemoryHandle algo, MemoryHandle tmp, float& target,
                                  size_t padding, Event* ev) {
  check_initialized(LOAD_KERNEL_MISC);
  require(gt_w > padding && gt_h > padding, "padding larger than the ground truth");
  size_t aw = gt_w - padding, ah = gt_h - padding;
  if (!SRCNN_HAS_SIZE(algo, sizeof(float) * aw * ah))
    throw std::runtime_error("Allocated gpu_buf_algo_res buffer size did not match calculated size");
  require(element_count(algo, sizeof(float)) >= aw * ah * n, "algo result smaller than sample_count samples");
  require(element_count(gt, sizeof(float)) >= gt_w * gt_h * n, "ground truth smaller than sample_count samples");
  if (tmp == gpu_nullptr) {
    if (!SRCNN_HAS_SIZE(_tmp_gpu_float, sizeof(float)))
      _tmp_gpu_float = _context->allocate(srcnn::MEM_READ_WRITE, sizeof(float));
    tmp = _tmp_gpu_float;
  }
  require(_context->raw_memory(tmp)->size >= sizeof(float), "tmp buffer must hold one float");
  _context->wait(ev);
  size_t ws = srcnn_reduce_workspace_bytes(aw * ah * n);
  void* w = reduce_scratch(ws);
  {
    srcnn::Context::Launch l(*_context, *_squared_error_kernel);
    check(srcnn_sq_err(_context->fptr(gt), _context->fptr(algo), _context->fptr(tmp), gt_w, gt_h, aw,
                       ah, n, w, ws, _context->stream()),
          "squared_error");
  }
  return _context->read_buffer(tmp, 0, sizeof(float), &target, true);
}

Event DataPipeline::last_layer_delta(MemoryHandle gt, size_t gt_w, size_t gt_h, size_t n,
                                     MemoryHandle algo, MemoryHandle& target, size_t padding,
                                     Event* ev) {
  check_initialized(LOAD_KERNEL_BACKPROPAGATE);
  require(gt_w > padding && gt_h > padding, "padding larger than the ground truth");
  size_t aw = gt_w - padding, ah = gt_h - padding;
  if (!SRCNN_HAS_SIZE(algo, sizeof(float) * aw * ah))
    throw std::runtime_error("Allocated gpu_buf_algo_res buffer size did not match calculated size");
  require(element_count(algo, sizeof(float)) >= aw * ah * n, "algo result smaller than sample_count samples");
  require(element_count(gt, sizeof(float)) >= gt_w * gt_h * n, "ground truth smaller than sample_count samples");
  if (!SRCNN_HAS_SIZE(target, sizeof(float) * aw * ah * n))
    target = _context->allocate(srcnn::MEM_READ_WRITE, sizeof(float) * aw * ah * n);
  _context->wait(ev);
  srcnn::Context::Launch l(*_context, *_last_layer_delta_kernel);
  check(srcnn_last_delta(_context->fptr(gt), _context->fptr(algo), _context->fptr(target), gt_w, gt_h,
                         aw, ah, n, _context->stream()),
        "last_layer_delta");
  return _context->mark();
}

Event DataPipeline::calculate_deltas(Kernel& kernel, const LayerData& curr, const LayerData& next,
                                     LayerAllocationPool& next_alloc, MemoryHandle curr_deltas,
                                     MemoryHandle next_deltas, size_t next_w, size_t next_h,
                                     size_t n, MemoryHandle curr_output, Event* ev) {
  check_initialized(LOAD_KERNEL_BACKPROPAGATE);
  LayerData::validate(next);
  if (curr.current_filter_count != next.n_prev_filter_cnt) {
    throw std::runtime_error(
        "When calculating deltas for layer it's filter count should be equal to next layer's "
        "previous filter count");
  }
  require(kernel.kind == srcnn::KernelKind::Deltas, "calculate_deltas needs a deltas kernel");
  size_t cw = next_w + next.f_spatial_size - 1, ch = next_h + next.f_spatial_size - 1;
  size_t out_bytes = sizeof(float) * cw * ch * next.n_prev_filter_cnt;
  if (!SRCNN_HAS_SIZE(next_alloc.weights, sizeof(float) * next.weight_size())) {
    next_alloc.weights = _context->allocate(srcnn::MEM_READ_WRITE, sizeof(float) * next.weight_size());
    _context->write_buffer(next_alloc.weights, 0, sizeof(float) * next.weight_size(), next.weights_ptr(), true);
  }
  if (!SRCNN_HAS_SIZE(curr_output, out_bytes)) {
    throw std::runtime_error(
        "Tried to calculate deltas for previous layer, but there are no previous layer output "
        "values.They are normally allocated during forward step.");
  }
  require(curr_deltas != gpu_nullptr && element_count(curr_deltas, 4) >= cw * ch * next.n_prev_filter_cnt * n,
          "Target deltas buffer is not allocated or too small");
  require(next_deltas != gpu_nullptr &&
              element_count(next_deltas, 4) >= next_w * next_h * next.current_filter_count * n,
          "Next layer deltas buffer is not allocated or too small");
  require(element_count(curr_output, 4) >= cw * ch * next.n_prev_filter_cnt * n,
          "Previous layer output smaller than sample_count samples");
  _context->wait(ev);
  srcnn::Context::Launch l(*_context, kernel);
  check(srcnn_conv_delta(_context->fptr(next_deltas), _context->fptr(curr_output),
                         _context->fptr(curr_deltas), _context->fptr(next_alloc.weights),
                         next.f_spatial_size, next.n_prev_filter_cnt, next.current_filter_count, cw,
                         ch, n, _context->stream()),
        "calculate_deltas");
  return _context->mark();
}

Event DataPipeline::backpropagate(LayerData& d, MemoryHandle input, MemoryHandle deltas,
                                  LayerAllocationPool& a, size_t ow, size_t oh, size_t n,
                                  Event* ev, size_t ev_cnt) {
  LayerData::validate(d);
  check_initialized(LOAD_KERNEL_BACKPROPAGATE);
  size_t iw = ow + d.f_spatial_size - 1, ih = oh + d.f_spatial_size - 1;
  size_t in_bytes = sizeof(float) * iw * ih * d.n_prev_filter_cnt;
  if (!SRCNN_HAS_SIZE(input, in_bytes)) {
    throw std::runtime_error(
        "Tried to calculate gradients, but there are no previous layer output values.They are "
        "normally allocated during forward step.");
  }
  require(element_count(input, 4) >= iw * ih * d.n_prev_filter_cnt * n,
          "Layer input smaller than sample_count samples");
  require(deltas != gpu_nullptr && element_count(deltas, 4) >= ow * oh * d.current_filter_count * n,
          "Tried to calculate gradients, but deltas for current layer are not valid");
  if (!SRCNN_HAS_SIZE(a.accumulating_grad_w, sizeof(float) * d.weight_size())) {
    a.accumulating_grad_w = _context->allocate(srcnn::MEM_READ_WRITE, sizeof(float) * d.weight_size());
    _context->zeros_float(a.accumulating_grad_w, false);
  }
  if (!SRCNN_HAS_SIZE(a.accumulating_grad_b, sizeof(float) * d.bias_size())) {
    a.accumulating_grad_b = _context->allocate(srcnn::MEM_READ_WRITE, sizeof(float) * d.bias_size());
    _context->zeros_float(a.accumulating_grad_b, false);
  }
  _context->wait(ev, ev ? (ev_cnt ? int(ev_cnt) : 1) : 0);
  size_t ws = srcnn_conv_grad_workspace_bytes(d.n_prev_filter_cnt, d.current_filter_count,
                                              d.f_spatial_size, ow, oh, n);
  void* w = scratch(ws);
  srcnn::Context::Launch l(*_context, *_backpropagate_kernel);
  check(srcnn_conv_grad_acc(_context->fptr(input), _context->fptr(deltas),
                            _context->fptr(a.accumulating_grad_w), _context->fptr(a.accumulating_grad_b),
                            d.n_prev_filter_cnt, d.current_filter_count, d.f_spatial_size, ow, oh, n,
                            w, ws, _context->stream()),
        "backpropagate");
  return _context->mark();
}

Event DataPipeline::update_parameters(LayerData& d, LayerAllocationPool& a, size_t batch,
                                      float momentum, float wd, float lr, Event* ev) {
  LayerData::validate(d);
  check_initialized(LOAD_KERNEL_BACKPROPAGATE);
  size_t wb = sizeof(float) * d.weight_size(), bb = sizeof(float) * d.bias_size();
  if (!SRCNN_HAS_SIZE(a.weights, wb))
    throw std::runtime_error("Tried to update weights, but old values are not valid. Impossible if forward pass was completed");
  if (!SRCNN_HAS_SIZE(a.bias, bb))
    throw std::runtime_error("Tried to update bias, but old values are not valid. Impossible if forward pass was completed");
  if (!SRCNN_HAS_SIZE(a.accumulating_grad_w, wb))
    throw std::runtime_error("Tried to update weights, but gradient values are not valid. Impossible if backpropagation was completed");
  if (!SRCNN_HAS_SIZE(a.accumulating_grad_b, bb))
    throw std::runtime_error("Tried to update bias, but gradient values are not valid. Impossible if backpropagation was completed");
  if (!SRCNN_HAS_SIZE(a.previous_batch_delta_w, wb)) {
    a.previous_batch_delta_w = _context->allocate(srcnn::MEM_READ_WRITE, wb);
    _context->zeros_float(a.previous_batch_delta_w, false);
  }
  if (!SRCNN_HAS_SIZE(a.previous_batch_delta_b, bb)) {
    a.previous_batch_delta_b = _context->allocate(srcnn::MEM_READ_WRITE, bb);
    _context->zeros_float(a.previous_batch_delta_b, false);
  }
  _context->wait(ev);
  srcnn::Context::Launch l(*_context, *_update_parameters_kernel);
  check(srcnn_sgd_update(_context->fptr(a.weights), _context->fptr(a.bias),
                         _context->fptr(a.accumulating_grad_w), _context->fptr(a.accumulating_grad_b),
                         _context->fptr(a.previous_batch_delta_w), _context->fptr(a.previous_batch_delta_b),
                         momentum, wd, lr, batch, d.weight_size(), d.bias_size(), _context->stream()),
        "update_parameters");
  return _context->mark();
}

}  // namespace cnn_sr
