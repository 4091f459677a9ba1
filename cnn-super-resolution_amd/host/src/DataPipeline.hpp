// cnn_sr::DataPipeline -- validated launchers of the SRCNN operators.
//
// Drop-in for the reference's DataPipeline (src/DataPipeline.hpp:39-222):
// same method names, argument order and meaning, same lazy-allocation
// contract (an output handle that is gpu_nullptr is allocated at the exact
// size; a too-small one throws instead of being reallocated,
// src/DataPipeline.cpp:66-86), same runtime_error checks.  Each launcher is
// one call into libsrcnn_hip.so (include/srcnn.h) on the context's stream;
// cl_event becomes srcnn::Event.
#ifndef CNN_SR_DATA_PIPELINE_HPP
#define CNN_SR_DATA_PIPELINE_HPP

#include "Context.hpp"
#include "LayerData.hpp"

namespace cnn_sr {

using srcnn::Event;
using srcnn::ImageData;
using srcnn::Kernel;
using srcnn::MemoryHandle;
using srcnn::gpu_nullptr;

/** Device handles of one layer (reference src/DataPipeline.hpp:11-29). */
struct LayerAllocationPool {
  MemoryHandle weights = gpu_nullptr;                 // f*f*n_prev*n_cur
  MemoryHandle bias = gpu_nullptr;                    // n_cur
  MemoryHandle accumulating_grad_w = gpu_nullptr;     // sum over the batch
  MemoryHandle accumulating_grad_b = gpu_nullptr;
  MemoryHandle previous_batch_delta_w = gpu_nullptr;  // momentum state
  MemoryHandle previous_batch_delta_b = gpu_nullptr;
};

class DataPipeline {
 public:
  static int LOAD_KERNEL_LUMA;
  static int LOAD_KERNEL_LAYERS;
  static int LOAD_KERNEL_BACKPROPAGATE;
  static int LOAD_KERNEL_MISC;
  static int LOAD_KERNEL_NONE;
  static int LOAD_KERNEL_ALL;

  explicit DataPipeline(srcnn::Context*);
  virtual ~DataPipeline() {}
  virtual void init(int load_flags = DataPipeline::LOAD_KERNEL_ALL);
  srcnn::Context* context();

  /** Upload `img` as an RGBA image to raw_img and its luma (optionally /255)
   * to luma (reference :186-220). */
  Event extract_luma(ImageData&, MemoryHandle& gpu_buf_raw_img, MemoryHandle& gpu_buf_luma,
                     bool normalize, Event* ev = nullptr);

  /** RGB (3 bytes/px) image made of the new luma (centre new_luma_w x
   * new_luma_h) and the CbCr of `img` (reference :222-266). */
  Event swap_luma(ImageData&, MemoryHandle& gpu_buf_org_img, MemoryHandle gpu_buf_new_luma,
                  MemoryHandle& target, size_t new_luma_w, size_t new_luma_h,
                  Event* ev = nullptr);

  /** Forward of one layer over `sample_count` samples (reference :358-410). */
  Event execute_layer(Kernel&, const LayerData&, LayerAllocationPool&, MemoryHandle& gpu_buf_in,
                      size_t input_w, size_t input_h, size_t sample_count,
                      MemoryHandle& gpu_buf_out, Event* ev = nullptr);

  /** Sum of squared differences between the result and the ground-truth
   * centre; the value lands in `target` (reference :416-472). */
  Event squared_error(MemoryHandle gpu_buf_ground_truth, size_t ground_truth_w,
                      size_t ground_truth_h, size_t sample_count, MemoryHandle gpu_buf_algo_res,
                      MemoryHandle tmp_buffer, float& target, size_t total_padding,
                      Event* ev = nullptr);

  /** delta3 = (y - gt_centre) * [y > 0] (reference :474-520). */
  Event last_layer_delta(MemoryHandle gpu_buf_ground_truth, size_t ground_truth_w,
                         size_t ground_truth_h, size_t sample_count,
                         MemoryHandle gpu_buf_algo_res, MemoryHandle& gpu_buf_target,
                         size_t total_padding, Event* ev = nullptr);

  /** Deltas of `curr_layer` from the next layer's deltas (reference :522-594). */
  Event calculate_deltas(Kernel&, const LayerData& curr_layer, const LayerData& next_layer,
                         LayerAllocationPool& next_gpu_alloc, MemoryHandle curr_deltas,
                         MemoryHandle next_deltas, size_t next_layer_out_w,
                         size_t next_layer_out_h, size_t sample_count,
                         MemoryHandle curr_output, Event* ev = nullptr);

  /** Accumulate (+=) weight / bias gradients of one layer (reference
   * :596-663), summed race-free over samples. */
  Event backpropagate(LayerData&, MemoryHandle layer_input, MemoryHandle layer_deltas,
                      LayerAllocationPool&, size_t layer_out_w, size_t layer_out_h,
                      size_t sample_count, Event* ev = nullptr, size_t ev_cnt = 0);

  /** Momentum SGD with weight decay on one layer (reference :665-729). */
  Event update_parameters(LayerData&, LayerAllocationPool&, size_t batch_size, float momentum,
                          float w_decay, float learning_rate, Event* ev = nullptr);

  /** x -= mean(x); the mean is returned through `mean` (reference :268-280). */
  Event subtract_mean(MemoryHandle, float* mean = nullptr, Event* ev = nullptr);
  /** Blocking sum of all floats of the buffer, optionally squared (:282-313). */
  float sum(MemoryHandle, bool squared = false, Event* ev = nullptr);
  /** x -= value (reference :315-333). */
  Event subtract_from_all(MemoryHandle, float, Event* ev = nullptr);

  Kernel* create_layer_kernel(const LayerData&, bool skip_relu);
  Kernel* create_deltas_kernel(const LayerData&);

  void print_buffer(MemoryHandle, const char* name, size_t lines);

 protected:
  void check_initialized(int kernel_load_flags);
  virtual void load_kernels(int load_flags);
  bool allocation_has_right_size__(MemoryHandle, size_t, size_t line, const char* name);
  size_t element_count(MemoryHandle, size_t el_size);
  /** device scratch of at least `bytes` (grown on demand, stream-ordered) */
  void* scratch(size_t bytes);
  /** reduction workspace (second scratch: may be used beside scratch()) */
  void* reduce_scratch(size_t bytes);

  srcnn::Context* const _context;
  bool _initialized;
  int _loaded = 0;

  /** Single float. */
  MemoryHandle _tmp_gpu_float = gpu_nullptr;
  MemoryHandle _scratch = gpu_nullptr;
  MemoryHandle _reduce_scratch = gpu_nullptr;

  Kernel* _luma_kernel_norm = nullptr;
  Kernel* _luma_kernel_raw = nullptr;
  Kernel* _swap_luma_kernel = nullptr;
  Kernel* _squared_error_kernel = nullptr;
  Kernel* _sum_kernel = nullptr;
  Kernel* _sum_squared_kernel = nullptr;
  Kernel* _subtract_from_all_kernel = nullptr;
  Kernel* _last_layer_delta_kernel = nullptr;
  Kernel* _update_parameters_kernel = nullptr;
  Kernel* _backpropagate_kernel = nullptr;

 private:
  void pre_execute_layer_validation(const LayerData&, MemoryHandle, size_t, size_t);
};

}  // namespace cnn_sr

#endif  // CNN_SR_DATA_PIPELINE_HPP
