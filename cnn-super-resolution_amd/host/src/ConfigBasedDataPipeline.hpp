// cnn_sr::ConfigBasedDataPipeline -- the three-layer SRCNN driven by a Config.
//
// Drop-in for the reference class (src/ConfigBasedDataPipeline.hpp:46-156):
// init() loads parameters.json or draws random parameters, execute_batch()
// runs forward + backpropagation (or forward + squared error) over a sample
// set in mini-batches, update_parameters() applies momentum SGD and zeroes
// the gradient accumulators, write_params_to_file() / write_result_image()
// save results.
//
// MI355X design: when the three LayerAllocationPools are left to the
// pipeline (all gpu_nullptr, the reference's normal use), the pipeline
// allocates ONE flat parameter buffer [W1|B1|W2|B2|W3|B3] (plus flat
// gradient and momentum buffers) and hands out views of it as the pools'
// handles.  A training chunk is then one srcnn_train_fwd_bwd call (the fused
// gfx950 kernels), the update one srcnn_update_all call, and the flat
// gradient buffer is what a data-parallel run all-reduces.  Pools that the
// caller allocated itself take the per-layer op-level path instead (same
// results; tests pin both).
#ifndef CNN_SR_CONFIG_BASED_DATA_PIPELINE_HPP
#define CNN_SR_CONFIG_BASED_DATA_PIPELINE_HPP

#include <cstdint>
#include <vector>

#include "Config.hpp"
#include "DataPipeline.hpp"

namespace cnn_sr {

/** Device buffers of one image (reference :12-31). */
struct SampleAllocationPool {
  MemoryHandle input_data = gpu_nullptr;  // RGBA image
  MemoryHandle input_luma = gpu_nullptr;  // w*h floats
  size_t input_w = 0, input_h = 0;
  MemoryHandle expected_data = gpu_nullptr;
  MemoryHandle expected_luma = gpu_nullptr;
  SampleAllocationPool() = default;
};

/** All allocations of a run (reference :34-40). */
struct GpuAllocationPool {
  LayerAllocationPool layer_1;
  LayerAllocationPool layer_2;
  LayerAllocationPool layer_3;
  std::vector<SampleAllocationPool> samples;
};

/** The one exchange step of data-parallel training (an extension; the
 * reference trains on one device): an in-place sum of `count` floats of device
 * memory over the ranks, ordered after the work already on `ctx`'s stream. */
class GradientExchange {
 public:
  virtual ~GradientExchange() = default;
  virtual void allreduce(srcnn::Context& ctx, float* buf, size_t count) = 0;
};

/** RCCL over xGMI: srcnn_allreduce_grads on the context's stream. */
class RcclExchange : public GradientExchange {
 public:
  explicit RcclExchange(srcnn_comm_t comm) : _comm(comm) {}
  void allreduce(srcnn::Context& ctx, float* buf, size_t count) override;

 private:
  srcnn_comm_t _comm;
};

class ConfigBasedDataPipeline : public DataPipeline {
 public:
  ConfigBasedDataPipeline(Config&, srcnn::Context*);

  void init(int load_flags = DataPipeline::LOAD_KERNEL_ALL) override;

  void set_mini_batch_size(size_t);
  size_t mini_batch_size() const { return _mini_batch_size; }

  /** Forward + (backpropagate ? gradient accumulation : squared error) over
   * all samples (same dims), in mini-batches; returns the summed squared
   * error of a validation run (0 for training). */
  float execute_batch(bool backpropagate, GpuAllocationPool&, std::vector<SampleAllocationPool*>&);

  /** Inference of one image; the result stays in result_buffer(). */
  Event forward(LayerAllocationPool&, LayerAllocationPool&, LayerAllocationPool&,
                SampleAllocationPool&);

  void update_parameters(LayerAllocationPool&, LayerAllocationPool&, LayerAllocationPool&,
                         size_t batch_size, Event* ev = nullptr);

  void write_params_to_file(const char* file_path, LayerAllocationPool, LayerAllocationPool,
                            LayerAllocationPool);

  void write_result_image(const char* out_path, ImageData& input_img, SampleAllocationPool&);

  const Config* config() const { return _config; }
  const LayerData* layer_1() const { return &layer_data_1; }
  const LayerData* layer_2() const { return &layer_data_2; }
  const LayerData* layer_3() const { return &layer_data_3; }

  // ---- extensions (not in the reference) ----
  /** seed the random initialisation (the reference seeds with the clock) */
  void set_random_seed(uint64_t seed) { _seed = seed; _seeded = true; }
  size_t epochs() const { return _epochs; }
  /** opt-in (the reference restarts momentum at zero on resume,
   * ConfigBasedDataPipeline.cpp:419-465): write_params_to_file() also stores
   * each layer's momentum ("momentum_weights" / "momentum_bias", keys the
   * reference's loader skips), and a parameters file that holds them resumes
   * the pipeline-owned momentum buffers from them */
  void set_save_momentum(bool on) { _save_momentum = on; }
  /** L3 output of the last forward / execute_batch chunk */
  MemoryHandle result_buffer() const { return _out_3_gpu_buf; }
  /** the flat [gW1|gB1|gW2|gB2|gW3|gB3] buffer (gpu_nullptr before training
   * on pipeline-owned pools): the one buffer a data-parallel run all-reduces */
  MemoryHandle flat_gradients() const { return _flat_grads; }
  MemoryHandle flat_parameters() const { return _flat_params; }
  srcnn_net net() const;

  /** Data-parallel extension (the reference is single-device): sum the
   * flat gradient buffer over the ranks in place, on this context's stream
   * (by default srcnn_allreduce_grads, RCCL over xGMI).  Call between
   * execute_batch(true, ...) on this rank's shard and update_parameters(...,
   * global training-set size).  The pools must be the pipeline's own flat
   * views (left unallocated by the caller; they are bound here if needed). */
  void allreduce_gradients(GpuAllocationPool&, GradientExchange& ex);
  void allreduce_gradients(GpuAllocationPool&, srcnn_comm_t comm);
  /** sum of one host float over the ranks (blocking) */
  float allreduce_sum(float value, GradientExchange& ex);
  float allreduce_sum(float value, srcnn_comm_t comm);

 protected:
  void load_kernels(int load_flags) override;

 private:
  void allocate_buffers(size_t w, size_t h);
  /** make the pools views of the flat buffers if they are unallocated;
   * true when the pools are the pipeline's flat views */
  bool bind_flat(LayerAllocationPool&, LayerAllocationPool&, LayerAllocationPool&);
  Event forward(LayerAllocationPool&, LayerAllocationPool&, LayerAllocationPool&, size_t w,
                size_t h, size_t n);
  Event backpropagate(LayerAllocationPool&, LayerAllocationPool&, LayerAllocationPool&, size_t w,
                      size_t h, size_t n, Event* ev = nullptr);
  void fill_random_parameters(LayerData&, ParametersDistribution&, uint64_t seed);
  size_t load_parameters_file(const char* file);

  Config* const _config;
  LayerData layer_data_1;
  LayerData layer_data_2;
  LayerData layer_data_3;
  size_t _epochs = 0;
  size_t _mini_batch_size = 0;
  uint64_t _seed = 0;
  bool _seeded = false;
  bool _save_momentum = false;
  std::vector<float> _momentum_in[3][2];  // momentum read from the parameters file [layer][W, B]

  size_t _buf_w = 0, _buf_h = 0, _buf_n = 0;
  MemoryHandle _ground_truth_gpu_buf = gpu_nullptr;
  MemoryHandle _forward_gpu_buf = gpu_nullptr;
  MemoryHandle _out_1_gpu_buf = gpu_nullptr, _out_2_gpu_buf = gpu_nullptr,
               _out_3_gpu_buf = gpu_nullptr;
  MemoryHandle _delta_1_gpu_buf = gpu_nullptr, _delta_2_gpu_buf = gpu_nullptr,
               _delta_3_gpu_buf = gpu_nullptr;

  // flat parameter / gradient / momentum buffers and their per-layer views
  MemoryHandle _flat_params = gpu_nullptr, _flat_grads = gpu_nullptr, _flat_moms = gpu_nullptr;
  LayerAllocationPool _views[3];

  Kernel* _layer_1_kernel = nullptr;
  Kernel* _layer_2_kernel = nullptr;
  Kernel* _layer_3_kernel = nullptr;
  Kernel* _layer_1_deltas_kernel = nullptr;
  Kernel* _layer_2_deltas_kernel = nullptr;
  Kernel* _train_kernel = nullptr;
  Kernel* _forward_kernel = nullptr;
  Kernel* _update_all_kernel = nullptr;
  Kernel* _allreduce_kernel = nullptr;
  MemoryHandle _comm_scalar = gpu_nullptr;
};

}  // namespace cnn_sr

#endif  // CNN_SR_CONFIG_BASED_DATA_PIPELINE_HPP
