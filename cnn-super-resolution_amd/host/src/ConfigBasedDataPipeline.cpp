#include "ConfigBasedDataPipeline.hpp"

#include <chrono>
#include <fstream>
#include <iostream>
#include <random>
#include <string>

#include "Image.hpp"
#include "Json.hpp"

namespace cnn_sr {

using srcnn::check;
using srcnn::require;

namespace {
const char* const kLayerKeys[3] = {"layer1", "layer2", "layer3"};
}

ConfigBasedDataPipeline::ConfigBasedDataPipeline(Config& cfg, srcnn::Context* ctx)
    : DataPipeline(ctx),
      _config(&cfg),
      layer_data_1(1, cfg.n1, cfg.f1),
      layer_data_2(cfg.n1, cfg.n2, cfg.f2),
      layer_data_3(cfg.n2, 1, cfg.f3) {}

srcnn_net ConfigBasedDataPipeline::net() const {
  srcnn_net n;
  n.n1 = uint32_t(_config->n1);
  n.n2 = uint32_t(_config->n2);
  n.f1 = uint32_t(_config->f1);
  n.f2 = uint32_t(_config->f2);
  n.f3 = uint32_t(_config->f3);
  return n;
}

void ConfigBasedDataPipeline::init(int load_flags) {
  DataPipeline::init(load_flags);
  if (!_config->parameters_file.empty()) {
    std::cout << "Loading layer parameters from: '" << _config->parameters_file << "'" << std::endl;
    _epochs = load_parameters_file(_config->parameters_file.c_str());
    std::cout << "Previous epochs:  " << _epochs << std::endl;
  } else {
    std::cout << "No parameters file provided, initializing random weights and biases" << std::endl;
    uint64_t seed = _seeded ? _seed
                            : uint64_t(std::chrono::system_clock::now().time_since_epoch().count());
    fill_random_parameters(layer_data_1, _config->params_distr_1, seed);
    fill_random_parameters(layer_data_2, _config->params_distr_2, seed + 1);
    fill_random_parameters(layer_data_3, _config->params_distr_3, seed + 2);
  }
  LayerData::validate(layer_data_1);
  LayerData::validate(layer_data_2);
  LayerData::validate(layer_data_3);
}

void ConfigBasedDataPipeline::load_kernels(int load_flags) {
  DataPipeline::load_kernels(load_flags);
  using srcnn::KernelKind;
  // net-level launches carry the net shape as their defines
  const std::string net_args = "-D N1=" + std::to_string(_config->n1) + " -D N2=" +
                               std::to_string(_config->n2) + " -D F1=" + std::to_string(_config->f1) +
                               " -D F2=" + std::to_string(_config->f2) + " -D F3=" +
                               std::to_string(_config->f3);
  if ((load_flags & LOAD_KERNEL_LAYERS) && !_layer_1_kernel) {
    _layer_1_kernel = create_layer_kernel(layer_data_1, false);
    _layer_2_kernel = create_layer_kernel(layer_data_2, false);
    _layer_3_kernel = create_layer_kernel(layer_data_3, true);
    _forward_kernel = _context->create_kernel(KernelKind::Net, "srcnn_forward", 0, 0, 0, false, net_args);
  }
  if ((load_flags & LOAD_KERNEL_BACKPROPAGATE) && !_layer_1_deltas_kernel) {
    _layer_1_deltas_kernel = create_deltas_kernel(layer_data_1);
    _layer_2_deltas_kernel = create_deltas_kernel(layer_data_2);
    _train_kernel = _context->create_kernel(KernelKind::Net, "srcnn_train_fwd_bwd", 0, 0, 0, false, net_args);
    _update_all_kernel = _context->create_kernel(KernelKind::Net, "srcnn_update_all", 0, 0, 0, false, net_args);
    _allreduce_kernel = _context->create_kernel(KernelKind::AllReduce, "srcnn_allreduce_grads", 0, 0, 0,
                                                false, net_args);
  }
  // the net-level gfx950 kernels are set up here, as the reference builds its
  // kernels at init (src/ConfigBasedDataPipeline.cpp:54-75), not in the first batch
  if (load_flags & (LOAD_KERNEL_LAYERS | LOAD_KERNEL_BACKPROPAGATE)) {
    srcnn_net nt = net();
    check(srcnn_preload(&nt), "srcnn_preload");
  }
}

void ConfigBasedDataPipeline::set_mini_batch_size(size_t n) {
  _mini_batch_size = n;
  std::cout << "mini-batch size: " << _mini_batch_size << std::endl;
}

void ConfigBasedDataPipeline::allocate_buffers(size_t w, size_t h) {
  if (_out_1_gpu_buf != gpu_nullptr && _buf_w == w && _buf_h == h && _buf_n >= _mini_batch_size)
    return;
  _context->block();
  for (MemoryHandle* m : {&_ground_truth_gpu_buf, &_forward_gpu_buf, &_out_1_gpu_buf, &_out_2_gpu_buf,
                          &_out_3_gpu_buf, &_delta_1_gpu_buf, &_delta_2_gpu_buf, &_delta_3_gpu_buf}) {
    if (*m != gpu_nullptr) _context->raw_memory(*m)->release();
    *m = gpu_nullptr;
  }
  size_t d1[2], d2[2], d3[2];
  layer_data_1.get_output_dimensions(d1, w, h);
  layer_data_2.get_output_dimensions(d2, d1[0], d1[1]);
  layer_data_3.get_output_dimensions(d3, d2[0], d2[1]);
  size_t n = _mini_batch_size * sizeof(float);
  size_t p0 = w * h, p1 = d1[0] * d1[1] * layer_data_1.current_filter_count,
         p2 = d2[0] * d2[1] * layer_data_2.current_filter_count,
         p3 = d3[0] * d3[1] * layer_data_3.current_filter_count;
  auto rw = srcnn::MEM_READ_WRITE;
  _ground_truth_gpu_buf = _context->allocate(rw, n * p0);
  _forward_gpu_buf = _context->allocate(rw, n * p0);
  _out_1_gpu_buf = _context->allocate(rw, n * p1);
  _out_2_gpu_buf = _context->allocate(rw, n * p2);
  _out_3_gpu_buf = _context->allocate(rw, n * p3);
  _delta_1_gpu_buf = _context->allocate(rw, n * p1);
  _delta_2_gpu_buf = _context->allocate(rw, n * p2);
  _delta_3_gpu_buf = _context->allocate(rw, n * p3);
  _buf_w = w;
  _buf_h = h;
  _buf_n = _mini_batch_size;
}

bool ConfigBasedDataPipeline::bind_flat(LayerAllocationPool& l1, LayerAllocationPool& l2,
                                        LayerAllocationPool& l3) {
  LayerAllocationPool* pools[3] = {&l1, &l2, &l3};
  auto handles = [](const LayerAllocationPool& p) {
    return std::vector<MemoryHandle>{p.weights, p.bias, p.accumulating_grad_w, p.accumulating_grad_b,
                                     p.previous_batch_delta_w, p.previous_batch_delta_b};
  };
  if (_flat_params != gpu_nullptr) {
    bool ours = true;
    for (int i = 0; i < 3; ++i) ours = ours && handles(*pools[i]) == handles(_views[i]);
    if (ours) return true;
  }
  for (int i = 0; i < 3; ++i)
    for (MemoryHandle m : handles(*pools[i]))
      if (m != gpu_nullptr) return false;  // caller-owned pools: op-level path

  if (_flat_params == gpu_nullptr) {
    srcnn_net nt = net();
    size_t P = srcnn_net_param_count(&nt), off[6];
    check(srcnn_net_offsets(&nt, off), "srcnn_net_offsets");
    const LayerData* layers[3] = {&layer_data_1, &layer_data_2, &layer_data_3};
    std::vector<float> host(P);
    for (int i = 0; i < 3; ++i) {
      LayerData::validate(*layers[i]);
      std::copy(layers[i]->weights.begin(), layers[i]->weights.begin() + layers[i]->weight_size(),
                host.begin() + off[2 * i]);
      std::copy(layers[i]->bias.begin(), layers[i]->bias.begin() + layers[i]->bias_size(),
                host.begin() + off[2 * i + 1]);
    }
    auto rw = srcnn::MEM_READ_WRITE;
    _flat_params = _context->allocate(rw, P * sizeof(float));
    _flat_grads = _context->allocate(rw, P * sizeof(float));
    _flat_moms = _context->allocate(rw, P * sizeof(float));
    _context->write_buffer(_flat_params, host.data(), true);
    _context->zeros_float(_flat_grads, false);
    _context->zeros_float(_flat_moms, false);
    bool resume = false;
    for (int i = 0; i < 3; ++i) resume = resume || !_momentum_in[i][0].empty() || !_momentum_in[i][1].empty();
    if (resume) {  // momentum saved by write_params_to_file (set_save_momentum)
      std::vector<float> mom(P, 0.0f);
      for (int i = 0; i < 3; ++i) {
        const size_t n[2] = {layers[i]->weight_size(), layers[i]->bias_size()};
        for (int k = 0; k < 2; ++k) {
          const auto& v = _momentum_in[i][k];
          if (v.empty()) continue;
          srcnn::require(v.size() == n[k], "parameters file: layer " + std::to_string(i + 1) + " momentum has " +
                                               std::to_string(v.size()) + " values, expected " + std::to_string(n[k]));
          std::copy(v.begin(), v.end(), mom.begin() + off[2 * i + k]);
        }
      }
      _context->write_buffer(_flat_moms, mom.data(), true);
    }
    for (int i = 0; i < 3; ++i) {
      size_t wb = layers[i]->weight_size() * sizeof(float), bb = layers[i]->bias_size() * sizeof(float);
      size_t wo = off[2 * i] * sizeof(float), bo = off[2 * i + 1] * sizeof(float);
      _views[i].weights = _context->view(_flat_params, wo, wb);
      _views[i].bias = _context->view(_flat_params, bo, bb);
      _views[i].accumulating_grad_w = _context->view(_flat_grads, wo, wb);
      _views[i].accumulating_grad_b = _context->view(_flat_grads, bo, bb);
      _views[i].previous_batch_delta_w = _context->view(_flat_moms, wo, wb);
      _views[i].previous_batch_delta_b = _context->view(_flat_moms, bo, bb);
    }
  }
  for (int i = 0; i < 3; ++i) *pools[i] = _views[i];
  return true;
}

// ---------------------------------------------------------------- forward

Event ConfigBasedDataPipeline::forward(LayerAllocationPool& l1, LayerAllocationPool& l2,
                                       LayerAllocationPool& l3, SampleAllocationPool& sample) {
  set_mini_batch_size(1);
  allocate_buffers(sample.input_w, sample.input_h);
  require(sample.input_luma != gpu_nullptr, "sample has no input luma");
  _context->copy_buffer(sample.input_luma, _forward_gpu_buf);
  return forward(l1, l2, l3, sample.input_w, sample.input_h, 1);
}

Event ConfigBasedDataPipeline::forward(LayerAllocationPool& l1, LayerAllocationPool& l2,
                                       LayerAllocationPool& l3, size_t w, size_t h, size_t n) {
  check_initialized(LOAD_KERNEL_LAYERS);
  if (n > _mini_batch_size) throw std::runtime_error("Allocation pool out of bounds exception");
  if (bind_flat(l1, l2, l3)) {
    srcnn_net nt = net();
    size_t ws = srcnn_forward_workspace_bytes(&nt, w, h, n);
    void* wsp = scratch(ws);
    srcnn::Context::Launch l(*_context, *_forward_kernel);
    check(srcnn_forward(&nt, _context->fptr(_forward_gpu_buf), w, h, n, _context->fptr(_flat_params),
                        _context->fptr(_out_3_gpu_buf), wsp, ws, _context->stream()),
          "forward");
    return _context->mark();
  }
  size_t d1[2], d2[2];
  layer_data_1.get_output_dimensions(d1, w, h);
  layer_data_2.get_output_dimensions(d2, d1[0], d1[1]);
  Event e1 = execute_layer(*_layer_1_kernel, layer_data_1, l1, _forward_gpu_buf, w, h, n, _out_1_gpu_buf);
  Event e2 = execute_layer(*_layer_2_kernel, layer_data_2, l2, _out_1_gpu_buf, d1[0], d1[1], n,
                           _out_2_gpu_buf, &e1);
  return execute_layer(*_layer_3_kernel, layer_data_3, l3, _out_2_gpu_buf, d2[0], d2[1], n,
                       _out_3_gpu_buf, &e2);
}

// ---------------------------------------------------------------- training

Event ConfigBasedDataPipeline::backpropagate(LayerAllocationPool& l1, LayerAllocationPool& l2,
                                             LayerAllocationPool& l3, size_t w, size_t h, size_t n,
                                             Event* ev) {
  size_t d1[2], d2[2], d3[2];
  layer_data_1.get_output_dimensions(d1, w, h);
  layer_data_2.get_output_dimensions(d2, d1[0], d1[1]);
  layer_data_3.get_output_dimensions(d3, d2[0], d2[1]);
  size_t pad = _config->total_padding();
  Event e = last_layer_delta(_ground_truth_gpu_buf, w, h, n, _out_3_gpu_buf, _delta_3_gpu_buf, pad, ev);
  e = calculate_deltas(*_layer_2_deltas_kernel, layer_data_2, layer_data_3, l3, _delta_2_gpu_buf,
                       _delta_3_gpu_buf, d3[0], d3[1], n, _out_2_gpu_buf, &e);
  e = calculate_deltas(*_layer_1_deltas_kernel, layer_data_1, layer_data_2, l2, _delta_1_gpu_buf,
                       _delta_2_gpu_buf, d2[0], d2[1], n, _out_1_gpu_buf, &e);
  DataPipeline::backpropagate(layer_data_3, _out_2_gpu_buf, _delta_3_gpu_buf, l3, d3[0], d3[1], n, &e);
  DataPipeline::backpropagate(layer_data_2, _out_1_gpu_buf, _delta_2_gpu_buf, l2, d2[0], d2[1], n, &e);
  return DataPipeline::backpropagate(layer_data_1, _forward_gpu_buf, _delta_1_gpu_buf, l1, d1[0],
                                     d1[1], n, &e);
}

float ConfigBasedDataPipeline::execute_batch(bool backprop, GpuAllocationPool& gpu_alloc,
                                             std::vector<SampleAllocationPool*>& samples) {
  if (samples.empty() || _mini_batch_size == 0) throw std::runtime_error("Batch cannot be empty");
  check_initialized(backprop ? (LOAD_KERNEL_LAYERS | LOAD_KERNEL_BACKPROPAGATE)
                             : (LOAD_KERNEL_LAYERS | LOAD_KERNEL_MISC));
  size_t w = samples[0]->input_w, h = samples[0]->input_h;
  for (auto* s : samples) {
    require(s && s->input_w == w && s->input_h == h, "All samples of a batch must have the same size");
    require(s->input_luma != gpu_nullptr && s->expected_luma != gpu_nullptr,
            "Sample without input / expected luma");
  }
  allocate_buffers(w, h);
  LayerAllocationPool &l1 = gpu_alloc.layer_1, &l2 = gpu_alloc.layer_2, &l3 = gpu_alloc.layer_3;
  bool flat = bind_flat(l1, l2, l3);
  srcnn_net nt = net();
  size_t tile_bytes = w * h * sizeof(float);
  float validation_error = 0.f;
  for (size_t i = 0; i < samples.size();) {
    size_t n = 0;
    for (; n < _mini_batch_size && i + n < samples.size(); ++n) {
      SampleAllocationPool& s = *samples[i + n];
      _context->copy_buffer(s.input_luma, _forward_gpu_buf, n * tile_bytes);
      _context->copy_buffer(s.expected_luma, _ground_truth_gpu_buf, n * tile_bytes);
    }
    if (backprop && flat) {
      size_t ws = srcnn_train_workspace_bytes(&nt, w, h, n);
      void* wsp = scratch(ws);
      srcnn::Context::Launch l(*_context, *_train_kernel);
      check(srcnn_train_fwd_bwd(&nt, _context->fptr(_forward_gpu_buf), _context->fptr(_ground_truth_gpu_buf),
                                w, h, n, _context->fptr(_flat_params), _context->fptr(_flat_grads),
                                nullptr, wsp, ws, _context->stream()),
            "execute_batch");
    } else if (backprop) {
      Event e = forward(l1, l2, l3, w, h, n);
      backpropagate(l1, l2, l3, w, h, n, &e);
    } else {
      Event e = forward(l1, l2, l3, w, h, n);
      float err = 0.f;
      squared_error(_ground_truth_gpu_buf, w, h, n, _out_3_gpu_buf, gpu_nullptr, err,
                    _config->total_padding(), &e);
      validation_error += err;
    }
    _context->block();
    i += n;
  }
  return validation_error;
}

void ConfigBasedDataPipeline::update_parameters(LayerAllocationPool& l1, LayerAllocationPool& l2,
                                                LayerAllocationPool& l3, size_t batch, Event* ev) {
  check_initialized(LOAD_KERNEL_BACKPROPAGATE);
  bool flat = _flat_params != gpu_nullptr;
  LayerAllocationPool* pools[3] = {&l1, &l2, &l3};
  for (int i = 0; flat && i < 3; ++i)
    flat = pools[i]->weights == _views[i].weights && pools[i]->accumulating_grad_w == _views[i].accumulating_grad_w &&
           pools[i]->previous_batch_delta_w == _views[i].previous_batch_delta_w;
  if (flat) {
    _context->wait(ev);
    srcnn_net nt = net();
    const float* lr = _config->learning_rate;
    srcnn::Context::Launch l(*_context, *_update_all_kernel);
    check(srcnn_update_all(&nt, _context->fptr(_flat_params), _context->fptr(_flat_grads),
                           _context->fptr(_flat_moms), _config->momentum,
                           _config->weight_decay_parameter, lr, uint32_t(batch), _context->stream()),
          "update_parameters");
  } else {
    // caller-owned pools: momentum read from the parameters file
    // (set_save_momentum checkpoints) goes into their previous_batch_delta_*
    // buffers before the first update, as bind_flat does for the flat ones
    const LayerData* layers[3] = {&layer_data_1, &layer_data_2, &layer_data_3};
    for (int i = 0; i < 3; ++i)
      for (int k = 0; k < 2; ++k) {
        auto& v = _momentum_in[i][k];
        if (v.empty()) continue;
        const size_t n = k ? layers[i]->bias_size() : layers[i]->weight_size();
        srcnn::require(v.size() == n, "parameters file: layer " + std::to_string(i + 1) + " momentum has " +
                                          std::to_string(v.size()) + " values, expected " + std::to_string(n));
        MemoryHandle& m = k ? pools[i]->previous_batch_delta_b : pools[i]->previous_batch_delta_w;
        if (m == gpu_nullptr) m = _context->allocate(srcnn::MEM_READ_WRITE, n * sizeof(float));
        _context->write_buffer(m, 0, n * sizeof(float), v.data(), true);  // size-checked
        v.clear();
      }
    DataPipeline::update_parameters(layer_data_3, l3, batch, _config->momentum,
                                    _config->weight_decay_parameter, _config->learning_rate[2], ev);
    DataPipeline::update_parameters(layer_data_2, l2, batch, _config->momentum,
                                    _config->weight_decay_parameter, _config->learning_rate[1], ev);
    DataPipeline::update_parameters(layer_data_1, l1, batch, _config->momentum,
                                    _config->weight_decay_parameter, _config->learning_rate[0], ev);
    for (auto* p : pools) {
      _context->zeros_float(p->accumulating_grad_w, false);
      _context->zeros_float(p->accumulating_grad_b, false);
    }
  }
  _context->block();
  ++_epochs;
}

// ---------------------------------------------------------------- data parallel

void RcclExchange::allreduce(srcnn::Context& ctx, float* buf, size_t count) {
  require(_comm != nullptr, "allreduce: null communicator");
  check(srcnn_allreduce_grads(_comm, buf, count, ctx.stream()), "srcnn_allreduce_grads");
}

void ConfigBasedDataPipeline::allreduce_gradients(GpuAllocationPool& pools, GradientExchange& ex) {
  check_initialized(LOAD_KERNEL_BACKPROPAGATE);
  require(bind_flat(pools.layer_1, pools.layer_2, pools.layer_3),
          "allreduce_gradients needs the pipeline's own (flat) parameter buffers");
  srcnn_net nt = net();
  srcnn::Context::Launch l(*_context, *_allreduce_kernel);
  ex.allreduce(*_context, _context->fptr(_flat_grads), srcnn_net_param_count(&nt));
}

void ConfigBasedDataPipeline::allreduce_gradients(GpuAllocationPool& pools, srcnn_comm_t comm) {
  require(comm != nullptr, "allreduce_gradients: null communicator");
  RcclExchange ex(comm);
  allreduce_gradients(pools, ex);
}

float ConfigBasedDataPipeline::allreduce_sum(float v, GradientExchange& ex) {
  if (_comm_scalar == gpu_nullptr) _comm_scalar = _context->allocate(srcnn::MEM_READ_WRITE, sizeof(float));
  _context->write_buffer(_comm_scalar, &v, true);
  ex.allreduce(*_context, _context->fptr(_comm_scalar), 1);
  float out = 0.f;
  _context->read_buffer(_comm_scalar, &out, true);
  return out;
}

float ConfigBasedDataPipeline::allreduce_sum(float v, srcnn_comm_t comm) {
  require(comm != nullptr, "allreduce_sum: null communicator");
  RcclExchange ex(comm);
  return allreduce_sum(v, ex);
}

// ---------------------------------------------------------------- parameters I/O

void ConfigBasedDataPipeline::fill_random_parameters(LayerData& d, ParametersDistribution& pd,
                                                     uint64_t seed) {
  std::mt19937_64 gen(seed);
  auto draw = [&gen](float mean, float sd) {
    if (!(sd > 0.f)) return mean;
    std::normal_distribution<float> dist(mean, sd);
    return dist(gen);
  };
  d.weights.clear();
  d.bias.clear();
  for (size_t i = 0; i < d.weight_size(); ++i) d.weights.push_back(draw(pd.mean_w, pd.sd_w));
  for (size_t i = 0; i < d.bias_size(); ++i) d.bias.push_back(draw(pd.mean_b, pd.sd_b));
}

size_t ConfigBasedDataPipeline::load_parameters_file(const char* file) {
  using namespace srcnn::json;
  Value root = parse_file(file, Tag::Object);
  size_t epochs = 0;
  LayerData* layers[3] = {&layer_data_1, &layer_data_2, &layer_data_3};
  for (auto& kv : root.object) {
    if (try_read_uint(kv.first, kv.second, epochs, "epochs")) continue;
    bool known = false;
    for (int i = 0; i < 3; ++i) {
      if (kv.first != kLayerKeys[i]) continue;
      known = true;
      for (auto& sub : kv.second.object) {
        try_read_vector(sub.first, sub.second, layers[i]->weights, "weights");
        try_read_vector(sub.first, sub.second, layers[i]->bias, "bias");
        try_read_vector(sub.first, sub.second, _momentum_in[i][0], "momentum_weights");
        try_read_vector(sub.first, sub.second, _momentum_in[i][1], "momentum_bias");
      }
    }
    if (!known) std::cout << "[Warning] Unknown key '" << kv.first << "' in parameters file" << std::endl;
  }
  return epochs;
}

void ConfigBasedDataPipeline::write_params_to_file(const char* path, LayerAllocationPool l1,
                                                   LayerAllocationPool l2, LayerAllocationPool l3) {
  std::cout << "Saving parameters to: '" << path << "'" << std::endl;
  LayerData* layers[3] = {&layer_data_1, &layer_data_2, &layer_data_3};
  LayerAllocationPool* pools[3] = {&l1, &l2, &l3};
  _context->block();
  for (int i = 0; i < 3; ++i) {
    LayerData& d = *layers[i];
    d.weights.resize(d.weight_size());
    d.bias.resize(d.bias_size());
    if (pools[i]->weights != gpu_nullptr)
      _context->read_buffer(pools[i]->weights, 0, d.weight_size() * sizeof(float), d.weights.data(), true);
    if (pools[i]->bias != gpu_nullptr)
      _context->read_buffer(pools[i]->bias, 0, d.bias_size() * sizeof(float), d.bias.data(), true);
  }
  std::vector<float> mom[3][2];
  if (_save_momentum)
    for (int i = 0; i < 3; ++i) {
      const MemoryHandle h[2] = {pools[i]->previous_batch_delta_w, pools[i]->previous_batch_delta_b};
      const size_t n[2] = {layers[i]->weight_size(), layers[i]->bias_size()};
      for (int k = 0; k < 2; ++k) {
        if (h[k] == gpu_nullptr) continue;
        mom[i][k].resize(n[k]);
        _context->read_buffer(h[k], 0, n[k] * sizeof(float), mom[i][k].data(), true);
      }
    }
  std::ofstream out(path);
  if (!out.is_open()) throw srcnn::IOException(std::string("Could not write parameters file: ") + path);
  auto dump = [&out](const std::vector<float>& v) {
    for (size_t i = 0; i < v.size(); ++i) out << (i ? ", " : "") << srcnn::json::format_float(v[i]);
  };
  out << "{\n  \"epochs\": " << _epochs << ",\n\n";
  for (int i = 0; i < 3; ++i) {
    out << "  \"" << kLayerKeys[i] << "\":{\n    \"weights\": [";
    dump(layers[i]->weights);
    out << "],\n    \"bias\": [";
    dump(layers[i]->bias);
    out << "]";
    if (!mom[i][0].empty()) {
      out << ",\n    \"momentum_weights\": [";
      dump(mom[i][0]);
      out << "]";
    }
    if (!mom[i][1].empty()) {
      out << ",\n    \"momentum_bias\": [";
      dump(mom[i][1]);
      out << "]";
    }
    out << "\n  }" << (i < 2 ? ",\n" : "\n");
  }
  out << "}";
}

void ConfigBasedDataPipeline::write_result_image(const char* out_path, ImageData& img,
                                                 SampleAllocationPool& sample) {
  std::cout << "Saving result image to: '" << out_path << "'" << std::endl;
  size_t pad = _config->total_padding();
  require(size_t(img.w) > pad && size_t(img.h) > pad, "image smaller than the network padding");
  size_t lw = img.w - pad, lh = img.h - pad;
  MemoryHandle target = gpu_nullptr;
  swap_luma(img, sample.input_data, _out_3_gpu_buf, target, lw, lh);
  ImageData res(img.w, img.h, 3);
  _context->read_buffer(target, 0, res.data.size(), res.data.data(), true);
  _context->raw_memory(target)->release();
  srcnn::image::write(out_path, res);
}

}  // namespace cnn_sr
