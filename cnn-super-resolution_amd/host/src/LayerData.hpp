// cnn_sr::LayerData -- shape + host copy of one layer's parameters.
// Same contract as the reference (src/LayerData.hpp:31-59, src/LayerData.cpp):
// weights W[dy][dx][c_in][c_out] (c_out innermost), bias[c_out]; validate()
// throws when the vectors are shorter than the declared shape.
#ifndef CNN_SR_LAYER_DATA_HPP
#define CNN_SR_LAYER_DATA_HPP

#include <cstddef>
#include <ostream>
#include <vector>

namespace cnn_sr {

struct LayerData {
  LayerData(size_t n_prev_filter_cnt, size_t current_filter_count, size_t f_spatial_size);

  static void validate(const LayerData&);

  /** append weight_size() / bias_size() values (no-op for nullptr) */
  void set_weights(const float*);
  void set_bias(const float*);

  size_t input_size(size_t w, size_t h) const;  // w*h*n_prev
  void get_output_dimensions(size_t* dim, size_t w, size_t h) const;
  size_t weight_size() const;  // f*f*n_prev*n_cur
  size_t bias_size() const;    // n_cur
  const float* weights_ptr() const { return weights.data(); }
  const float* bias_ptr() const { return bias.data(); }

  const size_t n_prev_filter_cnt;
  const size_t current_filter_count;
  const size_t f_spatial_size;

  /** host copies; stale once training runs on the device */
  std::vector<float> weights;
  std::vector<float> bias;
};

}  // namespace cnn_sr

std::ostream& operator<<(std::ostream&, const cnn_sr::LayerData&);

#endif  // CNN_SR_LAYER_DATA_HPP
