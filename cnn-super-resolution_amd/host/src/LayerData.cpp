#include "LayerData.hpp"

#include <stdexcept>
#include <string>

namespace cnn_sr {

LayerData::LayerData(size_t n_prev, size_t n_cur, size_t f)
    : n_prev_filter_cnt(n_prev), current_filter_count(n_cur), f_spatial_size(f) {
  weights.reserve(weight_size());
  bias.reserve(bias_size());
}

void LayerData::validate(const LayerData& d) {
  if (d.weights.size() < d.weight_size()) {
    throw std::runtime_error(
        "Declared f_spatial_size(" + std::to_string(d.f_spatial_size) + ")*f_spatial_size(" +
        std::to_string(d.f_spatial_size) + ")*n_prev_filter_cnt(" +
        std::to_string(d.n_prev_filter_cnt) + ")*current_filter_count(" +
        std::to_string(d.current_filter_count) + ")=" + std::to_string(d.weight_size()) +
        " is bigger then weights array (" + std::to_string(d.weights.size()) +
        " elements). Expected more elements in weights array. ");
  }
  if (d.bias.size() < d.bias_size()) {
    throw std::runtime_error("Bias array(size=" + std::to_string(d.bias.size()) +
                             ") should have equal size to current_filter_count(" +
                             std::to_string(d.bias_size()) + ").");
  }
}

void LayerData::set_weights(const float* x) {
  if (x) weights.insert(weights.end(), x, x + weight_size());
}

void LayerData::set_bias(const float* x) {
  if (x) bias.insert(bias.end(), x, x + bias_size());
}

size_t LayerData::input_size(size_t w, size_t h) const { return w * h * n_prev_filter_cnt; }

void LayerData::get_output_dimensions(size_t* dim, size_t w, size_t h) const {
  dim[0] = w - f_spatial_size + 1;
  dim[1] = h - f_spatial_size + 1;
}

size_t LayerData::weight_size() const {
  return f_spatial_size * f_spatial_size * n_prev_filter_cnt * current_filter_count;
}

size_t LayerData::bias_size() const { return current_filter_count; }

}  // namespace cnn_sr

std::ostream& operator<<(std::ostream& os, const cnn_sr::LayerData& d) {
  return os << "Layer { previous filters: " << d.n_prev_filter_cnt
            << ", current filters: " << d.current_filter_count
            << ", f_spatial_size: " << d.f_spatial_size << ", weights.size: " << d.weights.size()
            << ", bias.size: " << d.bias.size() << "}";
}
