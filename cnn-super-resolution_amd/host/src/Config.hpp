// cnn_sr::Config / ConfigReader -- the config.json format of the reference
// (src/Config.hpp, src/Config.cpp, example_config.json):
//   n1, n2, f1, f2, f3, momentum, weight_decay_parameter,
//   learning_rates[3], parameters_file,
//   parameters_distribution_{1,2,3}: {mean_w, mean_b, std_deviation_w, std_deviation_b}
// Reading: unknown keys are ignored, distributions are made non-negative
// (abs), exactly 3 learning rates are required, then validate() applies the
// reference's rules (odd f, positive n/f, wd >= 0, lr > 0, sd_w > 0, sd_b >= 0).
#ifndef CNN_SR_CONFIG_HPP
#define CNN_SR_CONFIG_HPP

#include <cstddef>
#include <ostream>
#include <string>

namespace cnn_sr {

struct ParametersDistribution {
  ParametersDistribution() {}
  ParametersDistribution(float mean_w, float mean_b, float sd_w, float sd_b);

  float mean_w = 0.01f, sd_w = 0.01f;
  float mean_b = 0.0f, sd_b = 0.0f;
};

struct Config {
  Config(size_t n1, size_t n2, size_t f1, size_t f2, size_t f3, float momentum,
         float weight_decay, const float* learning_rates, ParametersDistribution pd1,
         ParametersDistribution pd2, ParametersDistribution pd3,
         const char* parameters_file = nullptr);

  static void validate(Config&);

  /** f1 + f2 + f3 - 3: ground truth size minus output size */
  size_t total_padding() const;

  const size_t n1, n2;
  const size_t f1, f2, f3;
  const float momentum, weight_decay_parameter;
  float learning_rate[3];
  std::string parameters_file = "";

  ParametersDistribution params_distr_1;
  ParametersDistribution params_distr_2;
  ParametersDistribution params_distr_3;
};

class ConfigReader {
 public:
  /** throws srcnn::IOException (missing / unparsable file) or
   * std::runtime_error (invalid values) */
  Config read(const char* file);
};

}  // namespace cnn_sr

std::ostream& operator<<(std::ostream&, const cnn_sr::ParametersDistribution&);
std::ostream& operator<<(std::ostream&, const cnn_sr::Config&);

#endif  // CNN_SR_CONFIG_HPP
