#include "Config.hpp"

#include <cmath>
#include <vector>

#include "Context.hpp"
#include "Json.hpp"

namespace cnn_sr {

using srcnn::require;

ParametersDistribution::ParametersDistribution(float mw, float mb, float sw, float sb)
    : mean_w(mw), sd_w(sw), mean_b(mb), sd_b(sb) {}

Config::Config(size_t n1_, size_t n2_, size_t f1_, size_t f2_, size_t f3_, float mom, float wd,
               const float* lr, ParametersDistribution pd1, ParametersDistribution pd2,
               ParametersDistribution pd3, const char* params_file)
    : n1(n1_), n2(n2_), f1(f1_), f2(f2_), f3(f3_), momentum(mom), weight_decay_parameter(wd),
      parameters_file(params_file ? params_file : ""), params_distr_1(pd1),
      params_distr_2(pd2), params_distr_3(pd3) {
  for (int i = 0; i < 3; ++i) learning_rate[i] = lr ? lr[i] : 0.0f;
}

size_t Config::total_padding() const { return f1 + f2 + f3 - 3; }

void Config::validate(Config& c) {
  require(c.f1 % 2 == 1, "f1 should be odd");
  require(c.f2 % 2 == 1, "f2 should be odd");
  require(c.f3 % 2 == 1, "f3 should be odd");
  require(c.n1 > 0, "n1 should be >0");
  require(c.n2 > 0, "n2 should be >0");
  require(c.f1 > 0, "f1 should be >0");
  require(c.f2 > 0, "f2 should be >0");
  require(c.f3 > 0, "f3 should be >0");
  require(c.weight_decay_parameter >= 0, "weight_decay should be >0");
  require(c.learning_rate[0] > 0 && c.learning_rate[1] > 0 && c.learning_rate[2] > 0,
          "All learning rates should be >0");
  for (const ParametersDistribution* pd : {&c.params_distr_1, &c.params_distr_2, &c.params_distr_3}) {
    require(pd->sd_w > 0, "std dev. for weights should be > 0");
    require(pd->sd_b >= 0, "std dev. for bias should be >= 0");
  }
}

namespace {

void read_distribution(const srcnn::json::Value& obj, ParametersDistribution& d) {
  using namespace srcnn::json;
  for (auto& kv : obj.object) {
    try_read_float(kv.first, kv.second, d.mean_w, "mean_w");
    try_read_float(kv.first, kv.second, d.mean_b, "mean_b");
    try_read_float(kv.first, kv.second, d.sd_w, "std_deviation_w");
    try_read_float(kv.first, kv.second, d.sd_b, "std_deviation_b");
  }
  d.mean_w = std::fabs(d.mean_w);
  d.mean_b = std::fabs(d.mean_b);
  d.sd_w = std::fabs(d.sd_w);
  d.sd_b = std::fabs(d.sd_b);
}

}  // namespace

Config ConfigReader::read(const char* file) {
  using namespace srcnn::json;
  Value root = parse_file(file, Tag::Object);
  size_t n1 = 0, n2 = 0, f1 = 0, f2 = 0, f3 = 0;
  float momentum = 0.f, wd = 0.f;
  std::string params_file;
  std::vector<float> lr;
  ParametersDistribution pd[3];
  static const char* const pd_keys[3] = {"parameters_distribution_1", "parameters_distribution_2",
                                         "parameters_distribution_3"};
  for (auto& kv : root.object) {
    const std::string& k = kv.first;
    const Value& v = kv.second;
    try_read_uint(k, v, n1, "n1");
    try_read_uint(k, v, n2, "n2");
    try_read_uint(k, v, f1, "f1");
    try_read_uint(k, v, f2, "f2");
    try_read_uint(k, v, f3, "f3");
    try_read_float(k, v, momentum, "momentum");
    try_read_float(k, v, wd, "weight_decay_parameter");
    try_read_string(k, v, params_file, "parameters_file");
    try_read_vector(k, v, lr, "learning_rates");
    for (int i = 0; i < 3; ++i)
      if (k == pd_keys[i] && v.is(Tag::Object)) read_distribution(v, pd[i]);
  }
  require(lr.size() == 3, "Expected 3 learning rates (one per layer) to be provided");
  Config cfg(n1, n2, f1, f2, f3, momentum, wd, lr.data(), pd[0], pd[1], pd[2],
             params_file.c_str());
  Config::validate(cfg);
  return cfg;
}

}  // namespace cnn_sr

std::ostream& operator<<(std::ostream& os, const cnn_sr::ParametersDistribution& pd) {
  return os << "{ weights(" << pd.mean_w << ", " << pd.sd_w << "), bias(" << pd.mean_b << ", "
            << pd.sd_b << ")}";
}

std::ostream& operator<<(std::ostream& os, const cnn_sr::Config& c) {
  os << "Config {\n"
     << "  parameters file: '" << c.parameters_file << "'\n"
     << "  momentum: " << c.momentum << "\n"
     << "  weight decay: " << c.weight_decay_parameter << "\n"
     << "  learning rates: { " << c.learning_rate[0] << ", " << c.learning_rate[1] << ", "
     << c.learning_rate[2] << "}\n"
     << "  layer 1: " << c.n1 << " filters, " << c.f1 << " spatial size\n"
     << "  layer 2: " << c.n2 << " filters, " << c.f2 << " spatial size\n"
     << "  layer 3: " << c.f3 << " spatial size\n"
     << "  parameters dist. 1 " << c.params_distr_1 << "\n"
     << "  parameters dist. 2 " << c.params_distr_2 << "\n"
     << "  parameters dist. 3 " << c.params_distr_3 << "}" << std::endl;
  return os;
}
