// Spec runner for the cnn_sr C++ API on the HIP path.
//
// Mirrors the reference's test specs (test/specs/*.cpp driven by
// test/TestRunner.cpp): the same operations through the same DataPipeline
// calls, checked against the reference's golden vectors (extracted as data
// into tests/golden/ by tests/golden/make_golden.py) or their closed forms.
// Every float compare is two-sided.  Usage:
//   pipeline_specs [--golden DIR] [--cpu-only] [--filter SUBSTR]
// --cpu-only runs the specs that need no device (config / JSON / params I/O).
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <memory>
#include <iostream>
#include <random>
#include <sstream>
#include <string>
#include <vector>

#include "Config.hpp"
#include "ConfigBasedDataPipeline.hpp"
#include "Context.hpp"
#include "DataPipeline.hpp"
#include "Image.hpp"
#include "Json.hpp"

using namespace cnn_sr;
using srcnn::json::Value;

namespace {

struct TestFailure : std::runtime_error {
  explicit TestFailure(const std::string& m) : std::runtime_error(m) {}
};

void expect(bool ok, const std::string& msg) {
  if (!ok) throw TestFailure(msg);
}

void expect_close(const std::vector<float>& exp, const std::vector<float>& got, float atol,
                  float rtol, const char* what) {
  expect(exp.size() <= got.size(), std::string(what) + ": result too short");
  for (size_t i = 0; i < exp.size(); ++i) {
    float tol = atol + rtol * std::fabs(exp[i]);
    if (!(std::fabs(exp[i] - got[i]) <= tol)) {
      std::ostringstream s;
      s << what << "[" << i << "]: expected " << exp[i] << ", got " << got[i] << " (tol " << tol << ")";
      throw TestFailure(s.str());
    }
  }
}

std::string g_golden = "tests/golden";

Value golden(const std::string& name) { return srcnn::json::parse_file(g_golden + "/" + name); }

std::vector<float> floats(const Value& v) {
  std::vector<float> out;
  for (auto& e : v.array) out.push_back(float(e.number));
  return out;
}

size_t num(const Value& obj, const char* key) { return size_t(obj.find(key)->number); }

MemoryHandle upload(srcnn::Context& c, const std::vector<float>& v) {
  MemoryHandle h = c.allocate(srcnn::MEM_READ_WRITE, v.size() * sizeof(float));
  c.write_buffer(h, v.data(), true);
  return h;
}

std::vector<float> download(srcnn::Context& c, MemoryHandle h, size_t n = 0) {
  if (!n) n = c.raw_memory(h)->size / sizeof(float);
  std::vector<float> v(n);
  c.block();
  c.read_buffer(h, 0, n * sizeof(float), v.data(), true);
  return v;
}

struct Spec {
  std::string name;
  bool needs_device;
  std::function<void(DataPipeline*)> run;
};

// ---------------------------------------------------------------- specs

// test/specs/LayerTest.cpp:97-130 on test/data/test_cases.json
void layer_spec(DataPipeline* p, const std::string& key) {
  auto& c = *p->context();
  Value all = golden("layer_test_cases.json");
  const Value& d = *all.find(key);
  LayerData layer(num(d, "n_prev_filter_cnt"), num(d, "current_filter_count"), num(d, "f_spatial_size"));
  auto w = floats(*d.find("weights")), b = floats(*d.find("bias"));
  layer.set_weights(w.data());
  layer.set_bias(b.data());
  LayerAllocationPool pool;
  MemoryHandle in = upload(c, floats(*d.find("input"))), out = gpu_nullptr;
  Kernel* k = p->create_layer_kernel(layer, false);
  p->execute_layer(*k, layer, pool, in, num(d, "input_w"), num(d, "input_h"), 1, out);
  expect_close(floats(*d.find("output")), download(c, out), 5e-4f, 0.f, "layer output");
}

// test/specs/LayerDeltasTest.cpp:141-193
void layer_deltas_spec(DataPipeline* p) {
  auto& c = *p->context();
  Value d = golden("layer_deltas.json");
  size_t n_prev = num(d, "n_prev_layer"), n_next = num(d, "n_next"), f_next = num(d, "f_next");
  LayerData curr(1, n_prev, 3), next(n_prev, n_next, f_next);
  auto w = floats(*d.find("weights"));
  std::vector<float> bias(n_next, 0.f);
  next.set_weights(w.data());
  next.set_bias(bias.data());
  auto x = floats(*d.find("input_x"));
  for (auto& v : x) v = std::max(v, 0.f);  // the layer's output = relu(input)
  MemoryHandle y = upload(c, x), dn = upload(c, floats(*d.find("deltas")));
  MemoryHandle dc = c.allocate(srcnn::MEM_READ_WRITE, x.size() * sizeof(float));
  LayerAllocationPool next_pool;
  Kernel* k = p->create_deltas_kernel(curr);
  p->calculate_deltas(*k, curr, next, next_pool, dc, dn, num(d, "next_w"), num(d, "next_h"), 1, y);
  expect_close(floats(*d.find("expected")), download(c, dc), 2e-6f, 0.f, "deltas");
}

// test/specs/BackpropagationTest.cpp:135-159 (data set 0)
void backprop_spec(DataPipeline* p) {
  auto& c = *p->context();
  Value d = golden("backprop.json");
  size_t n_prev = num(d, "n_prev"), n_cur = num(d, "n_cur"), f = num(d, "f"), iw = num(d, "in_w");
  LayerData layer(n_prev, n_cur, f);
  std::vector<float> zw(layer.weight_size(), 0.f), zb(n_cur, 0.f);
  layer.set_weights(zw.data());
  layer.set_bias(zb.data());
  LayerAllocationPool pool;
  pool.accumulating_grad_w = upload(c, std::vector<float>(layer.weight_size(), float(d.find("grad_w_init")->number)));
  pool.accumulating_grad_b = upload(c, std::vector<float>(n_cur, 0.f));
  MemoryHandle in = upload(c, floats(*d.find("input"))), dl = upload(c, floats(*d.find("deltas")));
  size_t ow = iw - f + 1;
  p->backpropagate(layer, in, dl, pool, ow, ow, 1);
  expect_close(floats(*d.find("expected_grad_w")), download(c, pool.accumulating_grad_w), 6e-5f, 0.f, "grad_w");
  expect_close(floats(*d.find("expected_grad_b")), download(c, pool.accumulating_grad_b), 6e-4f, 0.f, "grad_b");
}

// test/specs/BackpropagationTest.cpp:160-170 (data set 1: big input, 32 -> 16, f = 3)
void backprop_big_spec(DataPipeline* p) {
  auto& c = *p->context();
  const size_t iw = 1024, n_prev = 32, n_cur = 16, f = 3, ow = iw - f + 1;
  LayerData layer(n_prev, n_cur, f);
  std::vector<float> zw(layer.weight_size(), 0.f), zb(n_cur, 0.f);
  layer.set_weights(zw.data());
  layer.set_bias(zb.data());
  std::vector<float> in(iw * iw * n_prev), dl(ow * ow * n_cur);
  std::mt19937 gen(5);
  std::uniform_real_distribution<float> u(-1.f, 1.f);
  for (auto& v : in) v = u(gen);
  for (auto& v : dl) v = u(gen);
  LayerAllocationPool pool;
  MemoryHandle hin = upload(c, in), hdl = upload(c, dl);
  p->backpropagate(layer, hin, hdl, pool, ow, ow, 1);
  auto gb = download(c, pool.accumulating_grad_b);
  // gB[n] = sum of the deltas of channel n (double reference)
  for (size_t n = 0; n < n_cur; ++n) {
    double s = 0;
    for (size_t i = 0; i < ow * ow; ++i) s += dl[i * n_cur + n];
    expect(std::fabs(gb[n] - s) <= 1e-3 * (1 + std::fabs(s)), "big grad_b");
  }
  auto gw = download(c, pool.accumulating_grad_w);
  for (float v : gw) expect(std::isfinite(v), "big grad_w finite");
}

// test/specs/LastLayerDeltaTest.cpp:34-83
void last_delta_spec(DataPipeline* p) {
  auto& c = *p->context();
  const size_t aw = 6, ah = 6, pad = 4, gw = aw + 2 * pad, gh = ah + 2 * pad;
  std::vector<float> gt(gw * gh, 99999.f), algo(aw * ah), exp(aw * ah);
  std::mt19937 gen(7);
  for (size_t i = 0; i < aw * ah; ++i) {
    size_t r = i / aw, col = i % aw;
    float t = float(gen() % 256) / 100.f, x = float(gen() % 2560) / 1000.f - 1.28f;
    float y = std::max(x, 0.f);
    exp[i] = (y - t) * (x > 0 ? 1.f : 0.f);
    gt[(r + pad) * gw + pad + col] = t;
    algo[i] = y;
  }
  MemoryHandle hg = upload(c, gt), ha = upload(c, algo), target = gpu_nullptr;
  p->last_layer_delta(hg, gw, gh, 1, ha, target, 2 * pad);
  expect_close(exp, download(c, target), 0.f, 0.f, "last layer delta");
}

// test/specs/UpdateParametersTest.cpp:65-105 (wd = 0) plus the wd term of update_parameters.cl
void update_spec(DataPipeline* p, float wd) {
  auto& c = *p->context();
  const size_t n_prev = 2, n_cur = 400, f = 5, batch = 2;
  const float momentum = 0.8f, lr = 0.001f;
  LayerData layer(n_prev, n_cur, f);
  std::mt19937 gen(1234);
  auto rnd = [&](size_t n, float s) {
    std::vector<float> v(n);
    for (auto& x : v) x = float(gen() % 2560) / s;
    return v;
  };
  size_t nw = layer.weight_size(), nb = layer.bias_size();
  auto w = rnd(nw, 10.f), gw = rnd(nw, 100.f), pw = rnd(nw, 10.f);
  auto b = rnd(nb, 10.f), gb = rnd(nb, 100.f), pb = rnd(nb, 10.f);
  layer.set_weights(w.data());
  layer.set_bias(b.data());
  LayerAllocationPool pool;
  pool.weights = upload(c, w);
  pool.bias = upload(c, b);
  pool.accumulating_grad_w = upload(c, gw);
  pool.accumulating_grad_b = upload(c, gb);
  pool.previous_batch_delta_w = upload(c, pw);
  pool.previous_batch_delta_b = upload(c, pb);
  p->update_parameters(layer, pool, batch, momentum, wd, lr);
  std::vector<float> ew(nw), dw(nw), eb(nb), db(nb);
  for (size_t i = 0; i < nw; ++i) {
    dw[i] = momentum * pw[i] + lr * gw[i] + wd * w[i];
    ew[i] = w[i] - dw[i] / float(batch);
  }
  for (size_t i = 0; i < nb; ++i) {
    db[i] = momentum * pb[i] + lr * gb[i];
    eb[i] = b[i] - db[i] / float(batch);
  }
  expect_close(ew, download(c, pool.weights), 1e-4f, 1e-6f, "weights");
  expect_close(dw, download(c, pool.previous_batch_delta_w), 1e-4f, 1e-6f, "delta w");
  expect_close(eb, download(c, pool.bias), 1e-4f, 1e-6f, "bias");
  expect_close(db, download(c, pool.previous_batch_delta_b), 1e-4f, 1e-6f, "delta b");
}

// test/specs/SquaredErrorTest.cpp:31-82
void squared_error_spec(DataPipeline* p) {
  auto& c = *p->context();
  const size_t aw = 1000, ah = 2000, pad = 4, gw = aw + 2 * pad, gh = ah + 2 * pad;
  std::vector<float> gt(gw * gh, 99999.f), algo(aw * ah);
  std::mt19937 gen(3);
  double expected = 0;
  for (size_t y = 0; y < ah; ++y)
    for (size_t x = 0; x < aw; ++x) {
      float t = float(gen() % 256), a = float(gen() % 2560) / 10.f;
      gt[(y + pad) * gw + x + pad] = t;
      algo[y * aw + x] = a;
      expected += double(t - a) * double(t - a);
    }
  MemoryHandle hg = upload(c, gt), ha = upload(c, algo);
  MemoryHandle tmp = c.allocate(srcnn::MEM_READ_WRITE, sizeof(float));
  float got = 0.f;
  p->squared_error(hg, gw, gh, 1, ha, tmp, got, 2 * pad);
  c.block();
  expect(std::fabs(got - expected) <= 1e-6 * expected, "squared error");
}

// test/specs/SumTest.cpp:27-58 (margin 20, :47)
void sum_spec(DataPipeline* p, bool squared) {
  auto& c = *p->context();
  std::vector<float> v(900);
  double expected = 0;
  for (size_t i = 0; i < v.size(); ++i) {
    v[i] = float(i);
    expected += squared ? double(i) * i : double(i);
  }
  MemoryHandle h = upload(c, v);
  float got = p->sum(h, squared);
  expect(std::fabs(got - expected) <= 20.0, "sum");
}

// test/specs/SubtractFromAllTest.cpp:27-50, and subtract_mean
void subtract_spec(DataPipeline* p) {
  auto& c = *p->context();
  std::vector<float> v(900);
  for (size_t i = 0; i < v.size(); ++i) v[i] = float(i);
  MemoryHandle h = upload(c, v);
  p->subtract_from_all(h, 450.f);
  std::vector<float> exp(v.size());
  for (size_t i = 0; i < v.size(); ++i) exp[i] = v[i] - 450.f;
  expect_close(exp, download(c, h), 0.f, 0.f, "subtract_from_all");
  MemoryHandle h2 = upload(c, v);
  float mean = 0.f;
  p->subtract_mean(h2, &mean);
  expect(std::fabs(mean - 449.5f) < 1e-3f, "mean");
  for (size_t i = 0; i < v.size(); ++i) exp[i] = v[i] - mean;
  expect_close(exp, download(c, h2), 1e-4f, 0.f, "subtract_mean");
}

// test/specs/ExtractLumaTest.cpp:50-74 (spec margin 0.005, test/TestCase.cpp:51)
void extract_luma_spec(DataPipeline* p, bool normalize) {
  auto& c = *p->context();
  Value d = golden("extract_luma.json");
  int w = int(num(d, "w")), h = int(num(d, "h"));
  std::vector<unsigned char> rgba;
  for (auto& e : d.find("rgba")->array) rgba.push_back((unsigned char)e.number);
  ImageData img(w, h, 4, rgba.data());
  MemoryHandle raw = gpu_nullptr, luma = gpu_nullptr;
  p->extract_luma(img, raw, luma, normalize);
  auto exp = floats(*d.find("expected_normalized"));
  if (!normalize)
    for (auto& v : exp) v *= 255.f;
  expect_close(exp, download(c, luma), normalize ? 5e-3f : 5e-3f * 255, 0.f, "luma");
}

// test/specs/SwapLumaTest.cpp:39-90 (<= 2 LSB on <= 2.5% of the channels:
// the fixture's JPEG was decoded by PIL, the reference's by stb_image)
void swap_luma_spec(DataPipeline* p) {
  auto& c = *p->context();
  Value d = golden("swap_luma.json");
  int w = int(num(d, "w")), h = int(num(d, "h")), pad = int(num(d, "padding"));
  std::vector<unsigned char> rgba, exp;
  for (auto& e : d.find("rgba")->array) rgba.push_back((unsigned char)e.number);
  for (auto& e : d.find("expected_rgba")->array) exp.push_back((unsigned char)e.number);
  ImageData img(w, h, 4, rgba.data());
  size_t lw = w - 2 * pad, lh = h - 2 * pad, n = lw * lw;
  std::vector<float> nl(n);
  for (size_t i = 0; i < n; ++i) nl[i] = float(i) / float(n);
  MemoryHandle org = gpu_nullptr, target = gpu_nullptr, hl = upload(c, nl);
  p->swap_luma(img, org, hl, target, lw, lh);
  std::vector<unsigned char> out(size_t(w) * h * 3);
  c.block();
  c.read_buffer(target, 0, out.size(), out.data(), true);
  size_t bad = 0;
  for (size_t i = 0; i < size_t(w) * h; ++i)
    for (int ch = 0; ch < 3; ++ch) {
      int diff = std::abs(int(out[3 * i + ch]) - int(exp[4 * i + ch]));
      expect(diff <= 2, "swap_luma channel off by more than 2 LSB");
      bad += diff != 0;
    }
  expect(bad <= out.size() / 40, "swap_luma: too many differing channels");
}

// test/specs/ConfigTest.cpp:68-121
void config_spec(const std::string& file, bool expect_io, bool expect_invalid) {
  ConfigReader reader;
  bool io = false, invalid = false;
  try {
    Config c = reader.read((g_golden + "/config/" + file).c_str());
    auto same_pd = [](const ParametersDistribution& a, float v) {
      return a.mean_w == v && a.mean_b == v && a.sd_w == v && a.sd_b == v;
    };
    bool ok = c.n1 == 32 && c.n2 == 16 && c.f1 == 9 && c.f2 == 1 && c.f3 == 5 &&
              c.momentum == 123.5f && c.weight_decay_parameter == 0.1f && c.learning_rate[0] == 12 &&
              c.learning_rate[1] == 34 && c.learning_rate[2] == 56 &&
              c.parameters_file == "cnn-parameters-a.json" && same_pd(c.params_distr_1, 0.9f) &&
              same_pd(c.params_distr_2, 2.001f) && same_pd(c.params_distr_3, 0.001f);
    if (!ok) invalid = true;
  } catch (srcnn::IOException&) {
    io = true;
  }
  expect(io == expect_io, "IO error expectation (" + file + ")");
  expect(invalid == expect_invalid, "value mismatch expectation (" + file + ")");
}

// Config::validate rules (src/Config.cpp validate)
void config_validate_spec() {
  float lr[3] = {1, 1, 1};
  ParametersDistribution pd(0, 0, 0.1f, 0);
  auto bad = [&](size_t n1, size_t f1, float lr0, float sdw) {
    float l[3] = {lr0, 1, 1};
    ParametersDistribution q(0, 0, sdw, 0);
    Config c(n1, 16, f1, 1, 5, 0.9f, 0.f, l, q, pd, pd);
    try {
      Config::validate(c);
    } catch (std::runtime_error&) {
      return true;
    }
    return false;
  };
  expect(!bad(32, 9, 1, 0.1f), "valid config rejected");
  expect(bad(32, 8, 1, 0.1f), "even f accepted");
  expect(bad(0, 9, 1, 0.1f), "n1 = 0 accepted");
  expect(bad(32, 9, 0, 0.1f), "lr = 0 accepted");
  expect(bad(32, 9, 1, 0.f), "sd_w = 0 accepted");
  Config c(64, 32, 9, 1, 5, 0.9f, 0.f, lr, pd, pd, pd);
  expect(c.total_padding() == 12, "total_padding");
}

// JSON reader edge cases + lossless float text
void json_spec() {
  using namespace srcnn::json;
  Value v = parse(R"({"a": [1, -2.5e3, 0.125], "s": "x\"é", "o": {"t": true, "n": null}})");
  expect(v.find("a")->array.size() == 3 && v.find("a")->array[1].number == -2500.0, "array");
  expect(v.find("s")->string == "x\"\xc3\xa9", "string escapes");
  expect(v.find("o")->find("t")->is(Tag::True) && v.find("o")->find("n")->is(Tag::Null), "literals");
  for (const char* badtxt : {"{", "{\"a\" 1}", "[1,]", "{\"a\":1} x", "{\"f1\":\n\"f2\": 1}"}) {
    bool threw = false;
    try {
      parse(badtxt);
    } catch (srcnn::IOException&) {
      threw = true;
    }
    expect(threw, std::string("parse error not raised for ") + badtxt);
  }
  std::mt19937 gen(11);
  std::normal_distribution<float> nd(0.f, 1e-3f);
  for (int i = 0; i < 10000; ++i) {
    float x = nd(gen);
    expect(std::strtof(format_float(x).c_str(), nullptr) == x, "lossless float text");
  }
}

// PNG / PNM writer + reader round trip
void image_spec() {
  for (int bpp : {1, 3, 4}) {
    srcnn::ImageData img(37, 23, bpp);
    for (size_t i = 0; i < img.data.size(); ++i) img.data[i] = (unsigned char)(i * 7 + bpp);
    for (const char* ext : {".png", bpp == 1 ? ".pgm" : ".ppm"}) {
      if (bpp == 4 && std::string(ext) != ".png") continue;
      std::string path = std::string("/tmp/srcnn_image_spec") + std::to_string(bpp) + ext;
      srcnn::image::write(path, img);
      srcnn::ImageData back;
      srcnn::image::load(path, back);
      expect(back.w == img.w && back.h == img.h && back.bpp == img.bpp && back.data == img.data,
             std::string("image round trip ") + ext);
    }
  }
}

// ConfigBasedDataPipeline: the fused flat path (pipeline-owned pools) and the
// per-layer op path (caller-owned pools) give the same training result, and
// parameters.json round-trips exactly.
void cbdp_spec(DataPipeline* p, size_t n1, size_t n2, size_t f1, size_t f2, size_t f3, size_t tile,
               size_t nsamples, size_t mini) {
  auto& c = *p->context();
  float lr[3] = {1e-3f, 1e-3f, 1e-4f};
  ParametersDistribution pd(0.f, 0.f, 0.05f, 0.01f);
  Config cfg(n1, n2, f1, f2, f3, 0.9f, 1e-3f, lr, pd, pd, pd);
  // samples: smooth patches, input mean-subtracted, target = patch
  std::mt19937 gen(99);
  std::uniform_real_distribution<float> u(0.f, 1.f);
  std::vector<SampleAllocationPool> samples(nsamples);
  for (auto& s : samples) {
    std::vector<float> t(tile * tile), x(tile * tile);
    float a = u(gen), b = u(gen), ph = 6.28f * u(gen);
    double mean = 0;
    for (size_t i = 0; i < t.size(); ++i) {
      size_t yy = i / tile, xx = i % tile;
      t[i] = 0.5f + 0.4f * std::sin(a * xx * 0.7f + b * yy * 0.5f + ph);
      mean += t[i];
    }
    mean /= t.size();
    for (size_t i = 0; i < t.size(); ++i) x[i] = t[i] - float(mean);
    s.input_w = s.input_h = tile;
    s.input_luma = upload(c, x);
    s.expected_luma = upload(c, t);
  }
  std::vector<SampleAllocationPool*> set;
  for (auto& s : samples) set.push_back(&s);

  std::vector<float> results[2];
  for (int variant = 0; variant < 2; ++variant) {
    ConfigBasedDataPipeline pipe(cfg, &c);
    pipe.set_random_seed(2024);
    pipe.init(DataPipeline::LOAD_KERNEL_ALL);
    pipe.set_mini_batch_size(mini);
    GpuAllocationPool pools;
    if (variant == 1) {  // caller-owned pools -> per-layer op path
      const LayerData* ls[3] = {pipe.layer_1(), pipe.layer_2(), pipe.layer_3()};
      LayerAllocationPool* ps[3] = {&pools.layer_1, &pools.layer_2, &pools.layer_3};
      for (int i = 0; i < 3; ++i) {
        ps[i]->weights = upload(c, ls[i]->weights);
        ps[i]->bias = upload(c, ls[i]->bias);
      }
    }
    for (int epoch = 0; epoch < 3; ++epoch) {
      pipe.execute_batch(true, pools, set);
      pipe.update_parameters(pools.layer_1, pools.layer_2, pools.layer_3, set.size());
    }
    float err = pipe.execute_batch(false, pools, set);
    expect(std::isfinite(err) && err > 0.f, "validation error");
    if (getenv("SRCNN_SPEC_DEBUG")) {
      float err2 = pipe.execute_batch(false, pools, set);
      std::cout << "variant " << variant << " validation error " << err << " / again " << err2 << std::endl;
    }
    std::string path = "/tmp/srcnn_cbdp_params_" + std::to_string(variant) + ".json";
    pipe.write_params_to_file(path.c_str(), pools.layer_1, pools.layer_2, pools.layer_3);
    std::vector<float>& r = results[variant];
    for (const LayerData* l : {pipe.layer_1(), pipe.layer_2(), pipe.layer_3()}) {
      r.insert(r.end(), l->weights.begin(), l->weights.end());
      r.insert(r.end(), l->bias.begin(), l->bias.end());
    }
    r.push_back(err);
    // the written file loads back to the same parameters, bit for bit
    Config cfg2(n1, n2, f1, f2, f3, 0.9f, 1e-3f, lr, pd, pd, pd, path.c_str());
    ConfigBasedDataPipeline again(cfg2, &c);
    again.init(DataPipeline::LOAD_KERNEL_ALL);
    expect(again.epochs() == 3, "epochs round trip");
    expect(again.layer_1()->weights == pipe.layer_1()->weights &&
               again.layer_2()->weights == pipe.layer_2()->weights &&
               again.layer_3()->bias == pipe.layer_3()->bias,
           "parameters.json round trip");
  }
  double scale = 0;
  for (float v : results[0]) scale = std::max(scale, double(std::fabs(v)));
  for (size_t i = 0; i + 1 < results[0].size(); ++i)
    expect(std::fabs(results[0][i] - results[1][i]) <= 1e-4 * (std::fabs(results[0][i]) + scale),
           "fused and op-level training disagree at " + std::to_string(i));
  float e0 = results[0].back(), e1 = results[1].back();
  double dmax = 0;
  for (size_t i = 0; i + 1 < results[0].size(); ++i)
    dmax = std::max(dmax, std::fabs(double(results[0][i]) - results[1][i]) / scale);
  expect(std::fabs(e0 - e1) <= 1e-3f * std::fabs(e1),
         "validation error mismatch: fused " + std::to_string(e0) + ", op path " + std::to_string(e1) +
             " (max parameter difference " + std::to_string(dmax) + " of the largest)");
}

// forward(sample) + write_result_image on a synthetic RGBA image
void inference_spec(DataPipeline* p) {
  auto& c = *p->context();
  float lr[3] = {1e-3f, 1e-3f, 1e-4f};
  ParametersDistribution pd(0.f, 0.f, 0.05f, 0.01f);
  Config cfg(32, 16, 9, 1, 5, 0.9f, 1e-3f, lr, pd, pd, pd);
  ConfigBasedDataPipeline pipe(cfg, &c);
  pipe.set_random_seed(1);
  pipe.init(DataPipeline::LOAD_KERNEL_ALL);
  srcnn::ImageData img(64, 48, 4);
  for (size_t i = 0; i < img.data.size(); ++i) img.data[i] = (unsigned char)((i * 37) % 251);
  SampleAllocationPool s;
  pipe.extract_luma(img, s.input_data, s.input_luma, true);
  s.input_w = img.w;
  s.input_h = img.h;
  pipe.subtract_mean(s.input_luma);
  GpuAllocationPool pools;
  pipe.forward(pools.layer_1, pools.layer_2, pools.layer_3, s);
  size_t ow = img.w - cfg.total_padding(), oh = img.h - cfg.total_padding();
  auto out = download(c, pipe.result_buffer(), ow * oh);
  for (float v : out) expect(std::isfinite(v), "finite output");
  pipe.write_result_image("/tmp/srcnn_result_spec.png", img, s);
  srcnn::ImageData back;
  srcnn::image::load("/tmp/srcnn_result_spec.png", back);
  expect(back.w == img.w && back.h == img.h && back.bpp == 3, "result image dims");
}

}  // namespace

int main(int argc, char** argv) {
  bool cpu_only = false;
  std::string filter;
  for (int i = 1; i < argc; ++i) {
    if (!std::strcmp(argv[i], "--golden") && i + 1 < argc) g_golden = argv[++i];
    else if (!std::strcmp(argv[i], "--cpu-only")) cpu_only = true;
    else if (!std::strcmp(argv[i], "--filter") && i + 1 < argc) filter = argv[++i];
  }
  std::vector<Spec> specs;
  for (const char* k : {"k=1, n=3, f=3, input:5*5", "k=3, n=2, f=3, input:3*3", "k=3, n=3, f=1, input:3*3"})
    specs.push_back({std::string("Layer test - ") + k, true, [k](DataPipeline* p) { layer_spec(p, k); }});
  specs.push_back({"Extract luma test - normalized", true, [](DataPipeline* p) { extract_luma_spec(p, true); }});
  specs.push_back({"Extract luma test - raw", true, [](DataPipeline* p) { extract_luma_spec(p, false); }});
  specs.push_back({"Swap luma test", true, swap_luma_spec});
  specs.push_back({"Squared error test", true, squared_error_spec});
  specs.push_back({"Subtract from all test", true, subtract_spec});
  specs.push_back({"Sum test", true, [](DataPipeline* p) { sum_spec(p, false); }});
  specs.push_back({"Sum test - squared", true, [](DataPipeline* p) { sum_spec(p, true); }});
  specs.push_back({"Layer deltas test", true, layer_deltas_spec});
  specs.push_back({"Backpropagation test", true, backprop_spec});
  specs.push_back({"Backpropagation test - big data", true, backprop_big_spec});
  specs.push_back({"Last layer delta test", true, last_delta_spec});
  specs.push_back({"Update parameters test", true, [](DataPipeline* p) { update_spec(p, 0.f); }});
  specs.push_back({"Update parameters test - weight decay", true, [](DataPipeline* p) { update_spec(p, 1e-2f); }});
  specs.push_back({"Config test - ok", false, [](DataPipeline*) { config_spec("config.json", false, false); }});
  specs.push_back({"Config test - invalid value", false,
                   [](DataPipeline*) { config_spec("config_invalid_val.json", false, true); }});
  specs.push_back({"Config test - invalid file", false,
                   [](DataPipeline*) { config_spec("config_non_parseable.json", true, false); }});
  specs.push_back({"Config test - file nonexistent", false, [](DataPipeline*) { config_spec("NOPE.json", true, false); }});
  specs.push_back({"Config validation", false, [](DataPipeline*) { config_validate_spec(); }});
  specs.push_back({"Json reader", false, [](DataPipeline*) { json_spec(); }});
  specs.push_back({"Image codec", false, [](DataPipeline*) { image_spec(); }});
  specs.push_back({"ConfigBasedDataPipeline - default net, fused vs op path", true,
                   [](DataPipeline* p) { cbdp_spec(p, 64, 32, 9, 1, 5, 33, 24, 10); }});
  specs.push_back({"ConfigBasedDataPipeline - wide net (f2=5)", true,
                   [](DataPipeline* p) { cbdp_spec(p, 128, 64, 9, 5, 5, 25, 5, 3); }});
  specs.push_back({"ConfigBasedDataPipeline - forward + result image", true, inference_spec});

  srcnn::Context context;
  DataPipeline* pipeline = nullptr;
  std::unique_ptr<DataPipeline> holder;
  if (!cpu_only) {
    context.init();
    std::cout << "device: " << context.device_name() << std::endl;
    holder.reset(new DataPipeline(&context));
    holder->init(DataPipeline::LOAD_KERNEL_ALL);
    pipeline = holder.get();
  }
  int run = 0, failed = 0;
  for (auto& s : specs) {
    if (cpu_only && s.needs_device) continue;
    if (!filter.empty() && s.name.find(filter) == std::string::npos) continue;
    ++run;
    try {
      s.run(pipeline);
      std::cout << "  ok    " << s.name << std::endl;
    } catch (const std::exception& e) {
      ++failed;
      std::cout << "  FAIL  " << s.name << ": " << e.what() << std::endl;
    }
  }
  std::cout << (run - failed) << " of " << run << " specs passed" << std::endl;
  return failed ? 1 : 0;
}
