// codec_fuzz -- deterministic mutation fuzzing of the host's file parsers,
// for the sanitizer build (tools/sanitize_host.sh: g++ -fsanitize=address,
// undefined): the JPEG / PNG / PNM decoders (srcnn::image::decode, the data
// path of `cnn train -i DIR` and `cnn dry -i IMAGE`), the JSON reader of
// config.json / parameters.json (srcnn::json::parse) and the config.json
// validation on top of it (cnn_sr::ConfigReader).  Every mutated input must
// decode or throw; a crash, a hang or a sanitizer report is a failure.
//   codec_fuzz [--iters N] [--seed S] FILE...
// Prints one summary line per seed file: mutations tried / decoded / rejected.
#include <unistd.h>

#include <cstdint>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <iostream>
#include <iterator>
#include <stdexcept>
#include <string>
#include <vector>

#include "Config.hpp"
#include "Image.hpp"
#include "Json.hpp"

// Context.cpp's srcnn::require (the harness links only the parsers, not the
// device-facing host library)
void srcnn::require(bool cond, const std::string& msg) {
  if (!cond) throw std::runtime_error(msg);
}

namespace {

struct Rng {  // xorshift64*: the same mutations on every run and host
  uint64_t s;
  explicit Rng(uint64_t seed) : s(seed * 0x9E3779B97F4A7C15ull + 1) {}
  uint64_t next() {
    s ^= s >> 12;
    s ^= s << 25;
    s ^= s >> 27;
    return s * 0x2545F4914F6CDD1Dull;
  }
  size_t below(size_t n) { return n ? size_t(next() % n) : 0; }
};

std::vector<unsigned char> mutate(const std::vector<unsigned char>& f, Rng& r) {
  std::vector<unsigned char> m = f;
  if (m.empty()) return m;
  switch (r.below(7)) {
    case 0:  // truncate
      m.resize(r.below(m.size()));
      break;
    case 1:  // a few random bytes
      for (size_t k = 1 + r.below(8); k--;) m[r.below(m.size())] = uint8_t(r.next());
      break;
    case 2: {  // boundary byte values
      static const uint8_t v[] = {0x00, 0xFF, 0x7F, 0x80, 0x01, 0xFE};
      m[r.below(m.size())] = v[r.below(sizeof(v))];
      break;
    }
    case 3: {  // duplicate a range
      const size_t a = r.below(m.size()), n = 1 + r.below(std::min<size_t>(m.size() - a, 256));
      std::vector<unsigned char> seg(m.begin() + a, m.begin() + a + n);
      m.insert(m.begin() + r.below(m.size() + 1), seg.begin(), seg.end());
      break;
    }
    case 4: {  // delete a range
      const size_t a = r.below(m.size()), n = 1 + r.below(std::min<size_t>(m.size() - a, 256));
      m.erase(m.begin() + a, m.begin() + a + n);
      break;
    }
    case 5: {  // a big-endian 16-bit field (segment lengths, dimensions, counts)
      const size_t a = r.below(m.size() - 1 + (m.size() == 1));
      const uint16_t v = uint16_t(r.next());
      m[a] = uint8_t(v >> 8);
      if (a + 1 < m.size()) m[a + 1] = uint8_t(v);
      break;
    }
    default: {  // a 32-bit field (PNG lengths and dimensions)
      const size_t a = r.below(m.size());
      const uint32_t v = uint32_t(r.next()) >> r.below(32);
      for (int k = 0; k < 4 && a + k < m.size(); ++k) m[a + k] = uint8_t(v >> (24 - 8 * k));
      break;
    }
  }
  return m;
}

bool is_json(const std::vector<unsigned char>& f) {
  for (unsigned char c : f) {
    if (c == ' ' || c == '\n' || c == '\r' || c == '\t') continue;
    return c == '{' || c == '[';
  }
  return false;
}

std::string g_tmp;  // config files go through ConfigReader::read(path)

// true: decoded, false: rejected with an exception
bool run_one(const std::vector<unsigned char>& m, bool json) {
  try {
    if (json) {
      const std::string text(m.begin(), m.end());
      const srcnn::json::Value v = srcnn::json::parse(text);
      if (v.find("n1") || v.find("parameters_file")) {  // a config.json: validate it too
        std::ofstream(g_tmp, std::ios::binary) << text;
        cnn_sr::ConfigReader().read(g_tmp.c_str());
      }
    } else {
      srcnn::ImageData img;
      srcnn::image::decode(m, img);
      if (img.w <= 0 || img.h <= 0 || img.data.size() != size_t(img.w) * img.h * img.bpp) {
        std::cerr << "decoded image with inconsistent size" << std::endl;
        std::abort();
      }
    }
    return true;
  } catch (const std::exception&) {
    return false;
  }
}

}  // namespace

int main(int argc, char** argv) {
  long iters = 2000;
  uint64_t seed = 1;
  std::vector<std::string> files;
  for (int i = 1; i < argc; ++i) {
    const std::string a = argv[i];
    if (a == "--iters" && i + 1 < argc) iters = std::stol(argv[++i]);
    else if (a == "--seed" && i + 1 < argc) seed = std::stoull(argv[++i]);
    else files.push_back(a);
  }
  g_tmp = "/tmp/codec_fuzz_" + std::to_string(::getpid()) + ".json";
  if (files.empty()) {
    std::cerr << "usage: codec_fuzz [--iters N] [--seed S] FILE..." << std::endl;
    return 2;
  }
  for (size_t fi = 0; fi < files.size(); ++fi) {
    std::ifstream in(files[fi], std::ios::binary);
    if (!in) {
      std::cerr << "cannot read " << files[fi] << std::endl;
      return 2;
    }
    const std::vector<unsigned char> f((std::istreambuf_iterator<char>(in)), std::istreambuf_iterator<char>());
    const bool json = is_json(f);
    if (!run_one(f, json)) {
      std::cerr << "seed file does not decode: " << files[fi] << std::endl;
      return 3;
    }
    Rng r(seed + 7919 * fi);
    long ok = 0, rejected = 0;
    for (long it = 0; it < iters; ++it) {
      // stack 1-3 mutations so damage can compound
      std::vector<unsigned char> m = mutate(f, r);
      for (size_t k = r.below(3); k--;) m = mutate(m, r);
      (run_one(m, json) ? ok : rejected)++;
    }
    std::cout << files[fi] << " " << (json ? "json" : "image") << " mutations=" << iters << " decoded=" << ok
              << " rejected=" << rejected << std::endl;
  }
  std::remove(g_tmp.c_str());
  return 0;
}
