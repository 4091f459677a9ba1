// cnn -- the command line of the reference (src/Main_cl.cpp) on the MI355X
// pipeline:
//
//   cnn [-h] [train] [dry] [profile] -c CONFIG -i IN [-o OUT] [-e EPOCHS]
//       [--seed N] [--device D] [--devices N] [--validation-percent P]
//       [--mini-batches M] [--save-momentum]
//
// forward:  IN is an image (JPEG / PNG / PNM), OUT the upscaled result image
// train:    IN is a directory of <name>_large.<ext> / <name>_small.<ext> pairs
//           (ground truth / degraded input, tools/make_samples.py makes
//           them), OUT the parameters.json written at the end.
// Differences from the reference, on purpose: paths are joined with '/'
// (the reference hard-codes "\\", src/Main_cl.cpp:284-287), the epoch
// shuffle is seeded (--seed; the reference uses unseeded rand()).
// Extension: `train --devices N` trains data-parallel on devices D .. D+N-1
// of one node: one host thread per device, the epoch's training set sharded
// contiguously over them, one RCCL all-reduce of the flat gradient buffer per
// epoch (srcnn_allreduce_grads over ncclCommInitAll communicators), the same
// update on every device.  Test seam: `--exchange host`
// replaces the RCCL all-reduce by a host-side sum in rank order (ranks may
// then share a device: `--same-device` puts every rank on --device), so the
// sharding, the split validation sums and the exchange logic of this driver
// run on a one-GPU machine.
#include <dirent.h>
#include <unistd.h>

#include <algorithm>
#include <cmath>
#include <condition_variable>
#include <mutex>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iostream>
#include <map>
#include <memory>
#include <random>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include "Config.hpp"
#include "ConfigBasedDataPipeline.hpp"
#include "Context.hpp"
#include "Image.hpp"

using namespace cnn_sr;

namespace {

struct Args {
  bool train = false, dry = false, profile = false, help = false, version = false;
  std::string config, in, out;
  size_t epochs = 0;
  uint64_t seed = 0;
  bool seeded = false;
  int device = 0;
  int devices = 1;
  bool devices_set = false;  // --devices given: the data-parallel driver (also for N = 1)
  bool host_exchange = false;  // --exchange host: the host-sum test seam instead of RCCL
  bool same_device = false;    // --same-device: every rank on --device (needs --exchange host)
  bool save_momentum = false;  // --save-momentum: momentum into the parameters file (resumable)
  size_t validation_percent = 20;  // src/Main_cl.cpp:87
  size_t mini_batches = 2;         // src/Main_cl.cpp:88
};

void usage() {
  std::cout
      << "usage: cnn [-h] [train] [dry] [profile] -c CONFIG -i IN [-o OUT] [-e EPOCHS]\n"
         "           [--seed N] [--device D] [--devices N] [--validation-percent P]\n"
         "           [--mini-batches M] [--save-momentum]\n\n"
         "  -h, --help            print this help\n"
         "  --version             library ABI, HIP runtime and RCCL the binary runs on\n"
         "  train                 train mode\n"
         "  dry                   do not store the result\n"
         "  profile               print kernel execution times\n"
         "  -c, --config CONFIG   CNN configuration (config.json)\n"
         "  -i, --in IN           image during forward, samples directory during training\n"
         "  -o, --out OUT         output path (result image or new parameters file)\n"
         "  -e, --epochs EPOCHS   number of epochs during training\n"
         "  --seed N              seed of the random parameters and the epoch shuffles\n"
         "  --device D            HIP device index (default 0)\n"
         "  --devices N           train data-parallel on devices D .. D+N-1 (default 1)\n"
         "  --exchange rccl|host  data-parallel gradient exchange (default rccl; host: a\n"
         "                        host-side sum, a test seam)\n"
         "  --same-device         every data-parallel rank on --device (with --exchange host)\n"
         "  --validation-percent  share of samples used for validation (default 20)\n"
         "  --mini-batches M      mini-batches per epoch (default 2)\n"
         "  --save-momentum       also store the momentum in the parameters file; a file\n"
         "                        that holds it resumes training with it (extension)\n";
}

bool parse(int argc, char** argv, Args& a) {
  for (int i = 1; i < argc; ++i) {
    std::string s = argv[i];
    auto value = [&](const char* name) -> std::string {
      if (i + 1 >= argc) throw std::runtime_error(std::string("missing value for ") + name);
      return argv[++i];
    };
    if (s == "-h" || s == "--help" || s == "help") a.help = true;
    else if (s == "--version") a.version = true;
    else if (s == "train") a.train = true;
    else if (s == "dry") a.dry = true;
    else if (s == "profile") a.profile = true;
    else if (s == "-c" || s == "--config") a.config = value("--config");
    else if (s == "-i" || s == "--in") a.in = value("--in");
    else if (s == "-o" || s == "--out") a.out = value("--out");
    else if (s == "-e" || s == "--epochs") a.epochs = std::stoul(value("--epochs"));
    else if (s == "--seed") { a.seed = std::stoull(value("--seed")); a.seeded = true; }
    else if (s == "--device") a.device = std::stoi(value("--device"));
    else if (s == "--devices") { a.devices = std::stoi(value("--devices")); a.devices_set = true; }
    else if (s == "--exchange") {
      const std::string v = value("--exchange");
      if (v != "rccl" && v != "host") throw std::runtime_error("--exchange must be rccl or host");
      a.host_exchange = v == "host";
    }
    else if (s == "--same-device") a.same_device = true;
    else if (s == "--save-momentum") a.save_momentum = true;
    else if (s == "--validation-percent") a.validation_percent = std::stoul(value("--validation-percent"));
    else if (s == "--mini-batches") a.mini_batches = std::stoul(value("--mini-batches"));
    else throw std::runtime_error("unknown argument '" + s + "'");
  }
  if (a.help || a.version) return false;
  if (a.config.empty() || a.in.empty()) throw std::runtime_error("--config and --in are required");
  if (a.devices < 1) throw std::runtime_error("--devices must be >= 1");
  if (a.same_device && !a.host_exchange)
    throw std::runtime_error("--same-device needs --exchange host (RCCL takes one rank per device)");
  return true;
}

/** <base>_large.* / <base>_small.* pairs of a samples directory
 * (src/Main_cl.cpp:267-301), sorted by base name. */
std::vector<std::pair<std::string, std::string>> training_samples(const std::string& dir) {
  DIR* d = opendir(dir.c_str());
  if (!d) throw srcnn::IOException("cannot open samples directory '" + dir + "'");
  std::map<std::string, std::pair<std::string, std::string>> by_base;
  while (dirent* e = readdir(d)) {
    std::string f = e->d_name;
    if (f == "." || f == "..") continue;
    size_t dot = f.rfind('.');
    std::string stem = dot == std::string::npos ? f : f.substr(0, dot);
    auto ends = [&](const char* suf) {
      size_t n = std::strlen(suf);
      return stem.size() > n && stem.compare(stem.size() - n, n, suf) == 0;
    };
    if (ends("_large")) by_base[stem.substr(0, stem.size() - 6)].first = dir + "/" + f;
    else if (ends("_small")) by_base[stem.substr(0, stem.size() - 6)].second = dir + "/" + f;
    else std::cout << "'" << f << "' is not a <name>_large / <name>_small image. Skipping sample" << std::endl;
  }
  closedir(d);
  std::vector<std::pair<std::string, std::string>> out;
  for (auto& kv : by_base) {
    if (kv.second.first.empty() || kv.second.second.empty())
      std::cout << "Only 1 image for pair with name '" << kv.first << "'. Skipping sample" << std::endl;
    else
      out.push_back(kv.second);
  }
  return out;
}

/** load + luma (normalised) on the device (src/Main_cl.cpp:303-318) */
void prepare_image(DataPipeline& p, const std::string& path, ImageData& img, MemoryHandle& data,
                   MemoryHandle& luma) {
  srcnn::image::load(path, img, 4);
  p.extract_luma(img, data, luma, true);
}

int forward(ConfigBasedDataPipeline& p, const Args& a) {
  auto& ctx = *p.context();
  ImageData img;
  SampleAllocationPool sample;
  prepare_image(p, a.in, img, sample.input_data, sample.input_luma);
  p.subtract_mean(sample.input_luma);
  sample.input_w = img.w;
  sample.input_h = img.h;
  ctx.block();
  GpuAllocationPool pools;
  p.forward(pools.layer_1, pools.layer_2, pools.layer_3, sample);
  if (!a.dry && !a.out.empty()) p.write_result_image(a.out.c_str(), img, sample);
  ctx.block();
  return 0;
}

/** Contiguous slice [start, start + count) of n items for `rank` of `world`
 * (the remainder goes to the lowest ranks; srcnn_amd/parallel.py shard). */
std::pair<size_t, size_t> shard(size_t n, int rank, int world) {
  size_t base = n / world, rem = n % world, r = size_t(rank);
  return {r * base + std::min(r, rem), base + (r < rem ? 1 : 0)};
}

/** One training run (src/Main_cl.cpp:157-195).  comm == nullptr: a single
 * device.  Otherwise rank `rank` of a data-parallel run: every rank loads
 * all samples and draws the same epoch split (same shuffle seed), trains on
 * its shard of the training set, the gradients are all-reduced, and every
 * rank applies the update with batch = |training set|. */
int train(ConfigBasedDataPipeline& p, const Args& a, uint64_t shuffle_seed, GradientExchange* comm = nullptr,
          int rank = 0, int world = 1) {
  auto& ctx = *p.context();
  const bool lead = rank == 0;
  auto files = training_samples(a.in);
  if (files.empty()) throw std::runtime_error("no training samples in '" + a.in + "'");
  const size_t nval = files.size() * a.validation_percent / 100, ntrain = files.size() - nval;
  if (lead) {
    if (nval == 0) std::cout << "[WARNING] Validation set is empty" << std::endl;
    else
      std::cout << "validation_set_size: " << nval << "/" << files.size() << " = "
                << (nval * 100.0f / files.size()) << "%" << std::endl;
  }
  srcnn::require(ntrain > 0, "Training set is empty");
  const size_t my_train = shard(ntrain, rank, world).second;
  p.set_mini_batch_size(std::max<size_t>(my_train, 1) / a.mini_batches + a.mini_batches);  // src/Main_cl.cpp:128-129

  GpuAllocationPool pools;
  for (auto& f : files) {
    ImageData large, small;
    SampleAllocationPool s;
    prepare_image(p, f.first, large, s.expected_data, s.expected_luma);
    prepare_image(p, f.second, small, s.input_data, s.input_luma);
    srcnn::require(large.w == small.w && large.h == small.h,
                   "sample pair sizes differ: " + f.first + " / " + f.second);
    p.subtract_mean(s.input_luma);
    s.input_w = small.w;
    s.input_h = small.h;
    ctx.block();
    ctx.raw_memory(s.input_data)->release();  // 3-channel images are not needed any more
    ctx.raw_memory(s.expected_data)->release();
    pools.samples.push_back(s);
  }
  const size_t px = pools.samples[0].input_w * pools.samples[0].input_h;

  std::mt19937_64 rng(shuffle_seed);
  std::vector<size_t> order(pools.samples.size());
  bool error = false;
  for (size_t epoch = 0; epoch < a.epochs; ++epoch) {
    // new random validation / training split every epoch (src/Main_cl.cpp:244-261)
    for (size_t i = 0; i < order.size(); ++i) order[i] = i;
    std::shuffle(order.begin(), order.end(), rng);
    std::vector<SampleAllocationPool*> val, tr;
    for (size_t i = 0; i < order.size(); ++i) (i < nval ? val : tr).push_back(&pools.samples[order[i]]);

    if (comm) {
      auto sh = shard(tr.size(), rank, world);
      std::vector<SampleAllocationPool*> mine(tr.begin() + sh.first, tr.begin() + sh.first + sh.second);
      if (!mine.empty()) p.execute_batch(true, pools, mine);
      p.allreduce_gradients(pools, *comm);
    } else {
      p.execute_batch(true, pools, tr);
    }
    p.update_parameters(pools.layer_1, pools.layer_2, pools.layer_3, tr.size());

    if (!val.empty() && (epoch % 25 == 0 || epoch == a.epochs - 1)) {
      float err;
      if (comm) {
        auto sh = shard(val.size(), rank, world);
        std::vector<SampleAllocationPool*> mine(val.begin() + sh.first, val.begin() + sh.first + sh.second);
        err = p.allreduce_sum(mine.empty() ? 0.f : p.execute_batch(false, pools, mine), *comm);
      } else {
        err = p.execute_batch(false, pools, val);
      }
      if (std::isnan(err)) {
        if (lead)
          std::cout << "Error: squared error is NAN, after " << epoch << "/" << a.epochs << " epochs"
                    << std::endl;
        error = true;
        break;
      }
      float mean = err / val.size();
      if (lead)
        std::cout << "[" << epoch << "] mean validation error: " << mean << " (" << (mean / px)
                  << " per px)" << std::endl;
    }
  }
  p.set_save_momentum(a.save_momentum);
  if (lead && !a.dry && !a.out.empty())
    p.write_params_to_file(a.out.c_str(), pools.layer_1, pools.layer_2, pools.layer_3);
  ctx.block();
  if (lead) std::cout << "DONE" << std::endl;
  return error ? 1 : 0;
}

/** `--exchange host` (test seam): the ranks' buffers meet in host memory
 * and every rank adds them up in rank order, so all ranks get bit-identical
 * sums; two barriers per exchange (deposit, then read) keep a fast rank from
 * overwriting its slot while a slow one still reads it. */
class HostSumExchange {
 public:
  explicit HostSumExchange(int n) : _n(n), _slots(n) {}
  class Rank : public GradientExchange {
   public:
    Rank(HostSumExchange* h, int r) : _h(h), _r(r) {}
    void allreduce(srcnn::Context& ctx, float* buf, size_t count) override {
      auto& mine = _h->_slots[_r];
      mine.resize(count);
      srcnn::check(srcnn_memcpy_d2h(mine.data(), buf, count * sizeof(float), ctx.stream()),
                   "host exchange: read");
      _h->barrier();
      std::vector<float> sum(_h->_slots[0]);
      for (int k = 1; k < _h->_n; ++k)
        for (size_t i = 0; i < count; ++i) sum[i] += _h->_slots[k][i];
      _h->barrier();
      srcnn::check(srcnn_memcpy_h2d(buf, sum.data(), count * sizeof(float), ctx.stream()),
                   "host exchange: write");
    }

   private:
    HostSumExchange* _h;
    int _r;
  };

 private:
  void barrier() {
    std::unique_lock<std::mutex> lk(_mu);
    if (_aborted) throw std::runtime_error("host exchange: another rank failed");
    const unsigned gen = _gen;
    if (++_arrived == _n) {
      _arrived = 0;
      ++_gen;
      _cv.notify_all();
    } else {
      _cv.wait(lk, [&] { return _gen != gen || _aborted; });
      if (_gen == gen) throw std::runtime_error("host exchange: another rank failed");
    }
  }

 public:
  /** A failing rank releases the ranks parked in barrier(): they throw
   * instead of waiting for an arrival that will never come. */
  void abort() {
    std::lock_guard<std::mutex> lk(_mu);
    _aborted = true;
    _cv.notify_all();
  }

 private:
  const int _n;
  std::vector<std::vector<float>> _slots;
  std::mutex _mu;
  std::condition_variable _cv;
  int _arrived = 0;
  unsigned _gen = 0;
  bool _aborted = false;
};

/** `train --devices N`: one thread per device, each with its own Context
 * (HIP device and stream) and pipeline over the same config and seed. */
int train_data_parallel(const Config& cfg, const Args& a) {
  const int n = a.devices;
  std::vector<int> devs(n);
  for (int i = 0; i < n; ++i) devs[i] = a.same_device ? a.device : a.device + i;
  std::vector<srcnn_comm_t> comms(n, nullptr);
  std::vector<std::unique_ptr<GradientExchange>> ex(n);
  HostSumExchange host(n);
  if (a.host_exchange) {
    for (int r = 0; r < n; ++r) ex[r].reset(new HostSumExchange::Rank(&host, r));
  } else {
    srcnn::check(srcnn_comm_init_all(comms.data(), n, devs.data()), "srcnn_comm_init_all");
    for (int r = 0; r < n; ++r) ex[r].reset(new RcclExchange(comms[r]));
  }
  std::cout << "Data-parallel training on " << n << " devices (" << devs.front() << ".."
            << devs.back() << "), " << (a.host_exchange ? "host-sum" : "RCCL") << " gradient all-reduce"
            << std::endl;
  const uint64_t seed = a.seeded ? a.seed : std::random_device{}();
  std::vector<int> rcs(n, 0);
  std::vector<std::thread> threads;
  for (int r = 0; r < n; ++r) {
    threads.emplace_back([&, r]() {
      try {
        Config my_cfg = cfg;
        srcnn::Context context;
        context.init(a.profile && r == 0, devs[r]);
        ConfigBasedDataPipeline pipeline(my_cfg, &context);
        pipeline.set_random_seed(seed);  // identical initial replicas
        pipeline.init(DataPipeline::LOAD_KERNEL_ALL);
        rcs[r] = train(pipeline, a, seed, ex[r].get(), r, n);
      } catch (const std::exception& e) {
        std::cout << "[ERROR] rank " << r << ": " << e.what() << std::endl;
        std::cout.flush();
        if (a.host_exchange) {
          // the host-sum seam: release the ranks parked in its barrier (they
          // throw and report in turn), then join them as usual
          host.abort();
          rcs[r] = 1;
          return;
        }
        // RCCL: the other ranks may be parked in a collective this one will
        // never join and cannot be released from here; leave without
        // unwinding them
        _exit(1);
      }
    });
  }
  for (auto& t : threads) t.join();
  for (auto c : comms)
    if (c) srcnn_comm_destroy(c);
  int rc = 0;
  for (int v : rcs) rc |= v;
  return rc;
}

/** `cnn --version`: the C ABI version, the HIP runtime and the RCCL this
 * process loaded (the RCCL matches the HIP runtime) */
void print_version() {
  std::cout << "libsrcnn_hip ABI " << srcnn_abi_version() << std::endl;
  std::string hip;
  std::ifstream maps("/proc/self/maps");
  for (std::string line; std::getline(maps, line);) {
    const size_t at = line.find('/');
    if (at != std::string::npos && line.find("libamdhip64.so") != std::string::npos) {
      hip = line.substr(at);
      break;
    }
  }
  std::cout << "HIP runtime " << (hip.empty() ? "(not loaded)" : hip) << std::endl;
  int v = 0;
  char path[4096] = {0};
  srcnn::check(srcnn_comm_version(&v, path, sizeof(path)), "srcnn_comm_version");
  std::cout << "RCCL " << v / 10000 << "." << (v / 100) % 100 << "." << v % 100 << " " << path << std::endl;
}

}  // namespace

int main(int argc, char** argv) {
  Args a;
  try {
    if (!parse(argc, argv, a)) {
      if (a.version) {
        print_version();
        return 0;
      }
      usage();
      return 0;
    }
  } catch (const std::exception& e) {
    std::cout << e.what() << std::endl;
    usage();
    return 1;
  }
  if (!a.dry && a.out.empty()) {
    std::cout << "Either provide out path or do the dry run" << std::endl;
    return 1;
  }
  if (a.profile)
    std::cout << "!!! RUNNING IN PROFILING MODE !!!" << std::endl;
  if (a.train)
    std::cout << "Training mode, epochs: " << a.epochs << std::endl
              << "Training samples directory: " << a.in << std::endl
              << "Output: " << (a.dry ? "-" : a.out) << std::endl;
  else
    std::cout << "Forward mode" << std::endl
              << "Input image: " << a.in << std::endl
              << "Output: " << (a.dry ? "-" : a.out) << std::endl;
  try {
    ConfigReader reader;
    Config cfg = reader.read(a.config.c_str());
    std::cout << cfg << std::endl;
    if (a.train && a.devices_set) return train_data_parallel(cfg, a);
    srcnn::Context context;
    context.init(a.profile, a.device);
    int rc;
    {
      ConfigBasedDataPipeline pipeline(cfg, &context);
      if (a.seeded) pipeline.set_random_seed(a.seed);
      pipeline.init(DataPipeline::LOAD_KERNEL_ALL);
      rc = a.train ? train(pipeline, a, a.seeded ? a.seed : std::random_device{}()) : forward(pipeline, a);
    }
    return rc;
  } catch (const std::exception& e) {
    std::cout << "[ERROR] " << e.what() << std::endl;
    return 1;
  }
}
