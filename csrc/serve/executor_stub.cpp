// Executor factory for the sanitizer build of dmlc-node (`dmlc-node-tsan`):
// the control plane compiled with -fsanitize=thread and linked without
// libtorch / HIP (uninstrumented libraries would drown real reports in
// false positives). Everything else (membership, RPC, SDFS, jobs, REPL) is
// the production code. Inference is replaced by a "digest" executor that
// classifies an image by a hash of its decoded pixels, so predict jobs still
// run end to end (decode, batching, leader bookkeeping, fail-over) under
// the race detector.
#include <cstdint>
#include <mutex>
#include <map>
#include <set>
#include <stdexcept>

#include "executor.h"

namespace dmlc {

namespace {

class DigestExecutor final : public Executor {
 public:
  std::string backend() const override { return "digest"; }
  void load_model(const std::string& model, const std::string&) override {
    std::lock_guard<std::mutex> g(mu_);
    models_.insert(model);
  }
  void load_model_weights(const std::string& model, const WeightMap&) override {
    std::lock_guard<std::mutex> g(mu_);
    models_.insert(model);
  }
  bool has_model(const std::string& model) const override {
    std::lock_guard<std::mutex> g(mu_);
    return models_.count(model) != 0;
  }
  std::vector<Prediction> predict(const std::string& model, const std::vector<Image>& imgs) override {
    if (!has_model(model)) throw std::runtime_error("model not loaded: " + model);
    std::vector<Prediction> out(imgs.size());
    for (size_t i = 0; i < imgs.size(); ++i) out[i] = Prediction{1.0, digest(imgs[i])};
    return out;
  }

  // Same cache protocol as the GPU executor (hit / miss / staged), with the
  // digest standing in for the HBM-resident image, so the prefetch thread
  // and concurrent queries run under the race detector too.
  std::vector<Prediction> predict_files(const std::string& model, const std::vector<std::string>& paths) override {
    if (!has_model(model)) throw std::runtime_error("model not loaded: " + model);
    std::vector<Prediction> out;
    for (const auto& p : paths) out.push_back(Prediction{1.0, lookup(p, true)});
    return out;
  }
  bool stage(const std::string& path) override {
    lookup(path, false);
    return true;
  }
  CacheStats cache_stats() const override {
    std::lock_guard<std::mutex> g(mu_);
    CacheStats c = stats_;
    c.entries = cache_.size();
    return c;
  }

 private:
  static int digest(const Image& img) {
    uint64_t h = 1469598103934665603ull;  // FNV-1a over the pixels
    for (uint8_t v : img.rgb) h = (h ^ v) * 1099511628211ull;
    return int(h % 1000);
  }
  int lookup(const std::string& path, bool query) {
    {
      std::lock_guard<std::mutex> g(mu_);
      auto it = cache_.find(path);
      if (it != cache_.end()) {
        if (query) ++stats_.hits;
        return it->second;
      }
    }
    const int d = digest(decode_jpeg_file(path));
    std::lock_guard<std::mutex> g(mu_);
    if (cache_.emplace(path, d).second) {
      if (query) ++stats_.misses; else ++stats_.staged;
    }
    return d;
  }

  mutable std::mutex mu_;
  std::set<std::string> models_;
  std::map<std::string, int> cache_;
  CacheStats stats_;
};

}  // namespace

std::unique_ptr<Executor> make_executor(const std::string& backend, int, int, size_t) {
  if (backend == "none") return nullptr;
  if (backend == "digest" || backend == "auto" || backend == "cpu") return std::make_unique<DigestExecutor>();
  throw std::runtime_error("executor '" + backend + "' is not available in the sanitizer build");
}

std::unique_ptr<Executor> make_executor(const std::string& backend, const std::vector<int>& devices, int max_batch,
                                        size_t cache_bytes, int, int, int) {
  return make_executor(backend, devices.empty() ? 0 : devices[0], max_batch, cache_bytes);
}

int hip_device_count() { return 0; }

}  // namespace dmlc
