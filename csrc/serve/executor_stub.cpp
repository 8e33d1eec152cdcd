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
    for (size_t i = 0; i < imgs.size(); ++i) {
      uint64_t h = 1469598103934665603ull;  // FNV-1a over the pixels
      for (uint8_t v : imgs[i].rgb) h = (h ^ v) * 1099511628211ull;
      out[i].class_idx = int(h % 1000);
      out[i].prob = 1.0;
    }
    return out;
  }

 private:
  mutable std::mutex mu_;
  std::set<std::string> models_;
};

}  // namespace

std::unique_ptr<Executor> make_executor(const std::string& backend, int, int) {
  if (backend == "none") return nullptr;
  if (backend == "digest" || backend == "auto" || backend == "cpu") return std::make_unique<DigestExecutor>();
  throw std::runtime_error("executor '" + backend + "' is not available in the sanitizer build");
}

int hip_device_count() { return 0; }

}  // namespace dmlc
