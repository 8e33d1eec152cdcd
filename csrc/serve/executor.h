// Inference executors used by the member service's `predict`.
//
// Reference: Member::predict (src/services.rs:475-497) decodes each queried
// image, runs `forward_t` under a per-model mutex on the CPU, applies softmax
// and takes the top-1 (prob, label). Here an executor classifies a whole
// batch of decoded images:
//   * GpuExecutor: the hand-written HIP engine (csrc/runtime/engine.cpp),
//     images uploaded once as u8, preprocess/forward/top-1 on the GPU.
//   * CpuExecutor: the same architectures on libtorch CPU ops (fp32); used
//     on nodes without a GPU (the BASELINE "AlexNet single-image classify on
//     CPU via libtorch .ot load" plumbing config).
#pragma once
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

#include "../runtime/jpeg.h"
#include "../runtime/weights.h"

namespace dmlc {

struct Prediction {
  double prob = 0;
  int class_idx = -1;
};

// Decoded-image cache statistics (GPU executor: images resident in HBM).
struct CacheStats {
  uint64_t hits = 0, misses = 0, staged = 0, evictions = 0;
  uint64_t bytes = 0, entries = 0, capacity = 0;
};

class Executor {
 public:
  virtual ~Executor() = default;
  virtual std::string backend() const = 0;
  // Loads (or hot-swaps) the weights of `model` (arch name) from a .ot file.
  virtual void load_model(const std::string& model, const std::string& ot_path) = 0;
  virtual void load_model_weights(const std::string& model, const WeightMap& w) = 0;
  virtual bool has_model(const std::string& model) const = 0;
  virtual std::vector<Prediction> predict(const std::string& model, const std::vector<Image>& imgs) = 0;

  // Classify image files. The default decodes every file on the host; the
  // GPU executor keeps decoded images resident in HBM and decodes only on a
  // miss.
  virtual std::vector<Prediction> predict_files(const std::string& model, const std::vector<std::string>& paths) {
    std::vector<Image> imgs;
    imgs.reserve(paths.size());
    for (const auto& p : paths) imgs.push_back(decode_jpeg_file(p));
    return predict(model, imgs);
  }
  // Make `path` resident ahead of use (side-stream upload); false if the
  // executor has no cache.
  virtual bool stage(const std::string& path) { return false; }
  virtual CacheStats cache_stats() const { return {}; }

  // SDFS replicas resident next to the compute (blobs): the GPU executor
  // keeps a staged file in the HBM of its coordinator GPU (pinned host buffer
  // -> hipMemcpyAsync on a side stream); the default keeps it in host memory.
  // Keys are caller-chosen (the member uses "<sdfs name>@v<version>").
  virtual void stage_blob(const std::string& key, const std::string& path);
  virtual void drop_blob(const std::string& key);
  virtual std::vector<std::string> blob_keys() const;
  virtual std::string blob_location() const { return "host"; }
  // Classify every image of a staged u8 shard blob (csrc/serve/shard.h), in
  // order. GPU: read in place from the HBM slices of the blob, each slice on
  // the partition GPU that holds it where possible.
  virtual std::vector<Prediction> predict_blob(const std::string& model, const std::string& key);
  // Images [first, first + n) of a staged shard blob (a shard job's query).
  virtual std::vector<Prediction> predict_blob_range(const std::string& model, const std::string& key, int64_t first,
                                                     int64_t n);

  // Several GPUs (GPU executor): the job order for the partition rule
  // (reference: first floor(n/2) GPUs to the first job,
  // src/services.rs:199-211), a human-readable placement, and declaring a GPU
  // lost (the fleet rebalances over the survivors).
  virtual void set_jobs(const std::vector<std::string>& models) { (void)models; }
  virtual std::string placement() const { return backend(); }
  virtual void lose_device(int device) {
    (void)device;
    throw std::runtime_error("lose_device: not a multi-GPU executor");
  }

 protected:
  mutable std::mutex blob_mu_;
  std::map<std::string, std::shared_ptr<const std::vector<uint8_t>>> host_blobs_;
};

// backend: "gpu", "cpu" or "auto" (GPU when a HIP device is visible).
// cache_bytes: HBM budget for decoded images (GPU executor).
std::unique_ptr<Executor> make_executor(const std::string& backend, int device, int max_batch,
                                        size_t cache_bytes = (size_t)4 << 30);
// Several GPUs of this node (GPU executor, csrc/comm/fleet.h): the GPUs are
// split between the loaded models; a query goes to the least-loaded GPU of
// its model's partition, and a batch of >= 2 x min_shard images is scattered
// over the partition with RCCL instead.
// lanes: concurrent forwards per GPU and model (one model instance each).
// batch_window_us: concurrent queries to one (model, GPU) instance are
// coalesced into one forward of up to max_batch images; a queued query waits
// at most this long for others to join (dp::FleetOptions).
std::unique_ptr<Executor> make_executor(const std::string& backend, const std::vector<int>& devices, int max_batch,
                                        size_t cache_bytes, int min_shard, int lanes = 2, int batch_window_us = 200);
int hip_device_count();

// Host-side reference preprocessing (same rule as csrc/kernels/preprocess.hip):
// short side -> S (long = floor(S*long/short)), centre crop, bilinear
// align_corners=False, /255, ImageNet mean/std. Output CHW float [3,S,S].
std::vector<float> preprocess_host(const Image& img, int S);

}  // namespace dmlc
