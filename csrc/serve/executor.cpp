#include "executor.h"

#include <ATen/ATen.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <list>
#include <map>
#include <unordered_map>
#include <exception>
#include <stdexcept>
#include <thread>

#include "../runtime/engine.h"
#include "../runtime/ot_io.h"
#include "../runtime/trace.h"
#include "../comm/dp.h"
#include "../comm/fleet.h"
#include <atomic>
#include <climits>
#include <set>
#include "shard.h"
#include "../control/common.h"
#include <fstream>
#include "../kernels/kernels.h"
#include <condition_variable>
#include <cstring>

namespace dmlc {

std::vector<float> preprocess_host(const Image& img, int S) {
  const int Hin = img.height, Win = img.width;
  int RH, RW;
  if (Hin <= Win) {
    RH = S;
    RW = (int)((long)S * Win / Hin);
  } else {
    RW = S;
    RH = (int)((long)S * Hin / Win);
  }
  const int oy = (RH - S) / 2, ox = (RW - S) / 2;
  const float sys = (float)Hin / RH, sxs = (float)Win / RW;
  const bool identity = Hin == S && Win == S;
  const float mean[3] = {0.485f, 0.456f, 0.406f}, stdv[3] = {0.229f, 0.224f, 0.225f};
  std::vector<float> out((size_t)3 * S * S);
  for (int y = 0; y < S; ++y)
    for (int x = 0; x < S; ++x) {
      float c[3];
      if (identity) {
        const uint8_t* p = &img.rgb[((size_t)y * Win + x) * 3];
        for (int k = 0; k < 3; ++k) c[k] = p[k];
      } else {
        float sy = (y + oy + 0.5f) * sys - 0.5f, sx = (x + ox + 0.5f) * sxs - 0.5f;
        sy = std::min(std::max(sy, 0.f), (float)(Hin - 1));
        sx = std::min(std::max(sx, 0.f), (float)(Win - 1));
        const int y0 = (int)sy, x0 = (int)sx, y1 = std::min(y0 + 1, Hin - 1), x1 = std::min(x0 + 1, Win - 1);
        const float fy = sy - y0, fx = sx - x0;
        for (int k = 0; k < 3; ++k) {
          const float a = img.rgb[((size_t)y0 * Win + x0) * 3 + k], b = img.rgb[((size_t)y0 * Win + x1) * 3 + k];
          const float d = img.rgb[((size_t)y1 * Win + x0) * 3 + k], e = img.rgb[((size_t)y1 * Win + x1) * 3 + k];
          const float top = a + (b - a) * fx, bot = d + (e - d) * fx;
          // resized to u8 before normalising, like the GPU path (resize.hip)
          // and the reference's image-crate resize
          c[k] = std::min(std::max(std::nearbyint(top + (bot - top) * fy), 0.f), 255.f);
        }
      }
      for (int k = 0; k < 3; ++k) out[(size_t)k * S * S + (size_t)y * S + x] = (c[k] / 255.f - mean[k]) / stdv[k];
    }
  return out;
}

int hip_device_count() {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

namespace {

// ------------------------------------------------------------------ CPU
class CpuExecutor : public Executor {
 public:
  std::string backend() const override { return "cpu"; }

  void load_model(const std::string& model, const std::string& path) override {
    load_model_weights(model, ot_load(path));
  }

  void load_model_weights(const std::string& model, const WeightMap& w) override {
    std::map<std::string, at::Tensor> t;
    for (const auto& kv : w)
      t[kv.first] = at::from_blob(const_cast<float*>(kv.second.data.data()), kv.second.shape, at::kFloat).clone();
    std::lock_guard<std::mutex> g(mu_);
    models_[model] = std::move(t);
  }

  bool has_model(const std::string& model) const override {
    std::lock_guard<std::mutex> g(mu_);
    return models_.count(model) > 0;
  }

  std::vector<Prediction> predict(const std::string& model, const std::vector<Image>& imgs) override {
    std::lock_guard<std::mutex> g(mu_);  // per-executor model lock, like the reference's Mutex<Box<dyn ModuleT>>
    auto it = models_.find(model);
    if (it == models_.end()) throw std::runtime_error("model not loaded: " + model);
    if (imgs.empty()) return {};
    const int S = 224;
    at::Tensor x = at::empty({(int64_t)imgs.size(), 3, S, S}, at::kFloat);
    for (size_t i = 0; i < imgs.size(); ++i) {
      auto v = preprocess_host(imgs[i], S);
      std::memcpy(x[i].data_ptr<float>(), v.data(), v.size() * 4);
    }
    at::Tensor logits = forward(model, it->second, x);
    at::Tensor p = at::softmax(logits, -1);
    auto mx = p.max(-1);
    at::Tensor pv = std::get<0>(mx).contiguous(), pi = std::get<1>(mx).contiguous();
    std::vector<Prediction> out(imgs.size());
    for (size_t i = 0; i < imgs.size(); ++i) {
      out[i].prob = pv[i].item<float>();
      out[i].class_idx = (int)pi[i].item<int64_t>();
    }
    return out;
  }

 private:
  using TM = std::map<std::string, at::Tensor>;
  static const at::Tensor& W(const TM& w, const std::string& k) {
    auto it = w.find(k);
    if (it == w.end()) throw std::runtime_error("missing weight: " + k);
    return it->second;
  }
  static at::Tensor conv(const TM& w, const at::Tensor& x, const std::string& c, const std::string& bn, int s, int p,
                         bool relu) {
    auto bi = w.find(c + ".bias");
    at::Tensor y = at::conv2d(x, W(w, c + ".weight"), bi == w.end() ? at::Tensor() : bi->second, {s, s}, {p, p});
    if (!bn.empty())
      y = at::batch_norm(y, W(w, bn + ".weight"), W(w, bn + ".bias"), W(w, bn + ".running_mean"),
                         W(w, bn + ".running_var"), false, 0.1, 1e-5, false);
    return relu ? at::relu(y) : y;
  }
  static at::Tensor forward(const std::string& arch, const TM& w, at::Tensor x) {
    if (arch == "alexnet") {
      x = conv(w, x, "features.0", "", 4, 2, true);
      x = at::max_pool2d(x, {3, 3}, {2, 2});
      x = conv(w, x, "features.3", "", 1, 2, true);
      x = at::max_pool2d(x, {3, 3}, {2, 2});
      x = conv(w, x, "features.6", "", 1, 1, true);
      x = conv(w, x, "features.8", "", 1, 1, true);
      x = conv(w, x, "features.10", "", 1, 1, true);
      x = at::max_pool2d(x, {3, 3}, {2, 2});
      x = at::adaptive_avg_pool2d(x, {6, 6}).flatten(1);
      x = at::relu(at::linear(x, W(w, "classifier.1.weight"), W(w, "classifier.1.bias")));
      x = at::relu(at::linear(x, W(w, "classifier.4.weight"), W(w, "classifier.4.bias")));
      return at::linear(x, W(w, "classifier.6.weight"), W(w, "classifier.6.bias"));
    }
    std::vector<int> blocks;
    bool bottleneck = false;
    if (arch == "resnet18") blocks = {2, 2, 2, 2};
    else if (arch == "resnet34") blocks = {3, 4, 6, 3};
    else if (arch == "resnet50") blocks = {3, 4, 6, 3}, bottleneck = true;
    else throw std::runtime_error("unknown arch: " + arch);
    x = conv(w, x, "conv1", "bn1", 2, 3, true);
    x = at::max_pool2d(x, {3, 3}, {2, 2}, {1, 1});
    for (int li = 0; li < 4; ++li)
      for (int bi = 0; bi < blocks[li]; ++bi) {
        const int stride = (li > 0 && bi == 0) ? 2 : 1;
        const std::string p = "layer" + std::to_string(li + 1) + "." + std::to_string(bi);
        at::Tensor idt = x;
        if (w.count(p + ".downsample.0.weight"))
          idt = conv(w, x, p + ".downsample.0", p + ".downsample.1", stride, 0, false);
        at::Tensor y;
        if (!bottleneck) {
          y = conv(w, x, p + ".conv1", p + ".bn1", stride, 1, true);
          y = conv(w, y, p + ".conv2", p + ".bn2", 1, 1, false);
        } else {
          y = conv(w, x, p + ".conv1", p + ".bn1", 1, 0, true);
          y = conv(w, y, p + ".conv2", p + ".bn2", stride, 1, true);
          y = conv(w, y, p + ".conv3", p + ".bn3", 1, 0, false);
        }
        x = at::relu(y + idt);
      }
    x = at::adaptive_avg_pool2d(x, {1, 1}).flatten(1);
    return at::linear(x, W(w, "fc.weight"), W(w, "fc.bias"));
  }

  mutable std::mutex mu_;
  std::map<std::string, TM> models_;
};

// ------------------------------------------------------------------ GPU
// The GPUs of this node as one serving fleet (csrc/comm/fleet.h): the GPUs
// are split between the loaded models with the reference's fair-share rule,
// every model has an instance (engine x compute lanes) on each GPU of its
// partition, a query of a few images runs on the least-loaded GPU of the
// partition, and a large batch is scattered over the partition with RCCL.
//
// Data placement (HBM, 288 GB per GPU):
//   * decoded query images: an LRU cache spread over the GPUs (each new entry
//     on the GPU holding the fewest cached bytes); a query on GPU d resizes
//     them (resize.hip) straight from wherever they live, over xGMI peer
//     access (a copy-engine peer copy where peer access is unavailable);
//   * SDFS u8 shard replicas: split into one slice per live GPU when they
//     arrive, streamed from disk through two pinned buffers on per-GPU side
//     streams (the read of chunk i+1 overlaps the DMA of chunk i); a shard
//     query runs on the GPU holding its slice when that GPU is in the model's
//     partition, reading the slice from that GPU's HBM (one on-device copy
//     into the lane's batch buffer, no host or xGMI traffic).
class GpuExecutor : public Executor {
 public:
  GpuExecutor(std::vector<int> devices, int max_batch, size_t cache_bytes, int min_shard, int lanes, int batch_window_us)
      : devices_(std::move(devices)), max_batch_(max_batch), lanes_(std::max(1, std::min(lanes, 4))),
        cache_cap_(cache_bytes) {
    if (devices_.empty()) throw std::invalid_argument("GpuExecutor: no devices");
    kernel_stagger_for_lanes(lanes_);  // (one lane: the stream convs staggered, stagger.hip)
    for (int d : devices_) cache_bytes_dev_[d] = 0;
    if (devices_.size() > 1) enable_peers();
    for (int i = 0; i < kStagers; ++i) free_stagers_.push_back(std::make_shared<Stager>());
    dp::FleetOptions o;
    o.max_per_rank = max_batch_;
    o.image_bytes = (size_t)kS * kS * 3;
    o.min_shard = std::max(1, min_shard);
    o.aux_bytes = sizeof(ImageDesc);  // per image: a coalesced request's descriptors at its batch offset
    o.batch_window_us = batch_window_us;
    fleet_ = std::make_unique<dp::Fleet>(
        devices_, [this](const std::string& m, int d, dp::Worker* rep) { return make_worker(m, d, rep); },
        [](const std::vector<int>& devs) { return comm::rccl_init_all(devs); }, o);
  }
  ~GpuExecutor() override {
    fleet_.reset();
    {
      std::lock_guard<std::mutex> g(blob_mu_);
      hbm_blobs_.clear();
    }
    for (auto& kv : cache_) {
      (void)hipSetDevice(kv.second.device);
      (void)hipFree(kv.second.dev);
    }
    free_stagers_.clear();
  }
  std::string backend() const override {
    std::string b = "gpu:" + std::to_string(devices_[0]);
    for (size_t i = 1; i < devices_.size(); ++i) b += "," + std::to_string(devices_[i]);
    return b;
  }
  std::string placement() const override {
    std::string s;
    for (const auto& kv : fleet_->partitions()) {
      s += (s.empty() ? "" : " ") + kv.first + "=gpu";
      for (size_t i = 0; i < kv.second.size(); ++i) s += (i ? "," : "") + std::to_string(kv.second[i]);
      if (kv.second.empty()) s += "-";
    }
    return s.empty() ? "none" : s;
  }
  void set_jobs(const std::vector<std::string>& models) override { fleet_->set_jobs(models); }
  void lose_device(int device) override {
    fleet_->lose(device);
    {
      // decoded query images homed on the lost GPU are gone with it (first:
      // a re-staging failure below must not leave them cached)
      std::lock_guard<std::mutex> g(cache_mu_);
      for (auto it = cache_.begin(); it != cache_.end();) {
        if (it->second.device == device && it->second.pins == 0) {
          cache_bytes_ -= it->second.bytes;
          cache_bytes_dev_[device] -= it->second.bytes;
          lru_.erase(it->second.lru);
          it = cache_.erase(it);  // (its memory went with the device)
        } else {
          ++it;
        }
      }
    }
    // the partitions moved: every staged shard is placed for the new ones now
    std::vector<std::pair<std::string, std::shared_ptr<HbmBlob>>> bs;
    {
      std::lock_guard<std::mutex> g(blob_mu_);
      for (const auto& kv : hbm_blobs_) bs.emplace_back(kv.first, kv.second);
    }
    for (auto& kv : bs) {
      try {
        current_blob(kv.first, kv.second);
      } catch (const std::exception& e) {
        // (a missing file, or HBM exhausted while the old and new copies
        // coexist): the blob stays placed for the old partitions, so the next
        // query that reads it retries the re-staging
        DMLC_LOG_WARN("re-staging " << kv.first << " after losing GPU " << device << " failed: " << e.what());
      }
    }
  }

  void load_model(const std::string& model, const std::string& path) override {
    load_model_weights(model, ot_load(path));
  }
  void load_model_weights(const std::string& model, const WeightMap& w) override {
    {
      std::lock_guard<std::mutex> g(weights_mu_);
      weights_[model] = std::make_shared<const WeightMap>(w);
    }
    fleet_->load(model);  // first load: partitions recomputed; later: hot swap
  }
  bool has_model(const std::string& model) const override { return fleet_->has(model); }

  // Host images (decoded): uploaded to the chosen GPU inside the stage.
  std::vector<Prediction> predict(const std::string& model, const std::vector<Image>& imgs) override {
    const int64_t n = (int64_t)imgs.size();
    std::vector<int32_t> idx(n);
    std::vector<float> prob(n);
    auto stage = [&](const dp::StageCtx& c, int64_t first, int64_t cnt) -> const uint8_t* {
      auto s = (hipStream_t)c.worker->stream(c.stream);
      auto* hd = (ImageDesc*)c.aux_host;
      std::vector<void*> tmp;
      for (int64_t i = 0; i < cnt; ++i) {
        const Image& im = imgs[first + i];
        void* d = nullptr;
        DMLC_HIP_CHECK(hipMallocAsync(&d, std::max<size_t>(im.rgb.size(), 1), s));
        DMLC_HIP_CHECK(hipMemcpyAsync(d, im.rgb.data(), im.rgb.size(), hipMemcpyHostToDevice, s));
        tmp.push_back(d);
        hd[i] = ImageDesc{(const uint8_t*)d, im.height, im.width};
      }
      resize_into(c, hd, cnt, s);
      for (void* d : tmp) DMLC_HIP_CHECK(hipFreeAsync(d, s));
      return (const uint8_t*)c.batch;
    };
    fleet_->classify(model, n, stage, idx.data(), prob.data());
    return to_preds(idx, prob);
  }

  // HBM-resident decoded images: a hit skips the JPEG decode and the H2D
  // copy. The query's entries are pinned (not evictable) until its forward
  // has consumed them.
  std::vector<Prediction> predict_files(const std::string& model, const std::vector<std::string>& paths) override {
    if (!fleet_->has(model)) throw std::runtime_error("model not loaded: " + model);
    {
      DMLC_TRACE("executor.stage");
      // misses decode in parallel (host JPEG decode dominates a miss)
      const size_t nt = std::min<size_t>(paths.size(), kDecodeThreads);
      if (nt <= 1) {
        for (const auto& p : paths) stage_one(p, /*count_as_miss=*/true);
      } else {
        std::vector<std::thread> ts;
        std::vector<std::exception_ptr> errs(nt);
        for (size_t t = 0; t < nt; ++t)
          ts.emplace_back([&, t] {
            try {
              for (size_t i = t; i < paths.size(); i += nt) stage_one(paths[i], /*count_as_miss=*/true);
            } catch (...) {
              errs[t] = std::current_exception();
            }
          });
        for (auto& th : ts) th.join();
        for (auto& e : errs)
          if (e) std::rethrow_exception(e);
      }
    }
    struct Src {
      const uint8_t* dev;
      int device, h, w;
    };
    std::vector<Src> src(paths.size());
    std::vector<std::string> pinned;
    {
      std::lock_guard<std::mutex> g(cache_mu_);
      for (size_t i = 0; i < paths.size(); ++i) {
        auto it = cache_.find(paths[i]);
        if (it == cache_.end()) {
          for (const auto& p : pinned) --cache_.at(p).pins;
          throw std::runtime_error("image not resident: " + paths[i]);
        }
        touch(it);
        ++it->second.pins;
        pinned.push_back(paths[i]);
        src[i] = Src{(const uint8_t*)it->second.dev, it->second.device, it->second.h, it->second.w};
      }
    }
    const int64_t n = (int64_t)paths.size();
    std::vector<int32_t> idx(n);
    std::vector<float> prob(n);
    // the GPU already holding most of the query's images, for locality
    std::map<int, int> where;
    for (const auto& x : src) ++where[x.device];
    int prefer = -1, most = 0;
    for (const auto& kv : where)
      if (kv.second > most) most = kv.second, prefer = kv.first;
    auto stage = [&](const dp::StageCtx& c, int64_t first, int64_t cnt) -> const uint8_t* {
      auto s = (hipStream_t)c.worker->stream(c.stream);
      auto* hd = (ImageDesc*)c.aux_host;
      std::vector<void*> tmp;
      for (int64_t i = 0; i < cnt; ++i) {
        const Src& x = src[first + i];
        const uint8_t* p = x.dev;
        if (x.device != c.device && !peer(c.device, x.device)) {
          // no peer mapping: a copy-engine copy over xGMI into a temporary
          const size_t bytes = (size_t)x.h * x.w * 3;
          void* d = nullptr;
          DMLC_HIP_CHECK(hipMallocAsync(&d, bytes, s));
          DMLC_HIP_CHECK(hipMemcpyPeerAsync(d, c.device, x.dev, x.device, bytes, s));
          tmp.push_back(d);
          p = (const uint8_t*)d;
        }
        hd[i] = ImageDesc{p, x.h, x.w};
      }
      resize_into(c, hd, cnt, s);
      for (void* d : tmp) DMLC_HIP_CHECK(hipFreeAsync(d, s));
      return (const uint8_t*)c.batch;
    };
    dp::Fleet::QueryOptions q;
    q.prefer_device = prefer;
    try {
      DMLC_TRACE("executor.forward");
      fleet_->classify(model, n, stage, idx.data(), prob.data(), q);
    } catch (...) {
      unpin(pinned);
      throw;
    }
    unpin(pinned);
    return to_preds(idx, prob);
  }

  bool stage(const std::string& path) override {
    stage_one(path, /*count_as_miss=*/false);
    return true;
  }

  // ---- SDFS shard replicas, one slice per live GPU
  std::string blob_location() const override {
    std::string s = "hbm:gpu";
    for (size_t i = 0; i < devices_.size(); ++i) s += (i ? "," : "") + std::to_string(devices_[i]);
    return s;
  }

  // SDFS u8 shard replica -> HBM: one full copy per serving partition, each
  // sliced over that partition's GPUs (shard.h shard_placement), so every
  // model reads the images of its queries from the HBM of a GPU it serves on.
  void stage_blob(const std::string& key, const std::string& path) override {
    auto b = load_blob(path);
    std::lock_guard<std::mutex> g(blob_mu_);
    hbm_blobs_[key] = std::move(b);  // a replaced blob is freed once no query holds it
  }
  void drop_blob(const std::string& key) override {
    std::lock_guard<std::mutex> g(blob_mu_);
    hbm_blobs_.erase(key);
  }
  std::vector<std::string> blob_keys() const override {
    std::lock_guard<std::mutex> g(blob_mu_);
    std::vector<std::string> out;
    for (const auto& kv : hbm_blobs_) out.push_back(kv.first);
    return out;
  }

  // Every image of a shard: slice-aligned chunks of at most max_batch images,
  // run concurrently as direct queries, each preferring the GPU that holds
  // its slice (the data is already spread over the GPUs: no scatter).
  std::vector<Prediction> predict_blob(const std::string& model, const std::string& key) override {
    auto b = current_blob(key, blob(key));
    const int64_t n = b->si.n;
    std::vector<int32_t> idx(n);
    std::vector<float> prob(n);
    std::vector<std::pair<int64_t, int64_t>> chunks;
    const int copy = std::max(0, copy_of(*b, model));
    for (const auto& pc : b->pieces)
      if (pc.copy == copy)
        for (int64_t f = pc.first; f < pc.first + pc.n; f += max_batch_)
          chunks.emplace_back(f, std::min<int64_t>(max_batch_, pc.first + pc.n - f));
    const auto parts = fleet_->partitions();
    const size_t width = parts.count(model) ? std::max<size_t>(1, parts.at(model).size() * lanes_) : 1;
    std::atomic<size_t> next{0};
    std::vector<std::exception_ptr> errs(std::min(width, std::max<size_t>(1, chunks.size())));
    std::vector<std::thread> ts;
    for (size_t t = 0; t < errs.size(); ++t)
      ts.emplace_back([&, t] {
        try {
          for (size_t c = next++; c < chunks.size(); c = next++)
            classify_range(model, b, key, chunks[c].first, chunks[c].second, idx.data() + chunks[c].first,
                           prob.data() + chunks[c].first);
        } catch (...) {
          errs[t] = std::current_exception();
        }
      });
    for (auto& th : ts) th.join();
    for (auto& e : errs)
      if (e) std::rethrow_exception(e);
    return to_preds(idx, prob);
  }
  std::vector<Prediction> predict_blob_range(const std::string& model, const std::string& key, int64_t first,
                                             int64_t n) override {
    auto b = blob(key);
    if (n < 0) n = (int64_t)b->si.n - first;
    if (first < 0 || n < 0 || first + n > (int64_t)b->si.n) throw std::runtime_error(key + ": image range out of bounds");
    std::vector<int32_t> idx(n);
    std::vector<float> prob(n);
    classify_range(model, b, key, first, n, idx.data(), prob.data());
    return to_preds(idx, prob);
  }

  CacheStats cache_stats() const override {
    std::lock_guard<std::mutex> g(cache_mu_);
    CacheStats c = stats_;
    c.bytes = cache_bytes_;
    c.entries = cache_.size();
    c.capacity = cache_cap_;
    return c;
  }

 private:
  static constexpr int kS = 224;
  static constexpr size_t kDecodeThreads = 8;
  static constexpr int kStagers = 16;  // held through a miss's decode (it decodes into the pinned buffer)

  // A pinned bounce buffer pair and one side stream per GPU it has uploaded to.
  struct Stager {
    void* pinned[2] = {nullptr, nullptr};
    size_t pinned_bytes = 0;
    std::map<int, hipStream_t> streams;
    void ensure_pinned(size_t bytes) {
      if (pinned_bytes >= bytes) return;
      for (auto& p : pinned) {
        if (p) DMLC_HIP_CHECK(hipHostFree(p));
        p = nullptr;
      }
      pinned_bytes = 0;
      for (auto& p : pinned) DMLC_HIP_CHECK(hipHostMalloc(&p, bytes, hipHostMallocDefault));
      pinned_bytes = bytes;
    }
    hipStream_t stream(int device) {
      auto it = streams.find(device);
      if (it != streams.end()) return it->second;
      hipStream_t s;
      DMLC_HIP_CHECK(hipSetDevice(device));
      DMLC_HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
      streams[device] = s;
      return s;
    }
    ~Stager() {
      for (auto& kv : streams) {
        (void)hipSetDevice(kv.first);
        (void)hipStreamSynchronize(kv.second);
        (void)hipStreamDestroy(kv.second);
      }
      for (auto p : pinned)
        if (p) (void)hipHostFree(p);
    }
  };

  struct Entry {
    void* dev = nullptr;
    int device = 0;
    int h = 0, w = 0;
    size_t bytes = 0;
    int pins = 0;
    std::list<std::string>::iterator lru;
  };
  struct HbmBlob {
    ShardInfo si;
    std::string path;                     // the replica file (re-staging after a partition change)
    std::vector<std::vector<int>> parts;  // the partitions it was placed for (one copy each)
    struct Piece {
      int device = 0;
      int copy = 0;
      void* dev = nullptr;
      int64_t first = 0, n = 0;
    };
    std::vector<Piece> pieces;
    ~HbmBlob() {
      for (auto& p : pieces)
        if (p.dev) {
          (void)hipSetDevice(p.device);
          (void)hipFree(p.dev);
        }
    }
  };

  std::unique_ptr<dp::Worker> make_worker(const std::string& model, int device, dp::Worker* replica_of) {
    std::shared_ptr<const WeightMap> w;
    if (!replica_of) {
      std::lock_guard<std::mutex> g(weights_mu_);
      auto it = weights_.find(model);
      if (it == weights_.end()) throw std::runtime_error("no weights for " + model);
      w = it->second;
    }
    DMLC_HIP_CHECK(hipSetDevice(device));
    std::vector<std::unique_ptr<Engine>> es;
    if (replica_of) es.push_back(std::make_unique<Engine>(*dp::hip_worker_engine(*replica_of, 0), device));
    else es.push_back(std::make_unique<Engine>(model, *w, device));
    es[0]->reserve(max_batch_);
    // further compute lanes: more instances on the same GPU (their own
    // activations, graphs and streams), so concurrent queries overlap
    for (int l = 1; l < lanes_; ++l) {
      es.push_back(std::make_unique<Engine>(*es[0], device));
      if (!replica_of) es.back()->copy_weights_from(*es[0]);  // a replica's lanes copy after the broadcast
      es.back()->reserve(max_batch_);
    }
    return dp::make_owned_hip_worker(std::move(es), kS, kS, /*use_graph=*/true);
  }

  void enable_peers() {
    for (int a : devices_)
      for (int b : devices_) {
        if (a == b) continue;
        int can = 0;
        if (hipDeviceCanAccessPeer(&can, a, b) != hipSuccess || !can) continue;
        DMLC_HIP_CHECK(hipSetDevice(a));
        const hipError_t e = hipDeviceEnablePeerAccess(b, 0);
        if (e == hipSuccess || e == hipErrorPeerAccessAlreadyEnabled) peers_.insert({a, b});
        (void)hipGetLastError();
      }
  }
  // kernels on `reader` may dereference memory of `owner`
  bool peer(int reader, int owner) const { return reader == owner || peers_.count({reader, owner}) > 0; }

  // descriptors (pinned host) -> the stage's device scratch -> one u8 batch
  void resize_into(const dp::StageCtx& c, const ImageDesc* hd, int64_t cnt, hipStream_t s) {
    if (cnt > c.capacity) throw std::logic_error("resize_into: more images than the stage buffer holds");
    for (int64_t i = 0; i < cnt; ++i)
      if (hd[i].h <= 0 || hd[i].w <= 0 || hd[i].h > 4096 || hd[i].w > 4096)
        throw std::runtime_error("resize_into: bad image size");
    DMLC_HIP_CHECK(hipMemcpyAsync(c.aux, hd, (size_t)cnt * sizeof(ImageDesc), hipMemcpyHostToDevice, s));
    resize_u8_ragged((const ImageDesc*)c.aux, (uint8_t*)c.batch, (int)cnt, kS, s);
  }

  std::shared_ptr<HbmBlob> blob(const std::string& key) const {
    std::lock_guard<std::mutex> g(blob_mu_);
    auto it = hbm_blobs_.find(key);
    if (it == hbm_blobs_.end()) throw std::runtime_error("blob not staged: " + key);
    return it->second;
  }

  std::shared_ptr<HbmBlob> load_blob(const std::string& path) {
    std::ifstream f(path, std::ios::binary);
    if (!f) throw std::runtime_error("cannot open " + path);
    f.seekg(0, std::ios::end);
    const size_t bytes = (size_t)f.tellg();
    f.seekg(0);
    uint8_t head[kShardHeader] = {};
    if (bytes < kShardHeader || !f.read((char*)head, kShardHeader)) throw std::runtime_error(path + ": not a u8 shard");
    auto b = std::make_shared<HbmBlob>();
    b->si = parse_shard(head, bytes);  // validates h, w <= 4096 and n * h * w * 3 == size
    b->path = path;
    const size_t ib = b->si.image_bytes();
    b->parts = partition_sets();
    if (b->parts.empty()) throw std::runtime_error("no live GPU to stage " + path);
    const int64_t n = b->si.n;
    for (const PlacedSlice& ps : shard_placement(n, b->parts)) {
      HbmBlob::Piece pc;
      pc.device = ps.slice.device;
      pc.copy = ps.copy;
      pc.first = ps.slice.first;
      pc.n = ps.slice.n;
      DMLC_HIP_CHECK(hipSetDevice(pc.device));
      DMLC_HIP_CHECK(hipMalloc(&pc.dev, std::max<size_t>((size_t)pc.n * ib, 256)));
      b->pieces.push_back(pc);
    }
    // Stream the images through two pinned buffers: the file read of one
    // chunk overlaps the DMA of the previous one (each slice's DMA on a side
    // stream of its GPU); a buffer is refilled only once its copies are done.
    auto st = take_stager();
    try {
      constexpr size_t kChunk = (size_t)32 << 20;
      const size_t chunk = std::max(ib, kChunk / ib * ib);  // whole images per chunk
      st->ensure_pinned(std::min(chunk, std::max<size_t>((size_t)n * ib, 256)));
      const size_t cap = st->pinned_bytes / ib * ib;
      if (cap == 0) throw std::runtime_error("stage_blob: staging buffer too small");
      std::vector<hipEvent_t> pending[2];
      int buf = 0;
      for (int64_t img = 0; img < n;) {
        for (hipEvent_t e : pending[buf]) {
          DMLC_HIP_CHECK(hipEventSynchronize(e));
          DMLC_HIP_CHECK(hipEventDestroy(e));
        }
        pending[buf].clear();
        const int64_t cnt = std::min<int64_t>(n - img, (int64_t)(cap / ib));
        uint8_t* hb = (uint8_t*)st->pinned[buf];
        if (!f.read((char*)hb, (std::streamsize)((size_t)cnt * ib))) throw std::runtime_error(path + ": short read");
        for (const auto& pc : b->pieces) {
          const int64_t lo = std::max(img, pc.first), hi = std::min(img + cnt, pc.first + pc.n);
          if (lo >= hi) continue;
          DMLC_HIP_CHECK(hipSetDevice(pc.device));
          hipStream_t s = st->stream(pc.device);
          DMLC_HIP_CHECK(hipMemcpyAsync((uint8_t*)pc.dev + (size_t)(lo - pc.first) * ib, hb + (size_t)(lo - img) * ib,
                                        (size_t)(hi - lo) * ib, hipMemcpyHostToDevice, s));
          hipEvent_t e;
          DMLC_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
          DMLC_HIP_CHECK(hipEventRecord(e, s));
          pending[buf].push_back(e);
        }
        img += cnt;
        buf ^= 1;
      }
      for (auto& v : pending)
        for (hipEvent_t e : v) {
          DMLC_HIP_CHECK(hipEventSynchronize(e));  // resident before it is visible
          DMLC_HIP_CHECK(hipEventDestroy(e));
        }
    } catch (...) {
      give_stager(st);
      throw;
    }
    give_stager(st);
    return b;
  }
  // The distinct GPU sets of the current partitions (sorted), the copies a
  // staged blob holds.
  std::vector<std::vector<int>> partition_sets() const {
    std::vector<std::vector<int>> out;
    for (auto kv : fleet_->partitions()) {
      if (kv.second.empty()) continue;
      std::sort(kv.second.begin(), kv.second.end());
      if (std::find(out.begin(), out.end(), kv.second) == out.end()) out.push_back(kv.second);
    }
    if (out.empty()) {  // no model loaded yet: one copy over the live GPUs
      auto l = fleet_->live();
      if (!l.empty()) out.push_back(l);
    }
    std::sort(out.begin(), out.end());
    return out;
  }
  // A blob placed for other partitions, or with a piece on a lost GPU (a GPU
  // loss rebalanced the fleet), is staged again from its file for the
  // current ones (the lost GPU's slices used to fail every query
  // that touched them).
  std::shared_ptr<HbmBlob> current_blob(const std::string& key, std::shared_ptr<HbmBlob> b) {
    auto ok = [&](const HbmBlob& x) {
      if (x.parts != partition_sets()) return false;
      const auto live = fleet_->live();
      for (const auto& pc : x.pieces)
        if (std::find(live.begin(), live.end(), pc.device) == live.end()) return false;
      return true;
    };
    if (ok(*b)) return b;
    std::lock_guard<std::mutex> rg(restage_mu_);
    {
      std::lock_guard<std::mutex> g(blob_mu_);
      auto it = hbm_blobs_.find(key);
      if (it != hbm_blobs_.end() && it->second != b && ok(*it->second)) return it->second;  // done meanwhile
    }
    auto nb = load_blob(b->path);  // long: the file read and the DMA run without blob_mu_
    std::lock_guard<std::mutex> g(blob_mu_);
    auto it = hbm_blobs_.find(key);
    if (it != hbm_blobs_.end() && it->second == b) {
      it->second = nb;  // still the stale blob we found: replace it
      return nb;
    }
    // stage_blob installed a newer replica meanwhile (keep it; this query
    // may still read its own fresh copy of the old one), or the key was
    // dropped: either way nb is not installed and is freed with the query
    if (it != hbm_blobs_.end() && ok(*it->second)) return it->second;
    return nb;
  }

  // Images [first, first + n) of a staged shard through the fleet (no scatter:
  // the slices are already spread over the GPUs; the query prefers the GPU
  // holding its first image).
  // The copy of a blob placed for `model`'s partition (-1: none matches).
  int copy_of(const HbmBlob& b, const std::string& model) const {
    const auto parts = fleet_->partitions();
    auto it = parts.find(model);
    if (it == parts.end()) return -1;
    auto mine = it->second;
    std::sort(mine.begin(), mine.end());
    for (size_t c = 0; c < b.parts.size(); ++c)
      if (b.parts[c] == mine) return (int)c;
    return -1;
  }
  // The piece that holds image `pos` best for a reader on `device`: one on
  // that device, else one of copy `copy`, else any (a peer read).
  static const HbmBlob::Piece* piece_for(const HbmBlob& b, int64_t pos, int device, int copy) {
    const HbmBlob::Piece* best = nullptr;
    int score = -1;
    for (const auto& pc : b.pieces) {
      if (pos < pc.first || pos >= pc.first + pc.n) continue;
      const int sc = pc.device == device ? 2 : pc.copy == copy ? 1 : 0;
      if (sc > score) score = sc, best = &pc;
    }
    return best;
  }

  // Images [first, first + n) of a staged shard through the fleet (no scatter:
  // the slices are already spread over the partition's GPUs; the query
  // prefers the GPU holding its first image in the model's copy). The stage
  // returns the slice's own HBM address when the range lies in a slice on the
  // serving GPU, and the fleet then copies it device-to-device into the
  // lane's batch buffer (Fleet::direct: a coalesced forward's batch address
  // is fixed per lane, so each lane replays one captured graph per bucket):
  // n x 150 KB at HBM copy speed, about 1-2 % of a 256-image forward.
  void classify_range(const std::string& model, std::shared_ptr<HbmBlob> b, const std::string& key, int64_t first,
                      int64_t n, int32_t* idx, float* prob) {
    b = current_blob(key, b);
    const size_t ib = b->si.image_bytes();
    const bool dense = b->si.h == (uint32_t)kS && b->si.w == (uint32_t)kS;
    const int copy = copy_of(*b, model);
    int prefer = -1;
    if (const auto* pc = piece_for(*b, first, -1, copy)) prefer = pc->device;
    auto stage = [&](const dp::StageCtx& c, int64_t off, int64_t cnt) -> const uint8_t* {
      const int64_t g0 = first + off;
      auto s = (hipStream_t)c.worker->stream(c.stream);
      if (dense) {
        for (const auto& pc : b->pieces)  // the whole range in a slice on this GPU (copied into the lane by the fleet)
          if (pc.device == c.device && g0 >= pc.first && g0 + cnt <= pc.first + pc.n)
            return (const uint8_t*)pc.dev + (size_t)(g0 - pc.first) * ib;
        for (int64_t pos = g0; pos < g0 + cnt;) {  // gather the range into the stage buffer
          const auto* pc = piece_for(*b, pos, c.device, copy);
          if (!pc) throw std::runtime_error("blob: image not staged");
          const int64_t hi = std::min(g0 + cnt, pc->first + pc->n);
          uint8_t* dst = (uint8_t*)c.batch + (size_t)(pos - g0) * ib;
          const uint8_t* srcp = (const uint8_t*)pc->dev + (size_t)(pos - pc->first) * ib;
          if (pc->device == c.device)
            DMLC_HIP_CHECK(hipMemcpyAsync(dst, srcp, (size_t)(hi - pos) * ib, hipMemcpyDeviceToDevice, s));
          else
            DMLC_HIP_CHECK(hipMemcpyPeerAsync(dst, c.device, srcp, pc->device, (size_t)(hi - pos) * ib, s));
          pos = hi;
        }
        return (const uint8_t*)c.batch;
      }
      // other sizes: resized on the GPU like query images
      auto* hd = (ImageDesc*)c.aux_host;
      std::vector<void*> tmp;
      for (int64_t pos = g0; pos < g0 + cnt;) {
        const auto* pc = piece_for(*b, pos, c.device, copy);
        if (!pc) throw std::runtime_error("blob: image not staged");
        const int64_t hi = std::min(g0 + cnt, pc->first + pc->n);
        const uint8_t* base = (const uint8_t*)pc->dev + (size_t)(pos - pc->first) * ib;
        if (!peer(c.device, pc->device)) {
          void* d = nullptr;
          DMLC_HIP_CHECK(hipMallocAsync(&d, (size_t)(hi - pos) * ib, s));
          DMLC_HIP_CHECK(hipMemcpyPeerAsync(d, c.device, base, pc->device, (size_t)(hi - pos) * ib, s));
          tmp.push_back(d);
          base = (const uint8_t*)d;
        }
        for (int64_t i = pos; i < hi; ++i)
          hd[i - g0] = ImageDesc{base + (size_t)(i - pos) * ib, (int)b->si.h, (int)b->si.w};
        pos = hi;
      }
      resize_into(c, hd, cnt, s);
      for (void* d : tmp) DMLC_HIP_CHECK(hipFreeAsync(d, s));
      return (const uint8_t*)c.batch;
    };
    dp::Fleet::QueryOptions q;
    q.prefer_device = prefer;
    q.allow_scatter = false;
    fleet_->classify(model, n, stage, idx, prob, q);
  }

  static std::vector<Prediction> to_preds(const std::vector<int32_t>& idx, const std::vector<float>& prob) {
    std::vector<Prediction> out(idx.size());
    for (size_t i = 0; i < idx.size(); ++i) out[i] = Prediction{prob[i], idx[i]};
    return out;
  }

  void touch(std::unordered_map<std::string, Entry>::iterator it) { lru_.splice(lru_.begin(), lru_, it->second.lru); }

  void unpin(const std::vector<std::string>& paths) {
    std::lock_guard<std::mutex> g(cache_mu_);
    for (const auto& p : paths) {
      auto it = cache_.find(p);
      if (it != cache_.end()) --it->second.pins;
    }
  }

  std::shared_ptr<Stager> take_stager() {
    std::unique_lock<std::mutex> g(stager_mu_);
    stager_cv_.wait(g, [&] { return !free_stagers_.empty(); });
    auto s = free_stagers_.back();
    free_stagers_.pop_back();
    return s;
  }
  void give_stager(const std::shared_ptr<Stager>& s) {
    std::lock_guard<std::mutex> g(stager_mu_);
    free_stagers_.push_back(s);
    stager_cv_.notify_one();
  }

  // Decode and upload without holding the cache lock: the JPEG is decoded on
  // this thread into the stager's pinned buffer and DMA'd into a new HBM
  // block on the GPU holding the fewest cached bytes; only the final
  // insert/evict locks.
  void stage_one(const std::string& path, bool count_as_miss) {
    int home;
    {
      std::lock_guard<std::mutex> g(cache_mu_);
      auto it = cache_.find(path);
      if (it != cache_.end()) {
        if (count_as_miss) ++stats_.hits;
        touch(it);
        return;
      }
      home = devices_[0];
      size_t least = SIZE_MAX;
      const auto live = fleet_->live();
      for (int d : live)
        if (cache_bytes_dev_[d] < least) least = cache_bytes_dev_[d], home = d;
    }
    std::vector<uint8_t> jpeg;
    {
      std::ifstream f(path, std::ios::binary);
      if (!f) throw std::runtime_error("cannot open " + path);
      jpeg.assign(std::istreambuf_iterator<char>(f), std::istreambuf_iterator<char>());
    }
    // (kStagers = 2 x the decode threads of one query: holding a stager through
    // the decode leaves concurrent queries' misses decoding in parallel)
    auto st = take_stager();
    void* dev = nullptr;
    int img_h = 0, img_w = 0;
    size_t bytes = 0;
    try {
      decode_jpeg_into(jpeg.data(), jpeg.size(), [&](int w, int h) {
        img_w = w;
        img_h = h;
        bytes = (size_t)w * h * 3;
        st->ensure_pinned(bytes);
        return (uint8_t*)st->pinned[0];
      });
      hipStream_t s = st->stream(home);
      DMLC_HIP_CHECK(hipSetDevice(home));
      // plain hipMalloc: peer-mapped for the other GPUs' resize kernels
      // (stream-ordered pool memory would need per-pool access grants)
      DMLC_HIP_CHECK(hipMalloc(&dev, std::max<size_t>(bytes, 256)));
      DMLC_HIP_CHECK(hipMemcpyAsync(dev, st->pinned[0], bytes, hipMemcpyHostToDevice, s));
      DMLC_HIP_CHECK(hipStreamSynchronize(s));  // resident before it is visible
    } catch (...) {
      give_stager(st);
      if (dev) (void)hipFree(dev);
      throw;
    }
    give_stager(st);
    std::lock_guard<std::mutex> g(cache_mu_);
    if (cache_.count(path)) {  // raced with another stager
      (void)hipSetDevice(home);
      (void)hipFree(dev);
      return;
    }
    if (count_as_miss) ++stats_.misses; else ++stats_.staged;
    // evict least-recently-used entries no query has pinned
    auto victim = lru_.end();
    while (cache_bytes_ + bytes > cache_cap_ && victim != lru_.begin()) {
      --victim;
      auto it = cache_.find(*victim);
      if (it->second.pins > 0) continue;
      (void)hipSetDevice(it->second.device);
      (void)hipFree(it->second.dev);  // unpinned: no queued kernel reads it
      cache_bytes_ -= it->second.bytes;
      cache_bytes_dev_[it->second.device] -= it->second.bytes;
      cache_.erase(it);
      victim = lru_.erase(victim);
      ++stats_.evictions;
    }
    Entry en;
    en.dev = dev;
    en.device = home;
    en.h = img_h;
    en.w = img_w;
    en.bytes = bytes;
    lru_.push_front(path);
    en.lru = lru_.begin();
    cache_bytes_ += bytes;
    cache_bytes_dev_[home] += bytes;
    cache_.emplace(path, en);
  }

  std::vector<int> devices_;
  int max_batch_, lanes_;
  std::set<std::pair<int, int>> peers_;  // (reader, owner) with peer access enabled
  std::unique_ptr<dp::Fleet> fleet_;
  std::mutex weights_mu_;
  std::map<std::string, std::shared_ptr<const WeightMap>> weights_;  // host copies (fresh instances build from them)
  std::map<std::string, std::shared_ptr<HbmBlob>> hbm_blobs_;  // under blob_mu_
  std::mutex restage_mu_;  // one re-staging at a time
  mutable std::mutex cache_mu_;
  std::unordered_map<std::string, Entry> cache_;
  std::list<std::string> lru_;
  size_t cache_bytes_ = 0, cache_cap_;
  std::map<int, size_t> cache_bytes_dev_;
  CacheStats stats_;
  std::mutex stager_mu_;
  std::condition_variable stager_cv_;
  std::vector<std::shared_ptr<Stager>> free_stagers_;
};

}  // namespace

std::unique_ptr<Executor> make_executor(const std::string& backend, const std::vector<int>& devices, int max_batch,
                                        size_t cache_bytes, int min_shard, int lanes, int batch_window_us) {
  std::string b = backend;
  if (b == "auto") b = hip_device_count() > 0 ? "gpu" : "cpu";
  if (b == "gpu") {
    for (int d : devices)
      if (d < 0 || hip_device_count() <= d) throw std::runtime_error("no HIP device " + std::to_string(d));
    return std::make_unique<GpuExecutor>(devices, max_batch, cache_bytes, min_shard, lanes, batch_window_us);
  }
  if (b == "cpu") return std::make_unique<CpuExecutor>();
  throw std::invalid_argument("unknown executor backend: " + backend);
}

std::unique_ptr<Executor> make_executor(const std::string& backend, int device, int max_batch, size_t cache_bytes) {
  return make_executor(backend, std::vector<int>{device}, max_batch, cache_bytes, 32, 2);
}

}  // namespace dmlc
