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
#include "shard.h"
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
// One or more GPUs of this node. Per model: an engine on every GPU and a
// dp::Group over them (GPU 0 coordinates; with more than one GPU the query
// batch is scattered over RCCL, csrc/comm/dp.h). Decoded images stay resident
// in GPU 0's HBM at their own sizes (LRU cache); a query's images, whatever
// their sizes, are resized into one u8 224x224 batch by one kernel
// (resize.hip) and classified by one graph-replayed forward per GPU.
class GpuExecutor : public Executor {
 public:
  GpuExecutor(std::vector<int> devices, int max_batch, size_t cache_bytes, int min_shard)
      : devices_(std::move(devices)), max_batch_(max_batch), min_shard_(min_shard), cache_cap_(cache_bytes) {
    if (devices_.empty()) throw std::invalid_argument("GpuExecutor: no devices");
    DMLC_HIP_CHECK(hipSetDevice(devices_[0]));
    for (int i = 0; i < kStagers; ++i) {
      Stager st;
      DMLC_HIP_CHECK(hipStreamCreateWithFlags(&st.stream, hipStreamNonBlocking));
      free_stagers_.push_back(st);
    }
  }
  ~GpuExecutor() override {
    (void)hipSetDevice(devices_[0]);
    (void)hipDeviceSynchronize();
    {
      std::lock_guard<std::mutex> g(models_mu_);
      models_.clear();
    }
    (void)hipSetDevice(devices_[0]);
    for (auto& kv : cache_) (void)hipFree(kv.second.dev);
    for (auto& st : free_stagers_) {
      if (st.pinned) (void)hipHostFree(st.pinned);
      (void)hipStreamDestroy(st.stream);
    }
  }
  std::string backend() const override {
    std::string b = "gpu:" + std::to_string(devices_[0]);
    for (size_t i = 1; i < devices_.size(); ++i) b += "," + std::to_string(devices_[i]);
    return b;
  }

  void load_model(const std::string& model, const std::string& path) override {
    load_model_weights(model, ot_load(path));
  }
  void load_model_weights(const std::string& model, const WeightMap& w) override {
    // Build the new replicas outside the lock; in-flight queries keep the old
    // slot alive (shared_ptr) until they finish: a hot swap.
    auto slot = std::make_shared<ModelSlot>(model, w, devices_, max_batch_, min_shard_);
    std::lock_guard<std::mutex> g(models_mu_);
    models_[model] = std::move(slot);
  }
  bool has_model(const std::string& model) const override {
    std::lock_guard<std::mutex> g(models_mu_);
    return models_.count(model) > 0;
  }

  std::vector<Prediction> predict(const std::string& model, const std::vector<Image>& imgs) override {
    auto slot = get(model);
    DMLC_HIP_CHECK(hipSetDevice(devices_[0]));
    std::vector<ImageDesc> descs(imgs.size());
    std::vector<void*> bufs;
    for (size_t i = 0; i < imgs.size(); ++i) {
      void* d = nullptr;
      DMLC_HIP_CHECK(hipMalloc(&d, imgs[i].rgb.size()));
      DMLC_HIP_CHECK(hipMemcpy(d, imgs[i].rgb.data(), imgs[i].rgb.size(), hipMemcpyHostToDevice));
      bufs.push_back(d);
      descs[i] = ImageDesc{(const uint8_t*)d, imgs[i].height, imgs[i].width};
    }
    std::vector<Prediction> out;
    try {
      out = slot->run(descs);
    } catch (...) {
      for (void* b : bufs) (void)hipFree(b);
      throw;
    }
    for (void* b : bufs) (void)hipFree(b);
    return out;
  }

  // HBM-resident decoded images: a hit skips the JPEG decode and the H2D
  // copy. The query's entries are pinned (not evictable) until its forward
  // has consumed them.
  std::vector<Prediction> predict_files(const std::string& model, const std::vector<std::string>& paths) override {
    auto slot = get(model);  // fail fast on an unknown model
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
    std::vector<ImageDesc> descs(paths.size());
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
        descs[i] = ImageDesc{(const uint8_t*)it->second.dev, it->second.h, it->second.w};
      }
    }
    std::vector<Prediction> out;
    try {
      out = slot->run(descs);
    } catch (...) {
      unpin(pinned);
      throw;
    }
    unpin(pinned);
    return out;
  }

  bool stage(const std::string& path) override {
    stage_one(path, /*count_as_miss=*/false);
    return true;
  }

  // ---- SDFS replicas resident in the coordinator GPU's HBM
  std::string blob_location() const override { return "hbm:gpu" + std::to_string(devices_[0]); }

  void stage_blob(const std::string& key, const std::string& path) override {
    std::ifstream f(path, std::ios::binary);
    if (!f) throw std::runtime_error("cannot open " + path);
    f.seekg(0, std::ios::end);
    const size_t bytes = (size_t)f.tellg();
    f.seekg(0);
    auto b = std::make_shared<HbmBlob>();
    b->bytes = bytes;
    b->device = devices_[0];
    DMLC_HIP_CHECK(hipSetDevice(devices_[0]));
    DMLC_HIP_CHECK(hipMalloc(&b->dev, std::max<size_t>(bytes, 256)));
    // pinned bounce buffer, 32 MB chunks, H2D on a stager's side stream
    Stager st = take_stager();
    try {
      constexpr size_t kChunk = (size_t)32 << 20;
      if (st.pinned_bytes < std::min(kChunk, bytes)) {
        if (st.pinned) DMLC_HIP_CHECK(hipHostFree(st.pinned));
        st.pinned = nullptr;
        st.pinned_bytes = 0;
        DMLC_HIP_CHECK(hipHostMalloc(&st.pinned, std::min(kChunk, std::max<size_t>(bytes, 256)), hipHostMallocDefault));
        st.pinned_bytes = std::min(kChunk, std::max<size_t>(bytes, 256));
      }
      for (size_t off = 0; off < bytes;) {
        const size_t n = std::min(st.pinned_bytes, bytes - off);
        f.read((char*)st.pinned, (std::streamsize)n);
        if (off == 0 && n >= kShardHeader) std::memcpy(b->head, st.pinned, kShardHeader);
        DMLC_HIP_CHECK(hipMemcpyAsync((uint8_t*)b->dev + off, st.pinned, n, hipMemcpyHostToDevice, st.stream));
        DMLC_HIP_CHECK(hipStreamSynchronize(st.stream));
        off += n;
      }
    } catch (...) {
      give_stager(st);
      throw;
    }
    give_stager(st);
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
  std::vector<Prediction> predict_blob(const std::string& model, const std::string& key) override {
    auto slot = get(model);
    std::shared_ptr<HbmBlob> b;
    {
      std::lock_guard<std::mutex> g(blob_mu_);
      auto it = hbm_blobs_.find(key);
      if (it == hbm_blobs_.end()) throw std::runtime_error("blob not staged: " + key);
      b = it->second;
    }
    if (b->bytes < kShardHeader || !is_shard(b->head, kShardHeader)) throw std::runtime_error(key + " is not a u8 shard");
    ShardInfo si;
    std::memcpy(&si.n, b->head + 8, 4);
    std::memcpy(&si.h, b->head + 12, 4);
    std::memcpy(&si.w, b->head + 16, 4);
    if (si.h == 0 || si.w == 0 || (uint64_t)si.n * si.image_bytes() + kShardHeader != b->bytes)
      throw std::runtime_error(key + ": bad shard header");
    const uint8_t* data = (const uint8_t*)b->dev + kShardHeader;
    if (si.h == ModelSlot::kS && si.w == ModelSlot::kS) return slot->run_dense(data, si.n);
    std::vector<ImageDesc> descs(si.n);
    for (uint32_t i = 0; i < si.n; ++i) descs[i] = ImageDesc{data + (size_t)i * si.image_bytes(), (int)si.h, (int)si.w};
    return slot->run(descs);
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
  static constexpr size_t kDecodeThreads = 8;
  static constexpr int kStagers = 16;  // held through a miss's decode (it decodes into the pinned buffer)

  // One model replicated on every GPU of the executor.
  struct ModelSlot {
    ModelSlot(const std::string& arch, const WeightMap& w, const std::vector<int>& devices, int max_batch,
              int min_shard)
        : max_batch(max_batch) {
      // The host packs the weights once (engine 0, one H2D copy); the other
      // GPUs get replicas whose arenas are filled by one RCCL broadcast over
      // xGMI (`train` = distribute + hot-swap).
      for (size_t k = 0; k < devices.size(); ++k) {
        DMLC_HIP_CHECK(hipSetDevice(devices[k]));
        if (k == 0) engines.push_back(std::make_unique<Engine>(arch, w, devices[0]));
        else engines.push_back(std::make_unique<Engine>(*engines[0], devices[k]));
        engines.back()->reserve(max_batch);
      }
      if (devices.size() > 1) {
        auto comms = comm::rccl_init_all(devices);
        comms[0]->group_start();
        for (size_t k = 0; k < devices.size(); ++k) {
          DMLC_HIP_CHECK(hipSetDevice(devices[k]));
          comms[k]->broadcast(engines[0]->weight_arena(), engines[k]->weight_arena(), engines[0]->weight_bytes(), 0,
                              engines[k]->stream());
        }
        comms[0]->group_end();
        for (size_t k = 0; k < devices.size(); ++k) {
          DMLC_HIP_CHECK(hipSetDevice(devices[k]));
          DMLC_HIP_CHECK(hipStreamSynchronize(engines[k]->stream()));
        }
      }
      // Two compute lanes per GPU (dp::Worker::lanes): a second instance of
      // the model whose forward overlaps the previous step's tail (+9% at
      // ResNet18 b256: profiles/r2_lanes.txt).
      for (size_t k = 0; k < devices.size(); ++k) {
        DMLC_HIP_CHECK(hipSetDevice(devices[k]));
        lane2.push_back(std::make_unique<Engine>(*engines[k], devices[k]));
        lane2.back()->copy_weights_from(*engines[k]);
        lane2.back()->reserve(max_batch);
        workers.push_back(dp::make_hip_worker(engines[k].get(), kS, kS, /*use_graph=*/true, {lane2.back().get()}));
      }
      std::vector<dp::Worker*> ws;
      for (auto& x : workers) ws.push_back(x.get());
      auto factory = [devices](const std::vector<int>& members) {
        std::vector<int> devs;
        for (int m : members) devs.push_back(devices.at(m));
        return comm::rccl_init_all(devs);
      };
      group = std::make_unique<dp::Group>(ws, factory, max_batch, (size_t)kS * kS * 3);
      group->set_min_per_rank(min_shard);
      dp::Worker* c = group->coordinator();
      c->activate();
      batch = c->alloc((size_t)max_batch * kS * kS * 3);
      d_descs = c->alloc((size_t)max_batch * sizeof(ImageDesc));
      h_descs = (ImageDesc*)c->alloc_host((size_t)max_batch * sizeof(ImageDesc));
      ev_src = c->new_event();
    }
    ~ModelSlot() {
      dp::Worker* c = group->coordinator();
      c->activate();
      c->sync_all();
      c->dealloc(batch);
      c->dealloc(d_descs);
      c->dealloc_host(h_descs);
      group.reset();
      workers.clear();
      lane2.clear();
      engines.clear();
    }
    // Resize the images into one u8 batch on the coordinator, then classify
    // it across the group.
    std::vector<Prediction> run(const std::vector<ImageDesc>& descs) {
      DMLC_TRACE("executor.forward");
      std::lock_guard<std::mutex> g(mu);
      std::vector<Prediction> out(descs.size());
      dp::Worker* c = group->coordinator();
      c->activate();
      auto s = (hipStream_t)c->stream(dp::Worker::kCompute);
      for (size_t first = 0; first < descs.size(); first += (size_t)max_batch) {
        const int B = (int)std::min(descs.size() - first, (size_t)max_batch);
        c->sync(ev_src);  // the previous chunk's resize has read h_descs
        std::memcpy(h_descs, descs.data() + first, (size_t)B * sizeof(ImageDesc));
        DMLC_HIP_CHECK(hipMemcpyAsync(d_descs, h_descs, (size_t)B * sizeof(ImageDesc), hipMemcpyHostToDevice, s));
        resize_u8_ragged((const ImageDesc*)d_descs, (uint8_t*)batch, B, kS, s);
        c->record(ev_src, dp::Worker::kCompute);
        std::vector<int32_t> idx(B);
        std::vector<float> prob(B);
        group->classify((const uint8_t*)batch, B, idx.data(), prob.data(), ev_src);
        for (int b = 0; b < B; ++b) out[first + b] = Prediction{prob[b], idx[b]};
      }
      return out;
    }
    // Images already u8 224x224 in coordinator memory (a staged shard):
    // straight into the group, no resize copy.
    std::vector<Prediction> run_dense(const uint8_t* src, int64_t n) {
      DMLC_TRACE("executor.forward_dense");
      std::lock_guard<std::mutex> g(mu);
      std::vector<int32_t> idx(n);
      std::vector<float> prob(n);
      group->coordinator()->activate();
      group->classify(src, n, idx.data(), prob.data());
      std::vector<Prediction> out(n);
      for (int64_t i = 0; i < n; ++i) out[i] = Prediction{prob[i], idx[i]};
      return out;
    }
    static constexpr int kS = 224;
    int max_batch;
    std::vector<std::unique_ptr<Engine>> engines;
    std::vector<std::unique_ptr<Engine>> lane2;  // second compute lane per GPU
    std::vector<std::unique_ptr<dp::Worker>> workers;
    std::unique_ptr<dp::Group> group;
    void* batch = nullptr;
    void* d_descs = nullptr;
    ImageDesc* h_descs = nullptr;
    int ev_src = -1;
    std::mutex mu;  // one query batch at a time per model
  };

  struct Entry {
    void* dev = nullptr;
    int h = 0, w = 0;
    size_t bytes = 0;
    int pins = 0;
    std::list<std::string>::iterator lru;
  };
  struct HbmBlob {
    void* dev = nullptr;
    size_t bytes = 0;
    int device = 0;
    uint8_t head[kShardHeader] = {};  // host copy of the first bytes (shard header)
    ~HbmBlob() {
      if (dev) {
        (void)hipSetDevice(device);
        (void)hipFree(dev);
      }
    }
  };
  std::map<std::string, std::shared_ptr<HbmBlob>> hbm_blobs_;  // under blob_mu_
  struct Stager {
    hipStream_t stream = nullptr;
    void* pinned = nullptr;
    size_t pinned_bytes = 0;
  };

  std::shared_ptr<ModelSlot> get(const std::string& model) const {
    std::lock_guard<std::mutex> g(models_mu_);
    auto it = models_.find(model);
    if (it == models_.end()) throw std::runtime_error("model not loaded: " + model);
    return it->second;
  }

  void touch(std::unordered_map<std::string, Entry>::iterator it) { lru_.splice(lru_.begin(), lru_, it->second.lru); }

  void unpin(const std::vector<std::string>& paths) {
    std::lock_guard<std::mutex> g(cache_mu_);
    for (const auto& p : paths) {
      auto it = cache_.find(p);
      if (it != cache_.end()) --it->second.pins;
    }
  }

  Stager take_stager() {
    std::unique_lock<std::mutex> g(stager_mu_);
    stager_cv_.wait(g, [&] { return !free_stagers_.empty(); });
    Stager s = free_stagers_.back();
    free_stagers_.pop_back();
    return s;
  }
  void give_stager(const Stager& s) {
    std::lock_guard<std::mutex> g(stager_mu_);
    free_stagers_.push_back(s);
    stager_cv_.notify_one();
  }

  // Decode and upload without holding the cache lock: the JPEG is decoded on
  // this thread, copied into the stager's pinned buffer and DMA'd into a new
  // HBM block on the stager's stream; only the final insert/evict locks.
  void stage_one(const std::string& path, bool count_as_miss) {
    {
      std::lock_guard<std::mutex> g(cache_mu_);
      auto it = cache_.find(path);
      if (it != cache_.end()) {
        if (count_as_miss) ++stats_.hits;
        touch(it);
        return;
      }
    }
    std::vector<uint8_t> jpeg;
    {
      std::ifstream f(path, std::ios::binary);
      if (!f) throw std::runtime_error("cannot open " + path);
      jpeg.assign(std::istreambuf_iterator<char>(f), std::istreambuf_iterator<char>());
    }
    // (kStagers = 2 x the decode threads of one query: holding a stager through
    // the decode leaves concurrent queries' misses decoding in parallel)
    Stager st = take_stager();
    void* dev = nullptr;
    int img_h = 0, img_w = 0;
    size_t bytes = 0;
    try {
      DMLC_HIP_CHECK(hipSetDevice(devices_[0]));
      // decoded straight into the stager's pinned buffer: no RGB vector to
      // zero-fill and copy per query image
      decode_jpeg_into(jpeg.data(), jpeg.size(), [&](int w, int h) {
        img_w = w;
        img_h = h;
        bytes = (size_t)w * h * 3;
        if (st.pinned_bytes < bytes) {
          if (st.pinned) DMLC_HIP_CHECK(hipHostFree(st.pinned));
          st.pinned = nullptr;
          st.pinned_bytes = 0;
          DMLC_HIP_CHECK(hipHostMalloc(&st.pinned, bytes, hipHostMallocDefault));
          st.pinned_bytes = bytes;
        }
        return (uint8_t*)st.pinned;
      });
      DMLC_HIP_CHECK(hipMallocAsync(&dev, bytes, st.stream));
      DMLC_HIP_CHECK(hipMemcpyAsync(dev, st.pinned, bytes, hipMemcpyHostToDevice, st.stream));
      DMLC_HIP_CHECK(hipStreamSynchronize(st.stream));  // resident before it is visible
    } catch (...) {
      give_stager(st);
      throw;
    }
    give_stager(st);
    std::lock_guard<std::mutex> g(cache_mu_);
    if (cache_.count(path)) {  // raced with another stager
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
      (void)hipFree(it->second.dev);  // unpinned: no queued kernel reads it
      cache_bytes_ -= it->second.bytes;
      cache_.erase(it);
      victim = lru_.erase(victim);
      ++stats_.evictions;
    }
    Entry en;
    en.dev = dev;
    en.h = img_h;
    en.w = img_w;
    en.bytes = bytes;
    lru_.push_front(path);
    en.lru = lru_.begin();
    cache_bytes_ += bytes;
    cache_.emplace(path, en);
  }

  std::vector<int> devices_;
  int max_batch_, min_shard_;
  mutable std::mutex models_mu_;
  std::map<std::string, std::shared_ptr<ModelSlot>> models_;
  mutable std::mutex cache_mu_;
  std::unordered_map<std::string, Entry> cache_;
  std::list<std::string> lru_;
  size_t cache_bytes_ = 0, cache_cap_;
  CacheStats stats_;
  std::mutex stager_mu_;
  std::condition_variable stager_cv_;
  std::vector<Stager> free_stagers_;
};

}  // namespace

std::unique_ptr<Executor> make_executor(const std::string& backend, const std::vector<int>& devices, int max_batch,
                                        size_t cache_bytes, int min_shard) {
  std::string b = backend;
  if (b == "auto") b = hip_device_count() > 0 ? "gpu" : "cpu";
  if (b == "gpu") {
    for (int d : devices)
      if (d < 0 || hip_device_count() <= d) throw std::runtime_error("no HIP device " + std::to_string(d));
    return std::make_unique<GpuExecutor>(devices, max_batch, cache_bytes, min_shard);
  }
  if (b == "cpu") return std::make_unique<CpuExecutor>();
  throw std::invalid_argument("unknown executor backend: " + backend);
}

std::unique_ptr<Executor> make_executor(const std::string& backend, int device, int max_batch, size_t cache_bytes) {
  return make_executor(backend, std::vector<int>{device}, max_batch, cache_bytes, 1);
}

}  // namespace dmlc
