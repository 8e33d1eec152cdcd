// Default (host-memory) blob store of the Executor interface: CPU and
// digest executors keep staged SDFS replicas in RAM; shards are decoded into
// Image structs and classified through predict(). The GPU executor
// overrides all of it with HBM-resident blobs (executor.cpp).
#include <fstream>
#include <iterator>

#include "executor.h"
#include "shard.h"

namespace dmlc {

void Executor::stage_blob(const std::string& key, const std::string& path) {
  std::ifstream f(path, std::ios::binary);
  if (!f) throw std::runtime_error("cannot open " + path);
  auto buf = std::make_shared<std::vector<uint8_t>>((std::istreambuf_iterator<char>(f)),
                                                    std::istreambuf_iterator<char>());
  std::lock_guard<std::mutex> g(blob_mu_);
  host_blobs_[key] = std::move(buf);
}

void Executor::drop_blob(const std::string& key) {
  std::lock_guard<std::mutex> g(blob_mu_);
  host_blobs_.erase(key);
}

std::vector<std::string> Executor::blob_keys() const {
  std::lock_guard<std::mutex> g(blob_mu_);
  std::vector<std::string> out;
  for (const auto& kv : host_blobs_) out.push_back(kv.first);
  return out;
}

std::vector<Prediction> Executor::predict_blob(const std::string& model, const std::string& key) {
  return predict_blob_range(model, key, 0, -1);
}

std::vector<Prediction> Executor::predict_blob_range(const std::string& model, const std::string& key, int64_t first,
                                                     int64_t count) {
  std::shared_ptr<const std::vector<uint8_t>> b;
  {
    std::lock_guard<std::mutex> g(blob_mu_);
    auto it = host_blobs_.find(key);
    if (it == host_blobs_.end()) throw std::runtime_error("blob not staged: " + key);
    b = it->second;
  }
  const ShardInfo s = parse_shard(b->data(), b->size());
  if (count < 0) count = (int64_t)s.n - first;
  if (first < 0 || count < 0 || first + count > (int64_t)s.n) throw std::runtime_error(key + ": image range out of bounds");
  std::vector<Image> imgs(count);
  for (int64_t i = 0; i < count; ++i) {
    imgs[i].height = (int)s.h;
    imgs[i].width = (int)s.w;
    const uint8_t* p = b->data() + kShardHeader + (size_t)(first + i) * s.image_bytes();
    imgs[i].rgb.assign(p, p + s.image_bytes());
  }
  return predict(model, imgs);
}

}  // namespace dmlc
