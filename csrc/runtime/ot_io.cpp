// `.ot` reader/writer on libtorch's serialize archives (see ot_io.h).
#include "ot_io.h"

#include <torch/serialize/archive.h>
#include <torch/torch.h>

#include <algorithm>

namespace dmlc {

namespace {
std::string to_archive_key(std::string k) {
  std::replace(k.begin(), k.end(), '.', '|');
  return k;
}
std::string from_archive_key(std::string k) {
  std::replace(k.begin(), k.end(), '|', '.');
  return k;
}
}  // namespace

WeightMap ot_load(const std::string& path) {
  torch::serialize::InputArchive ar;
  ar.load_from(path, torch::Device(torch::kCPU));
  WeightMap out;
  for (const auto& key : ar.keys()) {
    torch::Tensor t;
    if (!ar.try_read(key, t, /*is_buffer=*/false) && !ar.try_read(key, t, /*is_buffer=*/true)) continue;
    t = t.to(torch::kFloat32).contiguous();
    HostTensor h;
    h.shape.assign(t.sizes().begin(), t.sizes().end());
    h.data.assign(t.data_ptr<float>(), t.data_ptr<float>() + t.numel());
    out.emplace(from_archive_key(key), std::move(h));
  }
  return out;
}

void ot_save(const std::string& path, const WeightMap& weights) {
  torch::serialize::OutputArchive ar;
  for (const auto& kv : weights) {
    auto t = torch::from_blob(const_cast<float*>(kv.second.data.data()), kv.second.shape,
                              torch::kFloat32)
                 .clone();
    ar.write(to_archive_key(kv.first), t, /*is_buffer=*/false);
  }
  ar.save_to(path);
}

}  // namespace dmlc
