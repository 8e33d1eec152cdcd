// u8 image shard: the unit of dataset data the SDFS stores for the
// data-parallel path (BASELINE config 3: "SDFS-staged imagenet_1k shards").
// File = 32-byte header {magic "DMLCU8S1", u32 n, u32 h, u32 w, u32 label0,
// u32 flags, 4 zero bytes} then n images u8 [h, w, 3] back to back (already
// decoded and resized, so a shard
// resident in HBM is classified with no host I/O: the RCCL scatter reads it
// directly). flags bit 0: labelled, image i of the shard is class label0 + i
// (tools/make_shards.py cuts the reference's imagenet_1k, one image per
// class in wnid order, into such shards). Written by
// dmlc.utils.shards.write_shard.
#pragma once
#include <cstdint>
#include <algorithm>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

namespace dmlc {

constexpr char kShardMagic[8] = {'D', 'M', 'L', 'C', 'U', '8', 'S', '1'};
constexpr size_t kShardHeader = 32;

struct ShardInfo {
  uint32_t n = 0, h = 0, w = 0;
  uint32_t label0 = 0;
  bool labelled = false;
  size_t image_bytes() const { return (size_t)h * w * 3; }
};

inline bool is_shard(const uint8_t* p, size_t bytes) {
  return bytes >= kShardHeader && std::memcmp(p, kShardMagic, 8) == 0;
}

inline ShardInfo parse_shard(const uint8_t* p, size_t bytes) {
  if (!is_shard(p, bytes)) throw std::runtime_error("not a dmlc u8 shard");
  ShardInfo s;
  std::memcpy(&s.n, p + 8, 4);
  std::memcpy(&s.h, p + 12, 4);
  std::memcpy(&s.w, p + 16, 4);
  uint32_t flags = 0;
  std::memcpy(&s.label0, p + 20, 4);
  std::memcpy(&flags, p + 24, 4);
  s.labelled = flags & 1u;
  if (s.h == 0 || s.w == 0 || s.h > 4096 || s.w > 4096) throw std::runtime_error("shard: bad image size");
  if ((uint64_t)s.n * s.image_bytes() != bytes - kShardHeader) throw std::runtime_error("shard: size mismatch");
  return s;
}

// Placement of a shard replica's images over the GPUs of a node: one
// contiguous slice per live GPU (in the order given), as even as possible,
// never an empty slice (fewer images than GPUs: the first n GPUs get one).
struct ShardSlice {
  int device = 0;
  int64_t first = 0, n = 0;
};
inline std::vector<ShardSlice> shard_slices(int64_t n, const std::vector<int>& devices) {
  if (devices.empty()) throw std::runtime_error("shard_slices: no device");
  const int64_t P = std::max<int64_t>(1, std::min<int64_t>((int64_t)devices.size(), n));
  std::vector<ShardSlice> out;
  for (int64_t k = 0; k < P; ++k) {
    ShardSlice s;
    s.device = devices[k];
    s.first = n * k / P;
    s.n = n * (k + 1) / P - s.first;
    out.push_back(s);
  }
  return out;
}

// Placement of a shard replica over the node's serving partitions (the GPU
// sets dp::Fleet gives each model): one full copy per distinct partition,
// sliced over that partition's GPUs with shard_slices, so every model finds
// every image of the shard in the HBM of a GPU it serves from (both jobs run
// over the same shards: a single copy spread over all GPUs had each model
// read half its ranges over xGMI). Identical partitions (fewer GPUs than
// models: the models share their GPU) share one copy; a device listed in
// several partitions holds one slice per copy it is part of. copy = index of
// the partition copy the slice belongs to.
struct PlacedSlice {
  int copy = 0;
  ShardSlice slice;
};
inline std::vector<PlacedSlice> shard_placement(int64_t n, const std::vector<std::vector<int>>& partitions) {
  std::vector<std::vector<int>> copies;
  for (auto p : partitions) {
    if (p.empty()) continue;
    std::sort(p.begin(), p.end());
    p.erase(std::unique(p.begin(), p.end()), p.end());
    if (std::find(copies.begin(), copies.end(), p) == copies.end()) copies.push_back(p);
  }
  if (copies.empty()) throw std::runtime_error("shard_placement: no partition");
  std::vector<PlacedSlice> out;
  for (size_t c = 0; c < copies.size(); ++c)
    for (const ShardSlice& s : shard_slices(n, copies[c])) out.push_back(PlacedSlice{(int)c, s});
  return out;
}

}  // namespace dmlc
