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
#include <cstring>
#include <stdexcept>
#include <string>

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

}  // namespace dmlc
