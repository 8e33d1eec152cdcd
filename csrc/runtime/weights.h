// Host-side fp32 weight map shared by the checkpoint reader, the GPU engine
// and the CPU executor. Plain C++ (no HIP, no libtorch).
#pragma once
#include <cstdint>
#include <map>
#include <string>
#include <vector>

namespace dmlc {

struct HostTensor {
  std::vector<int64_t> shape;
  std::vector<float> data;
  int64_t numel() const {
    int64_t n = 1;
    for (auto s : shape) n *= s;
    return n;
  }
};
using WeightMap = std::map<std::string, HostTensor>;

}  // namespace dmlc
