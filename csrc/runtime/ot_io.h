// `.ot` checkpoint I/O (libtorch serialize archives, the format tch-rs
// `VarStore::save/load` uses; reference load sites src/services.rs:516,522).
// Archive keys use '|' where the module path has '.', because
// torch::nn::Module parameter names may not contain dots.
#pragma once
#include <string>

#include "weights.h"

namespace dmlc {

WeightMap ot_load(const std::string& path);
void ot_save(const std::string& path, const WeightMap& weights);

}  // namespace dmlc
