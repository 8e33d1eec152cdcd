#include "sdfs.h"

#include <fstream>
#include <stdexcept>

#include "common.h"

namespace dmlc {
namespace ctl {

std::string sanitize_filename(const std::string& s) {
  std::string out;
  for (unsigned char c : s) {
    if (c < 0x20 || c == 0x7f) continue;
    if (std::string("/\\?<>:*|\"").find((char)c) != std::string::npos) continue;
    out.push_back((char)c);
  }
  if (out == "." || out == ".." || out.empty()) out = "_";
  if (out.size() > 255) out.resize(255);
  return out;
}

std::string storage_filename(const std::string& filename, int version) {
  return sanitize_filename("v" + std::to_string(version) + "." + filename);
}

std::string version_delimiter(int version) {
  const std::string mid = " Version " + std::to_string(version) + " ";
  if (mid.size() >= 40) return mid;
  const size_t pad = 40 - mid.size();
  return std::string(pad / 2, '=') + mid + std::string(pad - pad / 2, '=');
}

std::string versioned_sibling(const std::string& dest, int version) {
  const auto slash = dest.rfind('/');
  const std::string dir = slash == std::string::npos ? "" : dest.substr(0, slash + 1);
  const std::string base = slash == std::string::npos ? dest : dest.substr(slash + 1);
  return dir + "v" + std::to_string(version) + "." + base;
}

void merge_versions(const std::string& dest, const std::set<int>& versions) {
  std::ofstream out(dest, std::ios::binary | std::ios::trunc);
  if (!out) throw std::runtime_error("cannot write " + dest);
  for (auto it = versions.rbegin(); it != versions.rend(); ++it) {
    out << version_delimiter(*it) << "\n";
    std::ifstream in(versioned_sibling(dest, *it), std::ios::binary);
    if (!in) throw std::runtime_error("missing fetched version " + std::to_string(*it));
    out << in.rdbuf();
    out << "\n";
  }
}

std::set<Id> choose_replicas(const std::string& filename, const std::vector<Id>& candidates, int need) {
  std::set<Id> out;
  if (candidates.empty() || need <= 0) return out;
  const uint64_t h = fnv1a(filename);
  for (int i = 0; i < need; ++i) out.insert(candidates[(size_t)((h + (uint64_t)i) % candidates.size())]);
  return out;
}

void write_directory(Writer& w, const Directory& d) {
  w.u32((uint32_t)d.size());
  for (const auto& f : d) {
    w.str(f.first);
    w.u32((uint32_t)f.second.size());
    for (const auto& r : f.second) {
      write_id(w, r.first);
      w.u32((uint32_t)r.second.size());
      for (int v : r.second) w.i32(v);
    }
  }
}

Directory read_directory(Reader& r) {
  Directory d;
  uint32_t nf = r.u32();
  for (uint32_t i = 0; i < nf; ++i) {
    std::string f = r.str();
    auto& m = d[f];
    uint32_t nr = r.u32();
    for (uint32_t j = 0; j < nr; ++j) {
      Id id = read_id(r);
      auto& s = m[id];
      uint32_t nv = r.u32();
      for (uint32_t k = 0; k < nv; ++k) s.insert(r.i32());
    }
  }
  return d;
}

}  // namespace ctl
}  // namespace dmlc
