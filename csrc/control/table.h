// ASCII tables in the style of the `tabled` crate the reference prints with
// (src/main.rs:134,184,200; src/membership.rs:107,129,218).
#pragma once
#include <algorithm>
#include <string>
#include <vector>

namespace dmlc {
namespace ctl {

inline std::string make_table(const std::vector<std::string>& headers,
                              const std::vector<std::vector<std::string>>& rows) {
  std::vector<size_t> w(headers.size());
  for (size_t i = 0; i < headers.size(); ++i) w[i] = headers[i].size();
  for (const auto& r : rows)
    for (size_t i = 0; i < r.size() && i < w.size(); ++i) w[i] = std::max(w[i], r[i].size());
  auto sep = [&] {
    std::string s = "+";
    for (size_t x : w) s += std::string(x + 2, '-') + "+";
    return s;
  };
  auto line = [&](const std::vector<std::string>& c) {
    std::string s = "|";
    for (size_t i = 0; i < w.size(); ++i) {
      const std::string v = i < c.size() ? c[i] : "";
      s += " " + v + std::string(w[i] - v.size(), ' ') + " |";
    }
    return s;
  };
  std::string out = sep() + "\n" + line(headers) + "\n" + sep() + "\n";
  for (const auto& r : rows) out += line(r) + "\n" + sep() + "\n";
  if (!out.empty()) out.pop_back();
  return out;
}

}  // namespace ctl
}  // namespace dmlc
