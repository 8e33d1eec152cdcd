// Shared control-plane utilities: clocks, logging, hashing, string helpers.
//
// Reference: the Rust node logs with simple_logging to "<hostname>.log" at
// Info (src/main.rs:28) and compares chrono::Local wall-clock timestamps
// across nodes (src/membership.rs:116,173,204,238,310). We keep wall-clock
// microseconds for membership LWW (nodes share NTP / one machine) and use the
// steady clock for every local period and latency.
#pragma once
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <mutex>
#include <sstream>
#include <string>
#include <vector>

namespace dmlc {
namespace ctl {

inline int64_t wall_us() {
  return std::chrono::duration_cast<std::chrono::microseconds>(
             std::chrono::system_clock::now().time_since_epoch())
      .count();
}

inline int64_t steady_us() {
  return std::chrono::duration_cast<std::chrono::microseconds>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

// "2026-10-15 22:10:01.123456" in local time.
std::string format_time_us(int64_t us);

// FNV-1a 64: deterministic across processes (replica placement hash; the
// reference used SipHash DefaultHasher, src/services.rs:346-364).
inline uint64_t fnv1a(const std::string& s) {
  uint64_t h = 1469598103934665603ull;
  for (unsigned char c : s) {
    h ^= c;
    h *= 1099511628211ull;
  }
  return h;
}

std::vector<std::string> split(const std::string& s, char sep);
std::vector<std::string> split_ws(const std::string& s);
std::string trim(const std::string& s);
bool starts_with(const std::string& s, const std::string& p);

// Thread-safe line logger (file), levels INFO/WARN/ERROR.
class Logger {
 public:
  static Logger& get();
  void open(const std::string& path);
  void log(const char* level, const std::string& msg);
  void close();

 private:
  std::mutex mu_;
  FILE* f_ = nullptr;
};

#define DMLC_LOG_INFO(msg)                                      \
  do {                                                          \
    std::ostringstream _os;                                     \
    _os << msg;                                                 \
    ::dmlc::ctl::Logger::get().log("INFO", _os.str());          \
  } while (0)
#define DMLC_LOG_WARN(msg)                                      \
  do {                                                          \
    std::ostringstream _os;                                     \
    _os << msg;                                                 \
    ::dmlc::ctl::Logger::get().log("WARN", _os.str());          \
  } while (0)

// stdout printing shared by REPL and background threads (one lock so lines
// from concurrent jobs never interleave).
void out_line(const std::string& s);

}  // namespace ctl
}  // namespace dmlc
