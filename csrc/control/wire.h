// Binary wire codec for the control plane (membership datagrams and RPC
// payloads): little-endian fixed-width integers, length-prefixed strings and
// sequences. Replaces flexbuffers (membership, src/membership.rs:293-300) and
// tarpc's JSON (RPC, src/main.rs:43-83); wire compatibility with the Rust
// node is not a goal.
#pragma once
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

namespace dmlc {
namespace ctl {

struct WireError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

class Writer {
 public:
  Writer& u8(uint8_t v) {
    buf_.push_back((char)v);
    return *this;
  }
  Writer& u16(uint16_t v) { return raw(&v, 2); }
  Writer& u32(uint32_t v) { return raw(&v, 4); }
  Writer& i32(int32_t v) { return raw(&v, 4); }
  Writer& u64(uint64_t v) { return raw(&v, 8); }
  Writer& i64(int64_t v) { return raw(&v, 8); }
  Writer& f64(double v) { return raw(&v, 8); }
  Writer& boolean(bool v) { return u8(v ? 1 : 0); }
  Writer& str(const std::string& s) {
    u32((uint32_t)s.size());
    buf_.append(s);
    return *this;
  }
  Writer& bytes(const void* p, size_t n) {
    u32((uint32_t)n);
    buf_.append((const char*)p, n);
    return *this;
  }
  const std::string& data() const { return buf_; }
  std::string take() { return std::move(buf_); }

 private:
  Writer& raw(const void* p, size_t n) {
    buf_.append((const char*)p, n);
    return *this;
  }
  std::string buf_;
};

class Reader {
 public:
  Reader(const char* p, size_t n) : p_(p), end_(p + n) {}
  explicit Reader(const std::string& s) : Reader(s.data(), s.size()) {}
  // Owning form for temporaries (e.g. Reader r(client.call(...))).
  explicit Reader(std::string&& s) : own_(std::move(s)), p_(own_.data()), end_(own_.data() + own_.size()) {}
  Reader(const Reader&) = delete;
  Reader& operator=(const Reader&) = delete;
  uint8_t u8() {
    need(1);
    return (uint8_t)*p_++;
  }
  uint16_t u16() { return get<uint16_t>(); }
  uint32_t u32() { return get<uint32_t>(); }
  int32_t i32() { return get<int32_t>(); }
  uint64_t u64() { return get<uint64_t>(); }
  int64_t i64() { return get<int64_t>(); }
  double f64() { return get<double>(); }
  bool boolean() { return u8() != 0; }
  std::string str() {
    uint32_t n = u32();
    need(n);
    std::string s(p_, n);
    p_ += n;
    return s;
  }
  bool done() const { return p_ == end_; }
  size_t left() const { return (size_t)(end_ - p_); }

 private:
  template <typename T>
  T get() {
    need(sizeof(T));
    T v;
    std::memcpy(&v, p_, sizeof(T));
    p_ += sizeof(T);
    return v;
  }
  void need(size_t n) {
    if ((size_t)(end_ - p_) < n) throw WireError("truncated message");
  }
  std::string own_;
  const char* p_;
  const char* end_;
};

}  // namespace ctl
}  // namespace dmlc
