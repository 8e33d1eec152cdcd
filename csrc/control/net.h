// Thin POSIX socket helpers (UDP datagrams, TCP streams) with timeouts.
#pragma once
#include <netinet/in.h>

#include <cstdint>
#include <string>

namespace dmlc {
namespace ctl {

struct NetError : std::exception {
  explicit NetError(std::string m, bool timeout = false) : msg(std::move(m)), timed_out(timeout) {}
  const char* what() const noexcept override { return msg.c_str(); }
  std::string msg;
  bool timed_out = false;  // a send / recv deadline passed (the peer is there but silent)
};

// "host:port" -> sockaddr_in (IPv4; hostnames resolved with getaddrinfo).
sockaddr_in resolve(const std::string& host, int port);
sockaddr_in resolve_addr(const std::string& host_port);
std::string host_of(const std::string& host_port);
int port_of(const std::string& host_port);

// RAII file descriptor.
class Fd {
 public:
  Fd() = default;
  explicit Fd(int fd) : fd_(fd) {}
  ~Fd() { reset(); }
  Fd(Fd&& o) noexcept : fd_(o.release()) {}
  Fd& operator=(Fd&& o) noexcept {
    if (this != &o) {
      reset();
      fd_ = o.release();
    }
    return *this;
  }
  Fd(const Fd&) = delete;
  Fd& operator=(const Fd&) = delete;
  int get() const { return fd_; }
  int release() {
    int f = fd_;
    fd_ = -1;
    return f;
  }
  void reset();
  explicit operator bool() const { return fd_ >= 0; }

 private:
  int fd_ = -1;
};

Fd udp_bind(const std::string& host, int port);  // port 0 = ephemeral
bool udp_send(int fd, const sockaddr_in& to, const std::string& data);
// Returns bytes received, 0 on timeout. `from` filled on success.
int udp_recv(int fd, char* buf, size_t cap, int timeout_ms, sockaddr_in* from);

Fd tcp_listen(const std::string& host, int port, int backlog = 128);
// Accept with timeout; returns invalid Fd on timeout.
Fd tcp_accept(int lfd, int timeout_ms);
Fd tcp_connect(const std::string& host, int port, int timeout_ms);
void set_timeouts(int fd, int timeout_ms);
void send_all(int fd, const void* p, size_t n);
// false on orderly EOF before any byte; throws on error/timeout/partial read.
bool recv_all(int fd, void* p, size_t n);

}  // namespace ctl
}  // namespace dmlc
