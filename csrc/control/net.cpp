#include "net.h"

#include <arpa/inet.h>
#include <errno.h>
#include <fcntl.h>
#include <netdb.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <cstring>

namespace dmlc {
namespace ctl {

void Fd::reset() {
  if (fd_ >= 0) ::close(fd_);
  fd_ = -1;
}

sockaddr_in resolve(const std::string& host, int port) {
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_port = htons((uint16_t)port);
  if (host.empty() || host == "0.0.0.0") {
    a.sin_addr.s_addr = INADDR_ANY;
    return a;
  }
  if (inet_pton(AF_INET, host.c_str(), &a.sin_addr) == 1) return a;
  addrinfo hints{}, *res = nullptr;
  hints.ai_family = AF_INET;
  if (getaddrinfo(host.c_str(), nullptr, &hints, &res) != 0 || !res)
    throw NetError("cannot resolve host " + host);
  a.sin_addr = ((sockaddr_in*)res->ai_addr)->sin_addr;
  freeaddrinfo(res);
  return a;
}

std::string host_of(const std::string& hp) {
  auto i = hp.rfind(':');
  return i == std::string::npos ? hp : hp.substr(0, i);
}

int port_of(const std::string& hp) {
  auto i = hp.rfind(':');
  if (i == std::string::npos) throw NetError("address without port: " + hp);
  return std::stoi(hp.substr(i + 1));
}

sockaddr_in resolve_addr(const std::string& hp) { return resolve(host_of(hp), port_of(hp)); }

Fd udp_bind(const std::string& host, int port) {
  Fd fd(::socket(AF_INET, SOCK_DGRAM | SOCK_CLOEXEC, 0));
  if (!fd) throw NetError("socket(udp) failed");
  int one = 1;
  setsockopt(fd.get(), SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  int sz = 4 << 20;
  setsockopt(fd.get(), SOL_SOCKET, SO_RCVBUF, &sz, sizeof(sz));
  sockaddr_in a = resolve(host, port);
  if (::bind(fd.get(), (sockaddr*)&a, sizeof(a)) != 0)
    throw NetError("udp bind " + host + ":" + std::to_string(port) + ": " + strerror(errno));
  return fd;
}

bool udp_send(int fd, const sockaddr_in& to, const std::string& data) {
  return ::sendto(fd, data.data(), data.size(), 0, (const sockaddr*)&to, sizeof(to)) ==
         (ssize_t)data.size();
}

int udp_recv(int fd, char* buf, size_t cap, int timeout_ms, sockaddr_in* from) {
  pollfd p{fd, POLLIN, 0};
  int r = ::poll(&p, 1, timeout_ms);
  if (r <= 0) return 0;
  socklen_t fl = sizeof(sockaddr_in);
  ssize_t n = ::recvfrom(fd, buf, cap, 0, (sockaddr*)from, &fl);
  return n < 0 ? 0 : (int)n;
}

Fd tcp_listen(const std::string& host, int port, int backlog) {
  Fd fd(::socket(AF_INET, SOCK_STREAM | SOCK_CLOEXEC, 0));
  if (!fd) throw NetError("socket(tcp) failed");
  int one = 1;
  setsockopt(fd.get(), SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  sockaddr_in a = resolve(host, port);
  if (::bind(fd.get(), (sockaddr*)&a, sizeof(a)) != 0)
    throw NetError("tcp bind " + host + ":" + std::to_string(port) + ": " + strerror(errno));
  if (::listen(fd.get(), backlog) != 0) throw NetError("listen failed");
  return fd;
}

Fd tcp_accept(int lfd, int timeout_ms) {
  pollfd p{lfd, POLLIN, 0};
  if (::poll(&p, 1, timeout_ms) <= 0) return Fd();
  int c = ::accept4(lfd, nullptr, nullptr, SOCK_CLOEXEC);
  if (c < 0) return Fd();
  int one = 1;
  setsockopt(c, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
  return Fd(c);
}

Fd tcp_connect(const std::string& host, int port, int timeout_ms) {
  sockaddr_in a = resolve(host, port);
  Fd fd(::socket(AF_INET, SOCK_STREAM | SOCK_CLOEXEC, 0));
  if (!fd) throw NetError("socket(tcp) failed");
  int fl = fcntl(fd.get(), F_GETFL, 0);
  fcntl(fd.get(), F_SETFL, fl | O_NONBLOCK);
  int r = ::connect(fd.get(), (sockaddr*)&a, sizeof(a));
  if (r != 0 && errno != EINPROGRESS)
    throw NetError("connect " + host + ":" + std::to_string(port) + ": " + strerror(errno));
  if (r != 0) {
    pollfd p{fd.get(), POLLOUT, 0};
    if (::poll(&p, 1, timeout_ms) <= 0) throw NetError("connect timeout " + host + ":" + std::to_string(port));
    int err = 0;
    socklen_t el = sizeof(err);
    getsockopt(fd.get(), SOL_SOCKET, SO_ERROR, &err, &el);
    if (err != 0) throw NetError("connect " + host + ":" + std::to_string(port) + ": " + strerror(err));
  }
  fcntl(fd.get(), F_SETFL, fl);
  int one = 1;
  setsockopt(fd.get(), IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
  return fd;
}

void set_timeouts(int fd, int timeout_ms) {
  timeval tv{timeout_ms / 1000, (timeout_ms % 1000) * 1000};
  setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv));
  setsockopt(fd, SOL_SOCKET, SO_SNDTIMEO, &tv, sizeof(tv));
}

void send_all(int fd, const void* p, size_t n) {
  const char* c = (const char*)p;
  while (n > 0) {
    ssize_t w = ::send(fd, c, n, MSG_NOSIGNAL);
    if (w < 0) {
      if (errno == EINTR) continue;
      throw NetError(std::string("send: ") + strerror(errno), errno == EAGAIN || errno == EWOULDBLOCK);
    }
    c += w;
    n -= (size_t)w;
  }
}

bool recv_all(int fd, void* p, size_t n) {
  char* c = (char*)p;
  size_t got = 0;
  while (got < n) {
    ssize_t r = ::recv(fd, c + got, n - got, 0);
    if (r == 0) {
      if (got == 0) return false;
      throw NetError("connection closed mid-message");
    }
    if (r < 0) {
      if (errno == EINTR) continue;
      throw NetError(std::string("recv: ") + strerror(errno), errno == EAGAIN || errno == EWOULDBLOCK);
    }
    got += (size_t)r;
  }
  return true;
}

}  // namespace ctl
}  // namespace dmlc
