#include "rpc.h"

#include <cerrno>

#include <cstring>

#include <chrono>

#include <poll.h>

#include <sys/socket.h>
#include <unistd.h>

#include "common.h"

namespace dmlc {
namespace ctl {

namespace {
constexpr uint32_t kMaxFrame = 128u << 20;  // > the 64 MiB fetch chunk; bounds what a peer can make us allocate

bool read_frame(int fd, std::string* out) {
  uint32_t len = 0;
  if (!recv_all(fd, &len, 4)) return false;
  if (len > kMaxFrame) throw NetError("frame too large");
  out->resize(len);
  if (len) recv_all(fd, &(*out)[0], len);
  return true;
}

void write_frame(int fd, const std::string& body) {
  uint32_t len = (uint32_t)body.size();
  std::string buf;
  buf.reserve(4 + body.size());
  buf.append((const char*)&len, 4);
  buf.append(body);
  send_all(fd, buf.data(), buf.size());
}
}  // namespace

RpcServer::RpcServer(std::string name, std::string host, int port, int max_conns)
    : name_(std::move(name)), host_(std::move(host)), port_(port), max_conns_(max_conns) {}

RpcServer::~RpcServer() { stop(); }

void RpcServer::handle(uint16_t method, RpcHandler h) { handlers_[method] = std::move(h); }

void RpcServer::start() {
  lfd_ = tcp_listen(host_, port_);
  acceptor_ = std::thread([this] { accept_loop(); });
}

void RpcServer::stop() {
  if (stop_.exchange(true)) return;
  if (acceptor_.joinable()) acceptor_.join();
  {
    std::lock_guard<std::mutex> g(conns_mu_);
    for (int fd : conn_fds_) ::shutdown(fd, SHUT_RDWR);
  }
  while (active_.load() > 0) std::this_thread::sleep_for(std::chrono::milliseconds(5));
  lfd_.reset();
}

void RpcServer::accept_loop() {
  while (!stop_.load()) {
    Fd c = tcp_accept(lfd_.get(), 200);
    if (!c) continue;
    if (active_.load() >= max_conns_) continue;  // over capacity: drop (client retries)
    int fd = c.release();
    {
      std::lock_guard<std::mutex> g(conns_mu_);
      conn_fds_.push_back(fd);
    }
    active_++;
    std::thread([this, fd] {
      serve_conn(fd);
      {
        std::lock_guard<std::mutex> g(conns_mu_);
        for (size_t i = 0; i < conn_fds_.size(); ++i)
          if (conn_fds_[i] == fd) {
            conn_fds_.erase(conn_fds_.begin() + i);
            break;
          }
      }
      ::close(fd);
      active_--;
    }).detach();
  }
}

void RpcServer::serve_conn(int fd) {
  std::string req;
  try {
    while (!stop_.load()) {
      if (!read_frame(fd, &req)) return;
      if (req.size() < 2) return;
      uint16_t method;
      memcpy(&method, req.data(), 2);
      Reader r(req.data() + 2, req.size() - 2);
      std::string resp;
      auto it = handlers_.find(method);
      if (it == handlers_.end()) {
        resp.push_back((char)2);
        resp += "unknown method " + std::to_string(method);
      } else {
        try {
          std::string body = it->second(r);
          resp.push_back((char)0);
          resp += body;
        } catch (const std::exception& e) {
          resp.clear();
          resp.push_back((char)1);
          resp += e.what();
          DMLC_LOG_WARN(name_ << ": handler " << method << " failed: " << e.what());
        }
      }
      write_frame(fd, resp);
    }
  } catch (const std::exception&) {
    // peer went away / timeout: close the connection
  }
}

RpcClient& RpcClient::shared() {
  static RpcClient c;
  return c;
}

std::string RpcClient::call(const std::string& host, int port, uint16_t method, const std::string& payload,
                            int timeout_ms, bool fresh, const std::function<bool()>& alive) {
  const std::string key = host + ":" + std::to_string(port);
  std::string body;
  body.append((const char*)&method, 2);
  body.append(payload);
  // Try a pooled connection first; a stale one (peer restarted) gets one retry
  // on a fresh connection.
  for (int attempt = 0; attempt < 2; ++attempt) {
    int fd = -1;
    bool pooled = false;
    if (attempt == 0 && !fresh) {
      std::lock_guard<std::mutex> g(mu_);
      auto& v = idle_[key];
      if (!v.empty()) {
        fd = v.back();
        v.pop_back();
        pooled = true;
      }
    }
    Fd conn;
    if (fd >= 0) {
      conn = Fd(fd);
    } else {
      conn = tcp_connect(host, port, std::min(timeout_ms, 3000));
    }
    set_timeouts(conn.get(), timeout_ms);
    std::string resp;
    try {
      write_frame(conn.get(), body);
      if (alive) {  // wait for the reply's first bytes in slices, asking the failure detector between them
        const auto t_end = std::chrono::steady_clock::now() + std::chrono::milliseconds(timeout_ms);
        for (;;) {
          pollfd p{conn.get(), POLLIN, 0};
          const int r = ::poll(&p, 1, 250);
          if (r > 0) break;
          if (r < 0 && errno != EINTR) throw NetError(std::string("poll: ") + strerror(errno));
          if (std::chrono::steady_clock::now() >= t_end) throw NetError("reply timed out", true);
          if (!alive()) throw NetError("peer declared failed while waiting for its reply", true);
        }
      }
      if (!read_frame(conn.get(), &resp)) throw NetError("connection closed");
    } catch (const NetError& e) {
      // a stale pooled socket (peer restarted: closed / reset) gets one retry
      // on a fresh connection; a deadline that passed does not (a hung peer
      // would otherwise cost the caller twice its timeout)
      if (pooled && !e.timed_out) continue;
      throw;
    }
    if (resp.empty()) throw RpcError("empty response");
    const uint8_t status = (uint8_t)resp[0];
    if (!fresh) {
      std::lock_guard<std::mutex> g(mu_);
      auto& v = idle_[key];
      if (v.size() < 16) v.push_back(conn.release());
    }
    if (status != 0) throw RpcError(resp.substr(1));
    return resp.substr(1);
  }
  throw RpcError("rpc to " + key + " failed");
}

void RpcClient::drop(const std::string& host, int port) {
  const std::string key = host + ":" + std::to_string(port);
  std::lock_guard<std::mutex> g(mu_);
  for (int fd : idle_[key]) ::close(fd);
  idle_[key].clear();
}

void RpcClient::clear() {
  std::lock_guard<std::mutex> g(mu_);
  for (auto& kv : idle_)
    for (int fd : kv.second) ::close(fd);
  idle_.clear();
}

}  // namespace ctl
}  // namespace dmlc
