// Length-prefixed binary RPC over TCP with pooled client connections.
//
// Reference: tarpc over TCP with a JSON codec, one new TCP connection per
// client call (LeaderClient::spawn / MemberClient::spawn,
// src/services.rs:436-441,583-588), 1 in-flight request per channel and 10
// channels served concurrently (src/main.rs:43-83). Here:
//   request  = u32 len | u16 method | payload
//   response = u32 len | u8 status (0 ok, 1 error, 2 unknown method) | payload
// Connections are kept open and reused by the client pool (one request at a
// time per connection); the server runs one handler thread per connection
// up to `max_conns`.
#pragma once
#include <atomic>
#include <functional>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "net.h"
#include "wire.h"

namespace dmlc {
namespace ctl {

struct RpcError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

using RpcHandler = std::function<std::string(Reader&)>;

class RpcServer {
 public:
  RpcServer(std::string name, std::string host, int port, int max_conns = 64);
  ~RpcServer();
  void handle(uint16_t method, RpcHandler h);
  void start();
  void stop();
  int port() const { return port_; }

 private:
  void accept_loop();
  void serve_conn(int fd);

  std::string name_, host_;
  int port_;
  int max_conns_;
  Fd lfd_;
  std::map<uint16_t, RpcHandler> handlers_;
  std::atomic<bool> stop_{false};
  std::atomic<int> active_{0};
  std::thread acceptor_;
  std::mutex conns_mu_;
  std::vector<int> conn_fds_;
};

class RpcClient {
 public:
  static RpcClient& shared();
  // Synchronous call; throws RpcError / NetError. timeout covers the whole call.
  // fresh: a new TCP connection for this call, closed after it (the
  // reference's per-query connect, src/services.rs:420,583-588; the default
  // reuses pooled connections).
  // alive (optional): polled every 250 ms while the reply has not started
  // arriving; the call gives up (NetError, timed_out) as soon as it returns
  // false: the caller's failure detector has declared the peer dead, so a
  // hung peer costs the call that long instead of its whole timeout.
  std::string call(const std::string& host, int port, uint16_t method, const std::string& payload,
                   int timeout_ms = 10000, bool fresh = false, const std::function<bool()>& alive = nullptr);
  void drop(const std::string& host, int port);  // close pooled connections
  void clear();

 private:
  std::mutex mu_;
  std::unordered_map<std::string, std::vector<int>> idle_;
};

}  // namespace ctl
}  // namespace dmlc
