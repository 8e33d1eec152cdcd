// In-process fake communicator (host memory): the data-parallel coordinator's
// shard / gather / rank-loss logic runs on it in CPU tests. Semantics match
// what the coordinator relies on from RCCL:
//   * point-to-point messages between a (src, dst) pair are delivered in the
//     order they were posted;
//   * a group posts all of its sends before it blocks on any receive, so one
//     thread may drive several ranks inside one group, and a rank may send
//     and receive in the same group without deadlock;
//   * a receive from a lost peer (host_kill) fails with CommError.
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <map>
#include <mutex>

#include "comm.h"

namespace dmlc {
namespace comm {

class HostWorld {
 public:
  HostWorld(int n, int timeout_ms) : n_(n), timeout_ms_(timeout_ms), dead_(n, false) {}

  void put(int src, int dst, const void* buf, size_t bytes) {
    std::lock_guard<std::mutex> g(mu_);
    if (aborted_ || dead_[src]) throw CommError("host comm: rank " + std::to_string(src) + " is lost");
    auto& q = box_[{src, dst}];
    q.emplace_back((const uint8_t*)buf, (const uint8_t*)buf + bytes);
    cv_.notify_all();
  }

  void take(int src, int dst, void* buf, size_t bytes) {
    std::unique_lock<std::mutex> g(mu_);
    auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(timeout_ms_);
    for (;;) {
      if (aborted_ || dead_[dst]) throw CommError("host comm: rank " + std::to_string(dst) + " is lost");
      auto it = box_.find({src, dst});
      if (it != box_.end() && !it->second.empty()) {
        auto& m = it->second.front();
        if (m.size() != bytes)
          throw CommError("host comm: size mismatch " + std::to_string(m.size()) + " vs " + std::to_string(bytes) +
                          " from rank " + std::to_string(src));
        if (bytes) std::memcpy(buf, m.data(), bytes);
        it->second.pop_front();
        return;
      }
      if (dead_[src]) throw CommError("host comm: peer " + std::to_string(src) + " is lost");
      if (cv_.wait_until(g, deadline) == std::cv_status::timeout)
        throw CommError("host comm: recv from " + std::to_string(src) + " timed out");
    }
  }

  void kill(int r) {
    std::lock_guard<std::mutex> g(mu_);
    dead_.at(r) = true;
    cv_.notify_all();
  }
  void abort_all() {
    std::lock_guard<std::mutex> g(mu_);
    aborted_ = true;
    cv_.notify_all();
  }
  bool healthy(int r) {
    std::lock_guard<std::mutex> g(mu_);
    if (aborted_ || dead_[r]) return false;
    for (bool d : dead_)
      if (d) return false;  // a lost peer breaks the whole communicator (as in RCCL)
    return true;
  }
  int size() const { return n_; }

 private:
  int n_, timeout_ms_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::map<std::pair<int, int>, std::deque<std::vector<uint8_t>>> box_;
  std::vector<bool> dead_;
  bool aborted_ = false;
};

namespace {

struct PendingOp {
  HostWorld* world;
  bool is_send;
  int self, peer;
  const void* sbuf;
  void* rbuf;
  size_t bytes;
};

// Thread-wide group state, like RCCL's.
thread_local int t_depth = 0;
thread_local std::vector<PendingOp> t_ops;

void run_ops(std::vector<PendingOp>& ops) {
  for (auto& o : ops)
    if (o.is_send) o.world->put(o.self, o.peer, o.sbuf, o.bytes);
  for (auto& o : ops)
    if (!o.is_send) o.world->take(o.peer, o.self, o.rbuf, o.bytes);
}

class HostComm : public Comm {
 public:
  HostComm(std::shared_ptr<HostWorld> w, int rank) : w_(std::move(w)), rank_(rank) {}
  int rank() const override { return rank_; }
  int size() const override { return w_->size(); }
  std::string backend() const override { return "host"; }

  void group_start() override { ++t_depth; }
  void group_end() override {
    if (t_depth <= 0) throw std::logic_error("host comm: group_end without group_start");
    if (--t_depth > 0) return;
    std::vector<PendingOp> ops;
    ops.swap(t_ops);
    run_ops(ops);
  }
  void send(const void* buf, size_t bytes, int peer, Stream) override {
    post({w_.get(), true, rank_, check_peer(peer), buf, nullptr, bytes});
  }
  void recv(void* buf, size_t bytes, int peer, Stream) override {
    post({w_.get(), false, rank_, check_peer(peer), nullptr, buf, bytes});
  }
  void broadcast(const void* sendbuf, void* recvbuf, size_t bytes, int root, Stream s) override {
    group_start();
    if (rank_ == root) {
      for (int r = 0; r < size(); ++r)
        if (r != root) send(sendbuf, bytes, r, s);
      if (recvbuf != sendbuf && bytes) std::memcpy(recvbuf, sendbuf, bytes);
    } else {
      recv(recvbuf, bytes, root, s);
    }
    group_end();
  }
  bool ok() override { return w_->healthy(rank_); }
  void abort() override { w_->abort_all(); }

  HostWorld* world() { return w_.get(); }

 private:
  int check_peer(int p) const {
    if (p < 0 || p >= size() || p == rank_) throw std::invalid_argument("host comm: bad peer " + std::to_string(p));
    return p;
  }
  void post(PendingOp op) {
    if (t_depth > 0) {
      t_ops.push_back(op);
    } else {
      std::vector<PendingOp> one{op};
      run_ops(one);
    }
  }
  std::shared_ptr<HostWorld> w_;
  int rank_;
};

}  // namespace

std::vector<std::unique_ptr<Comm>> host_world(int n, int timeout_ms) {
  if (n < 1) throw std::invalid_argument("host_world: n must be >= 1");
  auto w = std::make_shared<HostWorld>(n, timeout_ms);
  std::vector<std::unique_ptr<Comm>> out;
  for (int r = 0; r < n; ++r) out.push_back(std::make_unique<HostComm>(w, r));
  return out;
}

void host_kill(Comm& c, int rank) {
  auto* h = dynamic_cast<HostComm*>(&c);
  if (!h) throw std::invalid_argument("host_kill: not a host communicator");
  h->world()->kill(rank);
}

}  // namespace comm
}  // namespace dmlc
