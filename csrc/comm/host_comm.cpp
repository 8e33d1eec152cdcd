// In-process fake communicator (host memory): the data-parallel coordinator's
// shard / gather / rank-loss logic and the serving fleet's partition logic
// run on it in CPU tests. It models what RCCL point-to-point does, not what
// is convenient:
//   * rendezvous: a send completes only when the matching receive has been
//     posted (the bytes are copied straight from the sender's buffer into the
//     receiver's); nothing is buffered, so an issue order that would leave
//     two RCCL ranks each waiting on the other (rank 0 sends to 1 while 1
//     sends to 0, each before receiving) times out here too instead of
//     passing;
//   * FIFO per (src, dst) pair and communicator: the k-th send a -> b meets
//     the k-th receive at b from a, whichever threads post them, and the sizes
//     must agree;
//   * groups: every operation posted between a thread's outermost
//     group_start and group_end is posted at once when the group ends, and
//     group_end returns when all of them have completed (the host stand-in
//     for "the stream reached the end of the group's kernel"). One thread may
//     drive several ranks inside one group, and a rank may send and receive
//     in the same group;
//   * a lost peer (host_kill) or an abort fails every pending and later
//     operation that involves it with CommError; a timed-out group withdraws
//     its still-unmatched operations before it throws, so no later match
//     touches a buffer the caller has given up on.
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <map>
#include <mutex>

#include "comm.h"
#include "cv_wait.h"

namespace dmlc {
namespace comm {

namespace {
// One posted operation; owned by the group_end call that posted it (its
// stack frame outlives the op's presence in the world's queues).
struct Op {
  bool is_send = false;
  int self = 0, peer = 0;
  const void* sbuf = nullptr;
  void* rbuf = nullptr;
  size_t bytes = 0;
  Stream stream = nullptr;  // the rank's stream (data planes that order by stream)
  void* mark = nullptr;     // the data plane's token for the stream position at post
  bool done = false;
  std::string error;  // set with done = true on failure
};

// host memory: the bytes move at match time
class HostPlane : public FakeDataPlane {
 public:
  std::string name() const override { return "host"; }
  void* mark(Stream) override { return nullptr; }
  void move(const void* sbuf, void* rbuf, size_t bytes, void*, Stream, void*, Stream) override {
    if (bytes) std::memcpy(rbuf, sbuf, bytes);
  }
  void local_copy(void* dst, const void* src, size_t bytes, Stream) override {
    if (bytes && dst != src) std::memcpy(dst, src, bytes);
  }
  void release(void*) override {}
};
}  // namespace

class HostWorld {
 public:
  HostWorld(int n, int timeout_ms, std::shared_ptr<FakeDataPlane> dp)
      : n_(n), timeout_ms_(timeout_ms), dead_(n, false), dp_(std::move(dp)) {}
  FakeDataPlane& plane() { return *dp_; }

  // Post every op (matching what it can), then wait for all of them.
  // Throws CommError on failure or timeout (after withdrawing unmatched ops).
  void run(std::vector<Op*>& ops) {
    post_ops(ops);
    wait_ops(ops);
  }
  // The two halves of run(): a group spanning several worlds posts into all
  // of them before it waits on any (as an RCCL group spanning communicators).
  void post_ops(std::vector<Op*>& ops) {
    std::lock_guard<std::mutex> g(mu_);
    for (Op* o : ops) post(o);
  }
  void wait_ops(std::vector<Op*>& ops) {
    std::unique_lock<std::mutex> g(mu_);
    const auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(timeout_ms_);
    for (;;) {
      bool all = true;
      for (Op* o : ops) all &= o->done;
      if (all) break;
      if (cv_wait_until(cv_, g, deadline) == std::cv_status::timeout) {
        bool all2 = true;
        for (Op* o : ops) all2 &= o->done;
        if (all2) break;
        for (Op* o : ops)
          if (!o->done) {
            withdraw(o);
            o->done = true;
            o->error = std::string("host comm: ") + (o->is_send ? "send to " : "recv from ") +
                       std::to_string(o->peer) + " timed out (no matching " + (o->is_send ? "recv" : "send") +
                       " posted)";
          }
        break;
      }
    }
    for (Op* o : ops)
      if (!o->error.empty()) throw CommError(o->error);
  }

  void kill(int r) {
    std::lock_guard<std::mutex> g(mu_);
    dead_.at(r) = true;
    fail_where([&](const Op* o) { return o->self == r || o->peer == r; },
               "host comm: rank " + std::to_string(r) + " is lost");
    cv_.notify_all();
  }
  void abort_all() {
    std::lock_guard<std::mutex> g(mu_);
    aborted_ = true;
    fail_where([](const Op*) { return true; }, "host comm: communicator aborted");
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
  // operations posted but not matched yet (tests: nothing may be left over)
  size_t pending() {
    std::lock_guard<std::mutex> g(mu_);
    size_t k = 0;
    for (auto& kv : sends_) k += kv.second.size();
    for (auto& kv : recvs_) k += kv.second.size();
    return k;
  }

 private:
  using Key = std::pair<int, int>;  // (src, dst)
  void post(Op* o) {
    o->mark = dp_->mark(o->stream);
    if (aborted_) return fail(o, "host comm: communicator aborted");
    if (dead_[o->self] || dead_[o->peer])
      return fail(o, "host comm: rank " + std::to_string(dead_[o->self] ? o->self : o->peer) + " is lost");
    const Key k = o->is_send ? Key{o->self, o->peer} : Key{o->peer, o->self};
    auto& mine = o->is_send ? sends_[k] : recvs_[k];
    auto& theirs = o->is_send ? recvs_[k] : sends_[k];
    if (!theirs.empty() && mine.empty()) {
      Op* other = theirs.front();
      theirs.pop_front();
      Op* s = o->is_send ? o : other;
      Op* r = o->is_send ? other : o;
      if (s->bytes != r->bytes) {
        const std::string e = "host comm: size mismatch " + std::to_string(s->bytes) + " vs " +
                              std::to_string(r->bytes) + " from rank " + std::to_string(s->self) + " to " +
                              std::to_string(r->self);
        fail(s, e);
        fail(r, e);
        return;
      }
      dp_->move(s->sbuf, r->rbuf, s->bytes, s->mark, s->stream, r->mark, r->stream);
      dp_->release(s->mark);
      dp_->release(r->mark);
      s->mark = r->mark = nullptr;
      s->done = r->done = true;
      cv_.notify_all();
      return;
    }
    mine.push_back(o);
  }
  void fail(Op* o, const std::string& e) {
    dp_->release(o->mark);
    o->mark = nullptr;
    o->done = true;
    o->error = e;
    cv_.notify_all();
  }
  void withdraw(Op* o) {
    for (auto* m : {&sends_, &recvs_})
      for (auto& kv : *m) {
        auto& q = kv.second;
        for (auto it = q.begin(); it != q.end(); ++it)
          if (*it == o) {
            q.erase(it);
            dp_->release(o->mark);
            o->mark = nullptr;
            return;
          }
      }
  }
  template <class Pred>
  void fail_where(Pred p, const std::string& e) {
    for (auto* m : {&sends_, &recvs_})
      for (auto& kv : *m) {
        auto& q = kv.second;
        for (auto it = q.begin(); it != q.end();) {
          if (p(*it)) {
            fail(*it, e);
            it = q.erase(it);
          } else {
            ++it;
          }
        }
      }
  }

  int n_, timeout_ms_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::map<Key, std::deque<Op*>> sends_, recvs_;  // posted, unmatched, FIFO per pair
  std::vector<bool> dead_;
  bool aborted_ = false;
  std::shared_ptr<FakeDataPlane> dp_;
};

namespace {

struct Pending {
  HostWorld* world;
  Op op;
};

// Thread-wide group state, like RCCL's.
thread_local int t_depth = 0;
thread_local std::vector<Pending> t_ops;

void run_ops(std::vector<Pending>& ops) {
  // one HostWorld::run per world, all posted before any waits: a group may
  // span several communicators (RCCL groups do), so post everything first.
  std::map<HostWorld*, std::vector<Op*>> by_world;
  for (auto& p : ops) by_world[p.world].push_back(&p.op);
  if (by_world.empty()) return;
  if (by_world.size() == 1) {
    by_world.begin()->first->run(by_world.begin()->second);
    return;
  }
  // several worlds: post into every one before waiting on any (waiting world
  // by world after posting all cannot deadlock: a peer's matching group has
  // posted its side of every world too); the first error is rethrown once
  // every world's ops are done or withdrawn
  for (auto& kv : by_world) kv.first->post_ops(kv.second);
  std::exception_ptr err;
  for (auto& kv : by_world) {
    try {
      kv.first->wait_ops(kv.second);
    } catch (...) {
      if (!err) err = std::current_exception();
    }
  }
  if (err) std::rethrow_exception(err);
}

class HostComm : public Comm {
 public:
  HostComm(std::shared_ptr<HostWorld> w, int rank) : w_(std::move(w)), rank_(rank) {}
  int rank() const override { return rank_; }
  int size() const override { return w_->size(); }
  std::string backend() const override { return w_->plane().name(); }

  void group_start() override { ++t_depth; }
  void group_end() override {
    if (t_depth <= 0) throw std::logic_error("host comm: group_end without group_start");
    if (--t_depth > 0) return;
    std::vector<Pending> ops;
    ops.swap(t_ops);
    run_ops(ops);
  }
  void send(const void* buf, size_t bytes, int peer, Stream s) override {
    Op o;
    o.is_send = true;
    o.self = rank_;
    o.peer = check_peer(peer);
    o.sbuf = buf;
    o.bytes = bytes;
    o.stream = s;
    post(o);
  }
  void recv(void* buf, size_t bytes, int peer, Stream s) override {
    Op o;
    o.self = rank_;
    o.peer = check_peer(peer);
    o.rbuf = buf;
    o.bytes = bytes;
    o.stream = s;
    post(o);
  }
  void broadcast(const void* sendbuf, void* recvbuf, size_t bytes, int root, Stream s) override {
    group_start();
    if (rank_ == root) {
      for (int r = 0; r < size(); ++r)
        if (r != root) send(sendbuf, bytes, r, s);
      w_->plane().local_copy(recvbuf, sendbuf, bytes, s);
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
  void post(const Op& op) {
    if (t_depth > 0) {
      t_ops.push_back({w_.get(), op});
    } else {
      std::vector<Pending> one{{w_.get(), op}};
      run_ops(one);
    }
  }
  std::shared_ptr<HostWorld> w_;
  int rank_;
};

}  // namespace

std::vector<std::unique_ptr<Comm>> fake_world(int n, int timeout_ms, std::shared_ptr<FakeDataPlane> dp) {
  if (n < 1) throw std::invalid_argument("fake_world: n must be >= 1");
  if (!dp) throw std::invalid_argument("fake_world: no data plane");
  auto w = std::make_shared<HostWorld>(n, timeout_ms, std::move(dp));
  std::vector<std::unique_ptr<Comm>> out;
  for (int r = 0; r < n; ++r) out.push_back(std::make_unique<HostComm>(w, r));
  return out;
}

std::vector<std::unique_ptr<Comm>> host_world(int n, int timeout_ms) {
  return fake_world(n, timeout_ms, std::make_shared<HostPlane>());
}

void host_kill(Comm& c, int rank) {
  auto* h = dynamic_cast<HostComm*>(&c);
  if (!h) throw std::invalid_argument("host_kill: not a host communicator");
  h->world()->kill(rank);
}

size_t host_pending(Comm& c) {
  auto* h = dynamic_cast<HostComm*>(&c);
  if (!h) throw std::invalid_argument("host_pending: not a host communicator");
  return h->world()->pending();
}

}  // namespace comm
}  // namespace dmlc
