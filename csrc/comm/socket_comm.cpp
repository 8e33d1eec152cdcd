// Cross-process host communicator over TCP (loopback): the multi-process
// bench path on CPU (bench.py --dry-run, tests/test_bench_dryrun_cpu.py).
//
// RCCL's process-per-GPU model is one communicator rank per process,
// bootstrapped from a unique id that rank 0 creates and hands out over a side
// channel (bench.py: the gloo store). This communicator keeps that shape —
// socket_unique_id() is rank 0's bootstrap address, socket_init_rank() builds
// a full mesh of TCP connections — and the point-to-point semantics of the
// in-process host fake (host_comm.cpp):
//   * rendezvous: a receive announces itself to its peer (RTR, with its size)
//     and a send moves its bytes only once the peer's matching RTR has
//     arrived, so a send never completes before its receive is posted and an
//     issue order that would deadlock RCCL (both ranks send first) times out
//     here too;
//   * FIFO per (src, dst): the k-th send a -> b meets the k-th receive at b
//     from a (one TCP connection per pair keeps the order), sizes must agree;
//   * groups: thread-wide and nestable; every operation of the outermost
//     group (on any socket communicator) is posted at group_end, which returns
//     when all have completed;
//   * a closed peer connection (a process that died) or an abort fails every
//     pending and later operation with CommError.
// One progress thread per communicator owns all its socket I/O (poll over the
// peer connections and a wake-up pipe), so several threads may post.
#include <cerrno>
#include <arpa/inet.h>
#include <fcntl.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <map>
#include <mutex>
#include <random>
#include <sstream>
#include <thread>

#include "comm.h"
#include "cv_wait.h"

namespace dmlc {
namespace comm {

namespace {

using Clock = std::chrono::steady_clock;

[[noreturn]] void sys_fail(const std::string& what) { throw CommError("socket comm: " + what + ": " + std::strerror(errno)); }

void set_nodelay(int fd) {
  int one = 1;
  setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
}

int listen_any(int* port) {
  const int fd = socket(AF_INET, SOCK_STREAM | SOCK_CLOEXEC, 0);
  if (fd < 0) sys_fail("socket");
  int one = 1;
  setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
  a.sin_port = htons((uint16_t)*port);
  if (bind(fd, (sockaddr*)&a, sizeof(a)) != 0) {
    close(fd);
    sys_fail("bind port " + std::to_string(*port));
  }
  if (listen(fd, 64) != 0) {
    close(fd);
    sys_fail("listen");
  }
  socklen_t len = sizeof(a);
  getsockname(fd, (sockaddr*)&a, &len);
  *port = ntohs(a.sin_port);
  return fd;
}

int connect_retry(const std::string& host, int port, Clock::time_point deadline) {
  for (;;) {
    const int fd = socket(AF_INET, SOCK_STREAM | SOCK_CLOEXEC, 0);
    if (fd < 0) sys_fail("socket");
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_port = htons((uint16_t)port);
    inet_pton(AF_INET, host.c_str(), &a.sin_addr);
    if (connect(fd, (sockaddr*)&a, sizeof(a)) == 0) {
      set_nodelay(fd);
      return fd;
    }
    close(fd);
    if (Clock::now() > deadline) sys_fail("connect " + host + ":" + std::to_string(port));
    std::this_thread::sleep_for(std::chrono::milliseconds(20));
  }
}

int accept_until(int lfd, Clock::time_point deadline) {
  for (;;) {
    pollfd p{lfd, POLLIN, 0};
    const int ms = (int)std::max<int64_t>(
        0, std::chrono::duration_cast<std::chrono::milliseconds>(deadline - Clock::now()).count());
    const int r = poll(&p, 1, std::min(ms, 200));
    if (r > 0) {
      const int fd = accept4(lfd, nullptr, nullptr, SOCK_CLOEXEC);
      if (fd < 0 && (errno == EINTR || errno == ECONNABORTED)) continue;
      if (fd < 0) sys_fail("accept");
      set_nodelay(fd);
      return fd;
    }
    if (Clock::now() > deadline) throw CommError("socket comm: bootstrap timed out waiting for peers");
  }
}

// blocking helpers (bootstrap only)
void write_all(int fd, const void* p, size_t n) {
  const char* c = (const char*)p;
  while (n) {
    const ssize_t k = ::send(fd, c, n, MSG_NOSIGNAL);
    if (k < 0 && errno == EINTR) continue;
    if (k <= 0) sys_fail("bootstrap send");
    c += k;
    n -= (size_t)k;
  }
}
void read_all(int fd, void* p, size_t n) {
  char* c = (char*)p;
  while (n) {
    const ssize_t k = ::recv(fd, c, n, 0);
    if (k < 0 && errno == EINTR) continue;
    if (k <= 0) throw CommError("socket comm: bootstrap peer closed");
    c += k;
    n -= (size_t)k;
  }
}

// One posted operation; owned by the group_end frame that posted it.
struct SOp {
  bool is_send = false;
  int peer = 0;
  const void* sbuf = nullptr;
  void* rbuf = nullptr;
  uint64_t bytes = 0;
  bool done = false;
  std::string error;
};

// wire: 16-byte header {u64 kind (1 = RTR, 2 = DATA), u64 bytes}, DATA followed by the payload
constexpr uint64_t kRtr = 1, kData = 2;

class SocketWorld {
 public:
  SocketWorld(int n, int rank, std::vector<int> fds, int timeout_ms)
      : n_(n), rank_(rank), timeout_ms_(timeout_ms), peers_(n) {
    for (int p = 0; p < n_; ++p) {
      peers_[p].fd = fds[p];
      if (fds[p] >= 0) fcntl(fds[p], F_SETFL, fcntl(fds[p], F_GETFL) | O_NONBLOCK);
    }
    if (pipe2(wake_, O_CLOEXEC | O_NONBLOCK) != 0) sys_fail("pipe");
    thr_ = std::thread([this] { loop(); });
  }
  ~SocketWorld() {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
    }
    wake();
    thr_.join();
    for (auto& p : peers_)
      if (p.fd >= 0) close(p.fd);
    close(wake_[0]);
    close(wake_[1]);
  }
  int size() const { return n_; }
  int rank() const { return rank_; }

  void post_ops(std::vector<SOp*>& ops) {
    {
      std::lock_guard<std::mutex> g(mu_);
      for (SOp* o : ops) post(o);
    }
    wake();
  }
  void wait_ops(std::vector<SOp*>& ops) {
    std::unique_lock<std::mutex> g(mu_);
    const auto deadline = Clock::now() + std::chrono::milliseconds(timeout_ms_);
    for (;;) {
      bool all = true;
      for (SOp* o : ops) all &= o->done;
      if (all) break;
      if (cv_wait_until(cv_, g, deadline) == std::cv_status::timeout) {
        bool all2 = true;
        for (SOp* o : ops) all2 &= o->done;
        if (all2) break;
        // an RTR already on the wire cannot be recalled: the communicator is
        // broken from here on (as an RCCL communicator after a hang)
        fail_all_locked("socket comm: rank " + std::to_string(rank_) + " timed out (no matching operation posted)");
        break;
      }
    }
    for (SOp* o : ops)
      if (!o->error.empty()) throw CommError(o->error);
  }
  bool healthy() {
    std::lock_guard<std::mutex> g(mu_);
    return broken_.empty();
  }
  void abort() {
    {
      std::lock_guard<std::mutex> g(mu_);
      fail_all_locked("socket comm: communicator aborted");
      for (auto& p : peers_)
        if (p.fd >= 0) shutdown(p.fd, SHUT_RDWR);
    }
    wake();
  }

 private:
  struct Out {
    uint64_t hdr[2];
    size_t hdr_done = 0;
    SOp* data = nullptr;  // DATA: the send whose payload follows
    size_t body_done = 0;
  };
  struct Peer {
    int fd = -1;
    std::deque<SOp*> sends;      // posted sends waiting for the peer's RTR
    std::deque<uint64_t> rtrs;   // RTRs from the peer not matched by a send yet
    std::deque<SOp*> recvs;      // posted recvs (RTR sent), in order
    std::deque<Out> outq;        // messages to write
    uint64_t in_hdr[2] = {0, 0};
    size_t in_hdr_done = 0;
    SOp* in_data = nullptr;      // DATA payload being read into this recv
    size_t in_body_done = 0;
    uint64_t in_skip = 0;        // payload bytes of a failed recv to discard
  };

  void wake() {
    const char c = 1;
    (void)!write(wake_[1], &c, 1);
  }
  void finish(SOp* o, const std::string& err) {
    o->done = true;
    o->error = err;
    cv_.notify_all();
  }
  void fail_all_locked(const std::string& e) {
    if (broken_.empty()) broken_ = e;
    for (auto& p : peers_) {
      for (SOp* o : p.sends) finish(o, e);
      for (SOp* o : p.recvs) finish(o, e);
      p.sends.clear();
      p.recvs.clear();
      for (auto& m : p.outq)
        if (m.data && !m.data->done) finish(m.data, e);
      p.outq.clear();
      if (p.in_data && !p.in_data->done) finish(p.in_data, e);
      p.in_data = nullptr;
    }
  }
  void post(SOp* o) {
    if (!broken_.empty()) return finish(o, broken_);
    Peer& p = peers_.at(o->peer);
    if (o->is_send) {
      if (!p.rtrs.empty()) {
        const uint64_t want = p.rtrs.front();
        p.rtrs.pop_front();
        start_data(p, o, want);
      } else {
        p.sends.push_back(o);
      }
    } else {
      p.recvs.push_back(o);
      Out m;
      m.hdr[0] = kRtr;
      m.hdr[1] = o->bytes;
      p.outq.push_back(m);
    }
  }
  void start_data(Peer& p, SOp* s, uint64_t want) {
    if (want != s->bytes) {
      const std::string e = "socket comm: size mismatch " + std::to_string(s->bytes) + " vs " + std::to_string(want) +
                            " from rank " + std::to_string(rank_) + " to " + std::to_string(s->peer);
      fail_all_locked(e);
      return;
    }
    Out m;
    m.hdr[0] = kData;
    m.hdr[1] = s->bytes;
    m.data = s;
    p.outq.push_back(m);
  }

  // progress: returns false when the connection failed
  bool pump_out(Peer& p) {
    while (!p.outq.empty()) {
      Out& m = p.outq.front();
      if (m.hdr_done < sizeof(m.hdr)) {
        const ssize_t k = ::send(p.fd, (const char*)m.hdr + m.hdr_done, sizeof(m.hdr) - m.hdr_done, MSG_NOSIGNAL);
        if (k < 0) return errno == EAGAIN || errno == EWOULDBLOCK || errno == EINTR;
        m.hdr_done += (size_t)k;
        if (m.hdr_done < sizeof(m.hdr)) return true;
      }
      if (m.data) {
        const uint64_t n = m.data->bytes;
        while (m.body_done < n) {
          const ssize_t k = ::send(p.fd, (const char*)m.data->sbuf + m.body_done, n - m.body_done, MSG_NOSIGNAL);
          if (k < 0) return errno == EAGAIN || errno == EWOULDBLOCK || errno == EINTR;
          m.body_done += (size_t)k;
        }
        finish(m.data, "");
      }
      p.outq.pop_front();
    }
    return true;
  }
  bool pump_in(int peer) {
    Peer& p = peers_[peer];
    for (;;) {
      if (p.in_data || p.in_skip) {
        const uint64_t n = p.in_data ? p.in_data->bytes : p.in_skip;
        char sink[4096];
        while (p.in_body_done < n) {
          char* dst = p.in_data ? (char*)p.in_data->rbuf + p.in_body_done : sink;
          const size_t want = p.in_data ? n - p.in_body_done : std::min<uint64_t>(sizeof(sink), n - p.in_body_done);
          const ssize_t k = ::recv(p.fd, dst, want, 0);
          if (k == 0) return false;
          if (k < 0) return errno == EAGAIN || errno == EWOULDBLOCK || errno == EINTR;
          p.in_body_done += (size_t)k;
        }
        if (p.in_data) finish(p.in_data, "");
        p.in_data = nullptr;
        p.in_skip = 0;
        p.in_body_done = 0;
      }
      const ssize_t k = ::recv(p.fd, (char*)p.in_hdr + p.in_hdr_done, sizeof(p.in_hdr) - p.in_hdr_done, 0);
      if (k == 0) return false;
      if (k < 0) return errno == EAGAIN || errno == EWOULDBLOCK || errno == EINTR;
      p.in_hdr_done += (size_t)k;
      if (p.in_hdr_done < sizeof(p.in_hdr)) continue;
      p.in_hdr_done = 0;
      if (p.in_hdr[0] == kRtr) {
        if (!p.sends.empty()) {
          SOp* s = p.sends.front();
          p.sends.pop_front();
          start_data(p, s, p.in_hdr[1]);
        } else {
          p.rtrs.push_back(p.in_hdr[1]);
        }
      } else if (p.in_hdr[0] == kData) {
        // DATA only follows our RTR: the oldest posted recv from this peer
        if (p.recvs.empty()) {
          if (broken_.empty()) fail_all_locked("socket comm: unexpected DATA from rank " + std::to_string(peer));
          p.in_skip = p.in_hdr[1];
          continue;
        }
        SOp* r = p.recvs.front();
        p.recvs.pop_front();
        if (r->bytes != p.in_hdr[1]) {
          fail_all_locked("socket comm: size mismatch " + std::to_string(p.in_hdr[1]) + " vs " +
                          std::to_string(r->bytes) + " from rank " + std::to_string(peer) + " to " +
                          std::to_string(rank_));
          p.in_skip = p.in_hdr[1];
          continue;
        }
        p.in_data = r;
        if (r->bytes == 0) {
          finish(r, "");
          p.in_data = nullptr;
        }
      } else {
        return false;
      }
    }
  }
  void loop() {
    std::vector<pollfd> fds;
    std::vector<int> who;
    for (;;) {
      fds.clear();
      who.clear();
      {
        std::lock_guard<std::mutex> g(mu_);
        if (stop_) return;
        for (int p = 0; p < n_; ++p) {
          if (peers_[p].fd < 0 || peers_[p].fd == -2) continue;
          short ev = POLLIN;
          if (!peers_[p].outq.empty()) ev |= POLLOUT;
          fds.push_back({peers_[p].fd, ev, 0});
          who.push_back(p);
        }
      }
      fds.push_back({wake_[0], POLLIN, 0});
      poll(fds.data(), fds.size(), 100);
      if (fds.back().revents & POLLIN) {
        char buf[64];
        while (read(wake_[0], buf, sizeof(buf)) > 0) {
        }
      }
      std::lock_guard<std::mutex> g(mu_);
      if (stop_) return;
      for (size_t i = 0; i + 1 < fds.size(); ++i) {
        Peer& p = peers_[who[i]];
        bool ok = true;
        if (fds[i].revents & (POLLIN | POLLHUP | POLLERR)) ok = pump_in(who[i]);
        if (ok && !p.outq.empty()) ok = pump_out(p);
        if (!ok) {
          fail_all_locked("socket comm: rank " + std::to_string(who[i]) + " is lost (connection closed)");
          close(p.fd);
          p.fd = -2;
        }
      }
    }
  }

  int n_, rank_, timeout_ms_;
  std::vector<Peer> peers_;
  int wake_[2] = {-1, -1};
  std::mutex mu_;
  std::condition_variable cv_;
  std::string broken_;
  bool stop_ = false;
  std::thread thr_;
};

// Thread-wide group state (RCCL's groups are per thread, across communicators).
struct SPending {
  SocketWorld* world;
  SOp op;
};
thread_local int t_depth = 0;
thread_local std::vector<SPending> t_ops;

void run_sops(std::vector<SPending>& ops) {
  std::map<SocketWorld*, std::vector<SOp*>> by_world;
  for (auto& p : ops) by_world[p.world].push_back(&p.op);
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

class SocketComm : public Comm {
 public:
  explicit SocketComm(std::unique_ptr<SocketWorld> w) : w_(std::move(w)) {}
  int rank() const override { return w_->rank(); }
  int size() const override { return w_->size(); }
  std::string backend() const override { return "socket"; }
  void group_start() override { ++t_depth; }
  void group_end() override {
    if (t_depth <= 0) throw std::logic_error("socket comm: group_end without group_start");
    if (--t_depth > 0) return;
    std::vector<SPending> ops;
    ops.swap(t_ops);
    run_sops(ops);
  }
  void send(const void* buf, size_t bytes, int peer, Stream) override {
    SOp o;
    o.is_send = true;
    o.peer = check_peer(peer);
    o.sbuf = buf;
    o.bytes = bytes;
    post(o);
  }
  void recv(void* buf, size_t bytes, int peer, Stream) override {
    SOp o;
    o.peer = check_peer(peer);
    o.rbuf = buf;
    o.bytes = bytes;
    post(o);
  }
  void broadcast(const void* sendbuf, void* recvbuf, size_t bytes, int root, Stream s) override {
    group_start();
    try {
      if (rank() == root) {
        for (int r = 0; r < size(); ++r)
          if (r != root) send(sendbuf, bytes, r, s);
        if (recvbuf != sendbuf && bytes) std::memcpy(recvbuf, sendbuf, bytes);
      } else {
        recv(recvbuf, bytes, root, s);
      }
    } catch (...) {
      group_end();
      throw;
    }
    group_end();
  }
  bool ok() override { return w_->healthy(); }
  void abort() override { w_->abort(); }

 private:
  int check_peer(int p) const {
    if (p < 0 || p >= size() || p == rank())
      throw std::invalid_argument("socket comm: bad peer " + std::to_string(p));
    return p;
  }
  void post(const SOp& op) {
    if (t_depth > 0) {
      t_ops.push_back({w_.get(), op});
    } else {
      std::vector<SPending> one{{w_.get(), op}};
      run_sops(one);
    }
  }
  std::unique_ptr<SocketWorld> w_;
};

}  // namespace

std::string socket_unique_id() {
  // rank 0's bootstrap address + a nonce that every connecting rank presents
  int port = 0;
  const int fd = listen_any(&port);  // pick a free port now; rank 0 re-binds it in socket_init_rank
  close(fd);
  std::random_device rd;
  std::ostringstream s;
  s << "127.0.0.1:" << port << ":" << ((uint64_t)rd() << 32 | rd());
  return s.str();
}

std::unique_ptr<Comm> socket_init_rank(const std::string& unique_id, int nranks, int rank, int timeout_ms) {
  if (nranks < 1 || rank < 0 || rank >= nranks) throw std::invalid_argument("socket_init_rank: bad rank / size");
  const size_t c1 = unique_id.find(':'), c2 = unique_id.find(':', c1 + 1);
  if (c1 == std::string::npos || c2 == std::string::npos) throw std::invalid_argument("socket_init_rank: bad id");
  const std::string host = unique_id.substr(0, c1);
  const int port0 = std::stoi(unique_id.substr(c1 + 1, c2 - c1 - 1));
  const uint64_t nonce = std::stoull(unique_id.substr(c2 + 1));
  const auto deadline = Clock::now() + std::chrono::milliseconds(std::max(timeout_ms, 1000) * 3);
  std::vector<int> fds(nranks, -1);
  if (nranks == 1) return std::make_unique<SocketComm>(std::make_unique<SocketWorld>(1, 0, fds, timeout_ms));
  // every rank listens; rank 0 on the id's port (the bootstrap root)
  int my_port = rank == 0 ? port0 : 0;
  const int lfd = listen_any(&my_port);
  std::vector<int32_t> ports(nranks, 0);
  try {
    if (rank == 0) {
      // bootstrap: every other rank connects, presents {nonce, rank, port};
      // that connection is also the 0 <-> r mesh link
      ports[0] = my_port;
      for (int k = 1; k < nranks; ++k) {
        const int fd = accept_until(lfd, deadline);
        uint64_t hello[3];
        read_all(fd, hello, sizeof(hello));
        if (hello[0] != nonce || hello[1] == 0 || hello[1] >= (uint64_t)nranks || fds[hello[1]] >= 0) {
          close(fd);
          throw CommError("socket comm: bad bootstrap hello");
        }
        fds[hello[1]] = fd;
        ports[hello[1]] = (int32_t)hello[2];
      }
      for (int r = 1; r < nranks; ++r) write_all(fds[r], ports.data(), ports.size() * sizeof(int32_t));
    } else {
      fds[0] = connect_retry(host, port0, deadline);
      const uint64_t hello[3] = {nonce, (uint64_t)rank, (uint64_t)my_port};
      write_all(fds[0], hello, sizeof(hello));
      read_all(fds[0], ports.data(), ports.size() * sizeof(int32_t));
      // mesh: connect to every lower non-root rank, accept every higher one
      for (int j = 1; j < rank; ++j) {
        fds[j] = connect_retry(host, ports[j], deadline);
        const uint64_t me[2] = {nonce, (uint64_t)rank};
        write_all(fds[j], me, sizeof(me));
      }
      for (int k = rank + 1; k < nranks; ++k) {
        const int fd = accept_until(lfd, deadline);
        uint64_t who[2];
        read_all(fd, who, sizeof(who));
        if (who[0] != nonce || who[1] <= (uint64_t)rank || who[1] >= (uint64_t)nranks || fds[who[1]] >= 0) {
          close(fd);
          throw CommError("socket comm: bad mesh hello");
        }
        fds[who[1]] = fd;
      }
    }
  } catch (...) {
    close(lfd);
    for (int fd : fds)
      if (fd >= 0) close(fd);
    throw;
  }
  close(lfd);
  return std::make_unique<SocketComm>(std::make_unique<SocketWorld>(nranks, rank, fds, timeout_ms));
}

}  // namespace comm
}  // namespace dmlc
