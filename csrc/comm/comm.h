// Point-to-point communicators for the intra-node data plane.
//
// Reference counterpart: the reference has no collective library at all; its
// "fan-out" is one TCP RPC per single-image query to a random member
// (src/services.rs:407-433 -> Member::predict :475-497), and `train` copies a
// model file to every VM with scp (src/services.rs:139-144). Here the same
// roles are RCCL operations over xGMI between the GPUs of one node
// (SURVEY.md §2.4, §2.6):
//   * scatter of u8 image shards  = grouped send/recv (RCCL has no scatter)
//   * gather of top-1 answers     = grouped send/recv
//   * `train` weight distribution = broadcast
//
// Two implementations share this interface:
//   * RcclComm  (rccl_comm.cpp): ncclSend/ncclRecv/ncclBroadcast on a HIP
//     stream; one communicator per rank, built either per process from a
//     unique id (one process per GPU) or for all local GPUs of one process
//     (ncclCommInitAll).
//   * HostComm  (host_comm.cpp): an in-process fake over host memory with
//     RCCL's rendezvous, per-pair FIFO and grouping semantics, plus fault
//     injection (a rank can be declared lost). It runs the data-parallel
//     coordinator's shard/gather/recovery logic and the serving fleet's
//     partitions on CPU in tests (tests/test_dp_native_cpu.py,
//     tests/test_fleet_cpu.py).
#pragma once
#include <cstddef>
#include <cstdint>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace dmlc {
namespace comm {

using Stream = void*;  // hipStream_t for RCCL; ignored by the host fake

// A communicator error: a lost peer, an RCCL async error, an abort.
struct CommError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

class Comm {
 public:
  virtual ~Comm() = default;
  virtual int rank() const = 0;
  virtual int size() const = 0;
  virtual std::string backend() const = 0;

  // Grouping (RCCL: ncclGroupStart/End, thread-wide and nestable). Every
  // send/recv posted between the outermost start and end of a thread forms
  // one exchange; a single thread that drives several ranks puts all their
  // operations of a phase into one group.
  virtual void group_start() = 0;
  virtual void group_end() = 0;

  // Enqueued on `s`; the buffer must stay valid until the stream reaches
  // the operation (RCCL) / until group_end returns (host fake).
  virtual void send(const void* buf, size_t bytes, int peer, Stream s) = 0;
  virtual void recv(void* buf, size_t bytes, int peer, Stream s) = 0;
  virtual void broadcast(const void* sendbuf, void* recvbuf, size_t bytes, int root, Stream s) = 0;

  // Non-blocking health probe: false after an async error, a lost peer or
  // an abort.
  virtual bool ok() = 0;
  // Tear down without waiting for outstanding operations (RCCL:
  // ncclCommAbort, which also makes kernels stuck on a dead peer exit).
  virtual void abort() = 0;
};

// RAII group.
class Group {
 public:
  explicit Group(Comm& c) : c_(c) { c_.group_start(); }
  ~Group() noexcept(false) { c_.group_end(); }
  Group(const Group&) = delete;
  Group& operator=(const Group&) = delete;

 private:
  Comm& c_;
};

// ------------------------------------------------------------------ RCCL
constexpr size_t kUniqueIdBytes = 128;  // NCCL_UNIQUE_ID_BYTES

// ncclGetUniqueId, as raw bytes (rank 0 creates it and hands it to the other
// processes over any side channel; bench.py uses the gloo/TCP store).
std::string rccl_unique_id();
// One rank of an nranks communicator on HIP device `device` (one process
// per GPU).
std::unique_ptr<Comm> rccl_init_rank(const std::string& unique_id, int nranks, int rank, int device,
                                     int max_ctas = 0);
// Communicators for several GPUs driven by one process (ncclCommInitAll):
// result[i] is rank i on devices[i].
std::vector<std::unique_ptr<Comm>> rccl_init_all(const std::vector<int>& devices);

// ------------------------------------------------------------------ sockets
// Cross-process host communicator over loopback TCP (socket_comm.cpp): the
// process-per-rank shape of RCCL (a unique id from rank 0 handed out over a
// side channel, one rank per process) with the host fake's rendezvous, FIFO
// and grouping rules. bench.py --dry-run runs its multi-process path on it.
std::string socket_unique_id();
std::unique_ptr<Comm> socket_init_rank(const std::string& unique_id, int nranks, int rank, int timeout_ms = 20000);

// ------------------------------------------------------------------ host fake
// The data plane of an in-process fake world: how a matched send's bytes
// reach its receive. The host fake copies host memory at match time; the
// device loopback (loopback_comm.cpp) enqueues stream-ordered device copies.
class FakeDataPlane {
 public:
  virtual ~FakeDataPlane() = default;
  virtual std::string name() const = 0;
  // An operation is posted (its group ends) on stream s: a token for the
  // stream's position there (nullptr when positions do not matter).
  virtual void* mark(Stream s) = 0;
  // A send (posted at smark on ss) meets its receive (rmark on rs): move the
  // bytes after both positions, and order later work on both streams after
  // the move (RCCL: both kernels complete together).
  virtual void move(const void* sbuf, void* rbuf, size_t bytes, void* smark, Stream ss, void* rmark, Stream rs) = 0;
  // A copy within one rank, in stream order (a broadcast root's own buffer).
  virtual void local_copy(void* dst, const void* src, size_t bytes, Stream s) = 0;
  // The token of a matched, failed or withdrawn operation is no longer needed.
  virtual void release(void* mark) = 0;
};
// `n` communicators of one fake world over data plane `dp` (host_world: the
// host-memory plane).
std::vector<std::unique_ptr<Comm>> fake_world(int n, int timeout_ms, std::shared_ptr<FakeDataPlane> dp);
// The device loopback plane (loopback_comm.cpp, HIP): n virtual ranks whose
// buffers are device memory of the current device, a matched send/recv
// becoming hipMemcpyAsync on the world's copy stream between events recorded
// on the two ranks' streams. Matching stays the host fake's rendezvous rule,
// so a single-GPU test runs the multi-rank protocol with real streams,
// events and slot reuse (tests/test_dp_loopback_gpu.py).
std::vector<std::unique_ptr<Comm>> device_loopback_world(int n, int timeout_ms = 20000);
class HostWorld;  // shared mailbox state of one fake communicator
// `n` host communicators of one fake world; rank i = result[i]. Operations
// may be driven from one thread per rank or from one thread for all ranks.
// recv gives up after `timeout_ms` (a hang would otherwise stall the test).
std::vector<std::unique_ptr<Comm>> host_world(int n, int timeout_ms = 10000);
// Fault injection on a host communicator: every pending and later operation
// that involves `rank` fails with CommError.
void host_kill(Comm& any_member_of_world, int rank);
// Operations posted on the fake world but not matched yet (0 after every
// well-formed exchange: nothing is buffered).
size_t host_pending(Comm& any_member_of_world);

}  // namespace comm
}  // namespace dmlc
