// RCCL communicators (ROCm's NCCL) for the intra-node data plane over xGMI.
//
// Every MI355X of a node has a direct xGMI link to each of its 7 peers, so a
// grouped set of point-to-point sends from the coordinator uses distinct
// links concurrently; each leg is bound by one link (~150 GB/s). That is why
// the data plane is built from grouped ncclSend/ncclRecv (scatter of u8
// shards, gather of 8-byte answers) rather than ring collectives.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>

#include "comm.h"

namespace dmlc {
namespace comm {
namespace {

void check(ncclResult_t r, const char* what) {
  if (r != ncclSuccess && r != ncclInProgress)
    throw CommError(std::string("RCCL ") + what + ": " + ncclGetErrorString(r));
}

class RcclComm : public Comm {
 public:
  RcclComm(ncclComm_t c, int device) : c_(c), device_(device) {
    check(ncclCommUserRank(c_, &rank_), "ncclCommUserRank");
    check(ncclCommCount(c_, &size_), "ncclCommCount");
  }
  ~RcclComm() override {
    if (!c_) return;
    (void)hipSetDevice(device_);
    if (aborted_) return;
    ncclCommDestroy(c_);
  }
  int rank() const override { return rank_; }
  int size() const override { return size_; }
  std::string backend() const override { return "rccl"; }

  void group_start() override { check(ncclGroupStart(), "ncclGroupStart"); }
  void group_end() override { check(ncclGroupEnd(), "ncclGroupEnd"); }

  void send(const void* buf, size_t bytes, int peer, Stream s) override {
    live();
    check(ncclSend(buf, bytes, ncclUint8, peer, c_, (hipStream_t)s), "ncclSend");
  }
  void recv(void* buf, size_t bytes, int peer, Stream s) override {
    live();
    check(ncclRecv(buf, bytes, ncclUint8, peer, c_, (hipStream_t)s), "ncclRecv");
  }
  void broadcast(const void* sendbuf, void* recvbuf, size_t bytes, int root, Stream s) override {
    live();
    check(ncclBroadcast(sendbuf, recvbuf, bytes, ncclUint8, root, c_, (hipStream_t)s), "ncclBroadcast");
  }
  bool ok() override {
    if (aborted_) return false;
    ncclResult_t a = ncclSuccess;
    if (ncclCommGetAsyncError(c_, &a) != ncclSuccess) return false;
    return a == ncclSuccess || a == ncclInProgress;
  }
  void abort() override {
    if (aborted_) return;
    (void)hipSetDevice(device_);
    ncclCommAbort(c_);
    aborted_ = true;
  }

 private:
  void live() const {
    if (aborted_) throw CommError("RCCL communicator was aborted");
  }
  ncclComm_t c_ = nullptr;
  int device_ = 0, rank_ = 0, size_ = 1;
  bool aborted_ = false;
};

}  // namespace

std::string rccl_unique_id() {
  ncclUniqueId id;
  check(ncclGetUniqueId(&id), "ncclGetUniqueId");
  static_assert(sizeof(id.internal) == kUniqueIdBytes, "unique id size");
  return std::string(id.internal, sizeof(id.internal));
}

std::unique_ptr<Comm> rccl_init_rank(const std::string& unique_id, int nranks, int rank, int device, int max_ctas) {
  if (unique_id.size() != kUniqueIdBytes) throw std::invalid_argument("rccl_init_rank: unique id must be 128 bytes");
  if (rank < 0 || rank >= nranks) throw std::invalid_argument("rccl_init_rank: bad rank");
  ncclUniqueId id;
  std::memcpy(id.internal, unique_id.data(), kUniqueIdBytes);
  if (hipSetDevice(device) != hipSuccess) throw CommError("rccl_init_rank: hipSetDevice failed");
  ncclComm_t c = nullptr;
  if (max_ctas > 0) {
    // Cap the CTAs (= CUs held while an operation runs) of this
    // communicator's kernels: the answer gather moves 8 B per image and needs
    // one, and every CU it does not hold is one the forward keeps (its convs
    // run one workgroup per CU: a CU held by a comm kernel delays a whole
    // workgroup of them, profiles/r1_interference.txt).
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    cfg.minCTAs = 1;
    cfg.maxCTAs = max_ctas;
    check(ncclCommInitRankConfig(&c, nranks, id, rank, &cfg), "ncclCommInitRankConfig");
  } else {
    check(ncclCommInitRank(&c, nranks, id, rank), "ncclCommInitRank");
  }
  return std::make_unique<RcclComm>(c, device);
}

std::vector<std::unique_ptr<Comm>> rccl_init_all(const std::vector<int>& devices) {
  if (devices.empty()) throw std::invalid_argument("rccl_init_all: no devices");
  std::vector<ncclComm_t> cs(devices.size(), nullptr);
  check(ncclCommInitAll(cs.data(), (int)devices.size(), devices.data()), "ncclCommInitAll");
  std::vector<std::unique_ptr<Comm>> out;
  for (size_t i = 0; i < devices.size(); ++i) out.push_back(std::make_unique<RcclComm>(cs[i], devices[i]));
  return out;
}

}  // namespace comm
}  // namespace dmlc
