// Device loopback data plane for the in-process fake communicator: several
// virtual ranks on ONE GPU, each with its own HIP worker, engines and streams,
// exchange device buffers with stream-ordered copies.
//
// Why: the data-parallel protocol (dp::Runner's double-buffered slots and
// per-slot events, the HIP worker's lane alternation, dp::Group's recovery)
// runs at world > 1 on the boxes this repository gets only as one GPU. The
// host fake (host_comm.cpp) checks the protocol's matching and ordering on the
// host, but moves bytes synchronously, so a slot reused before the stream has
// finished sending it, or an answer read before its copy landed, cannot show
// up there. Here every operation keeps RCCL's stream semantics:
//   * posting an operation (its group's end) records an event on the rank's
//     stream: the point the RCCL kernel would start;
//   * a matched send/recv (the host fake's rendezvous and per-pair FIFO rule)
//     becomes hipMemcpyAsync on the world's copy stream after BOTH events, and
//     both ranks' streams wait for the copy's completion event before any
//     later work (an RCCL send/recv pair completes together);
//   * nothing is synchronised on the host: a protocol that reads a buffer
//     without waiting on the right stream reads stale or torn data.
// Faults (host_kill, abort) and timeouts behave as in the host fake.
#include <hip/hip_runtime.h>

#include <mutex>
#include <vector>

#include "comm.h"

#define DMLC_LB_CHECK(x)                                                                              \
  do {                                                                                                \
    hipError_t e_ = (x);                                                                              \
    if (e_ != hipSuccess) throw CommError(std::string("loopback comm: ") + hipGetErrorString(e_)); \
  } while (0)

namespace dmlc {
namespace comm {

namespace {

class DevicePlane : public FakeDataPlane {
 public:
  DevicePlane() {
    DMLC_LB_CHECK(hipGetDevice(&device_));
    DMLC_LB_CHECK(hipStreamCreateWithFlags(&copy_, hipStreamNonBlocking));
  }
  ~DevicePlane() override {
    (void)hipSetDevice(device_);
    (void)hipStreamSynchronize(copy_);
    for (hipEvent_t e : all_) (void)hipEventDestroy(e);
    (void)hipStreamDestroy(copy_);
  }
  std::string name() const override { return "loopback"; }
  void* mark(Stream s) override {
    hipEvent_t e = take();
    DMLC_LB_CHECK(hipEventRecord(e, (hipStream_t)s));
    return e;
  }
  void move(const void* sbuf, void* rbuf, size_t bytes, void* smark, Stream ss, void* rmark, Stream rs) override {
    DMLC_LB_CHECK(hipStreamWaitEvent(copy_, (hipEvent_t)smark, 0));
    DMLC_LB_CHECK(hipStreamWaitEvent(copy_, (hipEvent_t)rmark, 0));
    if (bytes) DMLC_LB_CHECK(hipMemcpyAsync(rbuf, sbuf, bytes, hipMemcpyDeviceToDevice, copy_));
    hipEvent_t done = take();
    DMLC_LB_CHECK(hipEventRecord(done, copy_));
    DMLC_LB_CHECK(hipStreamWaitEvent((hipStream_t)ss, done, 0));
    DMLC_LB_CHECK(hipStreamWaitEvent((hipStream_t)rs, done, 0));
    release(done);
  }
  void local_copy(void* dst, const void* src, size_t bytes, Stream s) override {
    if (bytes && dst != src) DMLC_LB_CHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, (hipStream_t)s));
  }
  // An event handed back here may still be waited on by enqueued work: it is
  // re-recorded only after the copy stream drained past every use (events
  // are recycled in batches behind a copy-stream synchronisation).
  void release(void* m) override {
    if (!m) return;
    std::lock_guard<std::mutex> g(mu_);
    used_.push_back((hipEvent_t)m);
  }

 private:
  hipEvent_t take() {
    std::lock_guard<std::mutex> g(mu_);
    if (free_.empty() && used_.size() >= 256) {
      // every released event's last use is behind work already enqueued on
      // the copy stream or on a rank stream waiting for it: once the device
      // is idle they are all reusable
      DMLC_LB_CHECK(hipDeviceSynchronize());
      free_.swap(used_);
    }
    if (free_.empty()) {
      hipEvent_t e;
      DMLC_LB_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
      all_.push_back(e);
      return e;
    }
    hipEvent_t e = free_.back();
    free_.pop_back();
    return e;
  }
  int device_ = 0;
  hipStream_t copy_ = nullptr;
  std::mutex mu_;
  std::vector<hipEvent_t> all_, free_, used_;
};

}  // namespace

std::vector<std::unique_ptr<Comm>> device_loopback_world(int n, int timeout_ms) {
  return fake_world(n, timeout_ms, std::make_shared<DevicePlane>());
}

}  // namespace comm
}  // namespace dmlc
