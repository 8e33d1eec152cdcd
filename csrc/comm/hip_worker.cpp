// dp::Worker on one MI355X: the HIP engine on a compute stream, and two
// communication streams (shards in, answers out) created at a higher
// priority, so the RCCL send/recv kernels of the next step are dispatched
// promptly next to the running forward instead of queueing behind its
// workgroups. With a second engine instance (lane 2) on its own stream,
// consecutive steps alternate between the two: step i+1's stem fills the
// CUs that step i's head kernel (16 workgroups) and the end of its graph
// leave idle (~40 us per ResNet18 b256 step: profiles/r2_lanes.txt).
#include <hip/hip_runtime.h>

#include "../kernels/kernels.h"
#include "../runtime/engine.h"
#include "dp.h"

namespace dmlc {
namespace dp {
namespace {

class HipWorker : public Worker {
 public:
  HipWorker(Engine* e, int H, int W, bool use_graph, std::vector<Engine*> more)
      : dev_(e->device()), H_(H), W_(W), graph_(use_graph) {
    e_.push_back(e);
    for (Engine* x : more) {
      if (!x || x->device() != dev_ || x->arch() != e->arch())
        throw std::invalid_argument("HipWorker: every lane must be the same model on the same device");
      e_.push_back(x);
    }
    if ((int)e_.size() > kMaxLanes) throw std::invalid_argument("HipWorker: too many lanes");
    DMLC_HIP_CHECK(hipSetDevice(dev_));
    int lo = 0, hi = 0;
    DMLC_HIP_CHECK(hipDeviceGetStreamPriorityRange(&lo, &hi));
    // With two lanes, lane 0 runs at high priority: its workgroups dispatch
    // first as CUs free up and lane 1 fills the gaps (its kernels' tails and
    // the one-workgroup-per-CU convs' partial last rounds), instead of the two
    // forwards contending evenly: +0.6-1.1% img/s in two same-box interleaved
    // A/Bs (profiles/r2_lanes.txt)
    DMLC_HIP_CHECK(hipStreamCreateWithPriority(&s_[kCompute], hipStreamNonBlocking, e_.size() > 1 ? hi : lo));
    DMLC_HIP_CHECK(hipStreamCreateWithPriority(&s_[kIn], hipStreamNonBlocking, hi));
    DMLC_HIP_CHECK(hipStreamCreateWithPriority(&s_[kOut], hipStreamNonBlocking, hi));
    for (size_t l = 1; l < e_.size(); ++l)
      DMLC_HIP_CHECK(hipStreamCreateWithPriority(&s_[compute_stream((int)l)], hipStreamNonBlocking, lo));
  }
  ~HipWorker() override {
    (void)hipSetDevice(dev_);
    for (auto s : s_)
      if (s) (void)hipStreamSynchronize(s);
    for (auto ev : evs_) (void)hipEventDestroy(ev);
    for (auto s : s_)
      if (s) (void)hipStreamDestroy(s);
  }
  int device() const override { return dev_; }
  void activate() override { DMLC_HIP_CHECK(hipSetDevice(dev_)); }
  void* alloc(size_t bytes) override {
    void* p = nullptr;
    activate();
    DMLC_HIP_CHECK(hipMalloc(&p, std::max<size_t>(bytes, 256)));
    return p;
  }
  void dealloc(void* p) override {
    activate();
    (void)hipFree(p);
  }
  void* alloc_host(size_t bytes) override {
    void* p = nullptr;
    DMLC_HIP_CHECK(hipHostMalloc(&p, std::max<size_t>(bytes, 256), hipHostMallocDefault));
    return p;
  }
  void dealloc_host(void* p) override { (void)hipHostFree(p); }
  Stream stream(int id) override { return s_[id]; }
  int lanes() const override { return (int)e_.size(); }
  int new_event() override {
    activate();
    hipEvent_t ev;
    DMLC_HIP_CHECK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    evs_.push_back(ev);
    return (int)evs_.size() - 1;
  }
  int new_timing_event() override {
    activate();
    hipEvent_t ev;
    DMLC_HIP_CHECK(hipEventCreate(&ev));
    evs_.push_back(ev);
    return (int)evs_.size() - 1;
  }
  double elapsed_ms(int a, int b) override {
    float ms = 0.f;
    DMLC_HIP_CHECK(hipEventElapsedTime(&ms, evs_.at(a), evs_.at(b)));
    return ms;
  }
  void record(int ev, int sid) override { DMLC_HIP_CHECK(hipEventRecord(evs_.at(ev), s_[sid])); }
  void wait(int sid, int ev) override { DMLC_HIP_CHECK(hipStreamWaitEvent(s_[sid], evs_.at(ev), 0)); }
  bool query(int ev) override {
    hipError_t e = hipEventQuery(evs_.at(ev));
    if (e == hipSuccess) return true;
    if (e == hipErrorNotReady) return false;
    throw comm::CommError(std::string("dp: device ") + std::to_string(dev_) + " error: " + hipGetErrorString(e));
  }
  void sync(int ev) override { DMLC_HIP_CHECK(hipEventSynchronize(evs_.at(ev))); }
  void sync_all() override {
    activate();
    for (auto s : s_)
      if (s) DMLC_HIP_CHECK(hipStreamSynchronize(s));
  }
  void classify(const uint8_t* images, int B, int32_t* idx, float* prob, int lane) override {
    if (lane < 0 || lane >= lanes()) throw std::invalid_argument("HipWorker: no such compute lane");
    e_[lane]->forward(images, B, H_, W_, idx, prob, nullptr, s_[compute_stream(lane)], graph_);
  }
  // dst is pinned host memory (alloc_host). A plain DeviceToHost copy runs as
  // a blit kernel (__amd_rocclr_copyBuffer, ~4 us): on the high-priority
  // answer stream it takes a CU slot while the forward's one-workgroup-per-CU
  // convs launch, and a displaced workgroup costs that conv a second round.
  // The NoCU kind goes through a copy engine (tools/probes/nocu_copy_probe.hip:
  // exact, no kernel in the trace).
  void copy_d2h(void* dst, const void* src, size_t bytes, int sid) override {
    DMLC_HIP_CHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDeviceNoCU, s_[sid]));
  }
  void copy(void* dst, const void* src, size_t bytes, int sid) override {
    DMLC_HIP_CHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDefault, s_[sid]));
  }
  void* weight_arena() override { return e_[0]->weight_arena(); }
  size_t weight_bytes() const override { return e_[0]->weight_bytes(); }
  void weights_updated() override {
    for (size_t l = 1; l < e_.size(); ++l) e_[l]->copy_weights_from(*e_[0]);
  }
  Engine* engine(int lane) const { return e_.at(lane); }
  // engines this worker owns (make_owned_hip_worker), destroyed after it
  std::vector<std::unique_ptr<Engine>> owned_;

  bool healthy() override {
    for (auto s : s_) {
      if (!s) continue;
      hipError_t e = hipStreamQuery(s);
      if (e != hipSuccess && e != hipErrorNotReady) return false;
    }
    return true;
  }

 private:
  std::vector<Engine*> e_;
  int dev_, H_, W_;
  bool graph_;
  hipStream_t s_[kCompute2 + kMaxLanes - 1] = {};
  std::vector<hipEvent_t> evs_;
};

}  // namespace

std::unique_ptr<Worker> make_hip_worker(Engine* engine, int H, int W, bool use_graph, std::vector<Engine*> more) {
  return std::make_unique<HipWorker>(engine, H, W, use_graph, std::move(more));
}

std::unique_ptr<Worker> make_owned_hip_worker(std::vector<std::unique_ptr<Engine>> engines, int H, int W,
                                              bool use_graph) {
  if (engines.empty()) throw std::invalid_argument("make_owned_hip_worker: no engines");
  std::vector<Engine*> more;
  for (size_t l = 1; l < engines.size(); ++l) more.push_back(engines[l].get());
  auto w = std::make_unique<HipWorker>(engines[0].get(), H, W, use_graph, std::move(more));
  w->owned_ = std::move(engines);
  return w;
}

Engine* hip_worker_engine(Worker& w, int lane) {
  auto* h = dynamic_cast<HipWorker*>(&w);
  if (!h) throw std::invalid_argument("hip_worker_engine: not a HIP worker");
  return h->engine(lane);
}

}  // namespace dp
}  // namespace dmlc
