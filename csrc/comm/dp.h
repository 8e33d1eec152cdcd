// Data-parallel batch inference over the GPUs of one node: the coordinator
// (rank 0) scatters u8 image shards, every rank classifies its shard, and the
// (class, probability) answers are gathered back to rank 0 — all enqueued on
// HIP streams so the transfers of one step overlap the compute of another.
//
// Reference counterpart: the leader's query fan-out (`run_job`,
// src/services.rs:407-433: one single-image TCP RPC per 0.5 s tick to a random
// member) and the member's forward (`Member::predict`, :475-497). SURVEY.md
// §2.3/§2.6 map that fan-out onto RCCL send/recv over xGMI.
//
// Layers:
//   Worker    one GPU's compute side: streams, events, memory, classify()
//             (HipWorker: the HIP engine; HostWorker: a CPU stand-in for tests)
//   Rank      one rank's per-step protocol (double-buffered slots, events)
//   Pipeline  the issue order of a run for the ranks one thread drives (one
//             rank per process, or every rank from one thread)
//   Group     one process owning several GPUs (dmlc-node --gpus N): runs a
//             classification job over them and survives the loss of a
//             non-coordinator GPU (abort, rebuild over the survivors, redo
//             every image whose answer was not yet committed).
#pragma once
#include <algorithm>
#include <cstdint>
#include <functional>
#include <memory>
#include <vector>

#include "comm.h"

namespace dmlc {
class Engine;
namespace dp {

using comm::Comm;
using comm::Stream;

class Worker {
 public:
  // kCompute2..: the streams of compute lanes 1.. (workers with lanes() > 1)
  enum StreamId { kCompute = 0, kIn = 1, kOut = 2, kCompute2 = 3 };
  static constexpr int kMaxLanes = 4;
  static int compute_stream(int lane) { return lane == 0 ? kCompute : kCompute2 + lane - 1; }
  virtual ~Worker() = default;
  virtual int device() const = 0;
  virtual void activate() {}                          // make this worker's device current
  virtual void* alloc(size_t bytes) = 0;              // device memory
  virtual void dealloc(void* p) = 0;
  virtual void* alloc_host(size_t bytes) = 0;         // pinned host memory
  virtual void dealloc_host(void* p) = 0;
  virtual Stream stream(int id) = 0;
  virtual int new_event() = 0;
  virtual void record(int ev, int stream_id) = 0;
  virtual void wait(int stream_id, int ev) = 0;       // stream waits for the event
  virtual bool query(int ev) = 0;                     // event reached?
  virtual void sync(int ev) = 0;
  virtual void sync_all() = 0;
  // Events that carry a timestamp (the coordinator-share calibration times
  // every rank's forward): elapsed_ms(a, b) once both have completed.
  virtual int new_timing_event() { return new_event(); }
  virtual double elapsed_ms(int ev_a, int ev_b) { (void)ev_a, (void)ev_b; return 0.0; }
  // Independent compute lanes (model instances with their own activations,
  // on their own streams): step slots alternate between them, so one step's
  // forward may start while the previous one's tail (head kernel, graph
  // completion) still runs.
  virtual int lanes() const { return 1; }
  // images: u8 [B, H, W, 3] (worker memory); answers written on
  // compute_stream(lane).
  virtual void classify(const uint8_t* images, int B, int32_t* idx, float* prob, int lane = 0) = 0;
  virtual void copy_d2h(void* dst, const void* src, size_t bytes, int stream_id) = 0;
  virtual void copy(void* dst, const void* src, size_t bytes, int stream_id) = 0;
  // False once the device reported an error (a lost GPU); never blocks.
  virtual bool healthy() { return true; }
  // The model's packed weights in worker memory (lane 0's): the fleet fills
  // a new replica's arena with an RCCL broadcast from a live instance of the
  // same model, then calls weights_updated() so the other lanes copy it.
  virtual void* weight_arena() { return nullptr; }
  virtual size_t weight_bytes() const { return 0; }
  virtual void weights_updated() {}
  // Never throws: used on teardown paths, where the device may be lost.
  virtual void sync_all_noexcept() noexcept {
    try {
      sync_all();
    } catch (...) {
    }
  }
};

// Host stand-in: plain memory, synchronous "streams" (events are no-ops), and
// a deterministic classifier: class = (sum of the image's bytes + w) %
// classes, prob = (first byte + 1) / 257, where w is the u32 at the start of
// its weight arena (`seed` for a worker built from "host weights"; 0 for a
// replica until the fleet broadcasts the arena into it).
// lanes: concurrent classify() calls it accepts (one per lane); delay_us:
// time one classify() takes (so concurrent queries overlap in tests).
// An unhealthy host worker's classify() throws CommError (a lost GPU).
// us_per_image / extra_us (calibration tests): a classify of B images takes
// delay_us + B x us_per_image + extra_us; extra_us on the coordinator stands
// for the CUs its scatter legs' copy kernels take from its forward on a GPU.
std::unique_ptr<Worker> make_host_worker(int device, int H, int W, int classes = 1000, int lanes = 1,
                                         uint32_t seed = 0, int delay_us = 0, int us_per_image = 0,
                                         int extra_us = 0);
// Test hook: a host worker that reports itself unhealthy (a lost GPU).
void host_worker_set_healthy(Worker& w, bool healthy);
// The HIP engine on its device (csrc/comm/hip_worker.cpp): images are u8
// [B, H, W, 3]; use_graph replays the engine's captured hipGraph.
// more: further instances of the model on the same device (their own
// activation arenas, captured graphs and streams; weights copied from
// `engine`), owned by the caller like `engine`: lanes() == 1 + more.size().
std::unique_ptr<Worker> make_hip_worker(Engine* engine, int H, int W, bool use_graph = true,
                                        std::vector<Engine*> more = {});
// The same, owning its engines (engines[0] = lane 0): the serving fleet's
// per-(model, GPU) instances.
std::unique_ptr<Worker> make_owned_hip_worker(std::vector<std::unique_ptr<Engine>> engines, int H, int W,
                                              bool use_graph = true);
// Lane `lane`'s engine of a HIP worker (throws for other workers).
Engine* hip_worker_engine(Worker& w, int lane = 0);
int host_class_of(const uint8_t* img, size_t bytes, int classes = 1000);
float host_prob_of(const uint8_t* img);

// Balanced split of n images over `world` ranks (lower ranks take the
// remainder), every count <= cap.
std::vector<int> shard_counts(int64_t n, int world, int cap);

// Coordinator-share calibration. The coordinator drives every scatter leg
// next to its own forward (on a GPU, RCCL's copy kernels hold CUs its
// one-workgroup-per-CU convs need), so with an even split the whole job runs
// at its pace. One round: a run at weight w (its share of a fair per-rank
// batch) measures the coordinator's forward busy time b0 and the slowest
// other rank's bw (ms per step).
struct CalibRound {
  double weight = 1.0;
  double busy_coord = 0.0, busy_worker = 0.0;
  int coord_count = 0, per_rank = 0, world = 1;
  // images per ms of the job at this weight, if the step runs at the pace of
  // its slowest rank
  double rate() const;
};
// Next weight to try: the coordinator's count scaled by bw / b0 (equal busy
// times under a time ~ count model), within [min_weight, 1].
double next_coord_weight(const CalibRound& r, double min_weight = 0.5);
// The measured weight with the highest rate (ties: the larger weight).
double best_coord_weight(const std::vector<CalibRound>& rounds);
// A step's split of n images with the coordinator weighted: rank 0 takes a
// w0 share relative to each other rank (at most round(w0 x cap)), the others
// a balanced split of the rest (at most cap each).
std::vector<int> weighted_shards(int64_t n, int world, int cap, double w0);

struct StepPlan {
  int64_t step = 0;          // sequence number; slot = step % slots
  std::vector<int> counts;   // images per rank (same on every rank)
  // scatter mode: the step's images on the coordinator (rank r's shard at
  // image offset sum(counts[0..r))); local mode: this rank's own images.
  const uint8_t* src = nullptr;
  int src_event = -1;        // coordinator: event (on kCompute) after which src is valid
};

class Rank {
 public:
  // scatter: the coordinator sends every other rank its shard; otherwise
  // each rank reads its own images (local mode: no input transfer).
  Rank(Worker* w, int max_per_rank, size_t image_bytes, bool scatter, int slots = 2);
  ~Rank();
  Rank(const Rank&) = delete;
  Rank& operator=(const Rank&) = delete;

  // (Re)bind to communicators: `in` carries shards, `out` carries answers
  // (separate communicators on separate streams, so a gather is never queued
  // behind the next step's scatter). The coordinator is rank 0 of both.
  void attach(Comm* in, Comm* out);
  int rank() const { return in_ ? in_->rank() : 0; }
  int world() const { return in_ ? in_->size() : 1; }
  bool root() const { return rank() == 0; }
  Worker* worker() const { return w_; }
  int max_per_rank() const { return max_; }
  int slots() const { return slots_; }

  // Phases of one step; post_* go inside a comm group, after_* right after it.
  void post_input(const StepPlan& p);
  void after_input(const StepPlan& p);
  void compute(const StepPlan& p);
  void post_output(const StepPlan& p);
  void after_output(const StepPlan& p);
  // Coordinator: wait for the step's answers (timeout_ms < 0: forever; on a
  // timeout or a communicator error throws CommError) and copy them in
  // global image order.
  void collect(const StepPlan& p, int32_t* idx, float* prob, int timeout_ms = -1);
  // Wait until the step's answers have left (non-root) / landed (root).
  void wait_step(const StepPlan& p, int timeout_ms = -1);
  // Forward time of the steps completed since reset_busy() (timing events
  // around each classify on its compute stream): total ms, steps, images.
  double busy_ms() const { return busy_ms_; }
  int64_t busy_steps() const { return busy_steps_; }
  int64_t busy_images() const { return busy_images_; }
  void reset_busy() { busy_ms_ = 0.0, busy_steps_ = 0, busy_images_ = 0; }
  // Account every step whose forward has completed but was not waited on
  // through this rank (a group's non-coordinator ranks, after a run).
  void settle_busy();
  Comm* comm_in() const { return in_; }
  Comm* comm_out() const { return out_; }
  // Forget slot history (after a rebuild every slot is free again).
  void reset();

 private:
  int slot(const StepPlan& p) const { return (int)(p.step % slots_); }
  size_t block_bytes() const { return (size_t)max_ * 8; }  // [idx int32 x max][prob f32 x max]
  Worker* w_;
  Comm* in_ = nullptr;
  Comm* out_ = nullptr;
  int max_, slots_;
  size_t ib_;
  bool scatter_;
  std::vector<void*> inbuf_;       // non-root scatter: received shards
  std::vector<void*> ans_;         // answers: root world blocks, others one block
  std::vector<void*> host_ans_;    // root: pinned copy of the gathered answers
  std::vector<int> ev_in_, ev_comp_, ev_out_;
  std::vector<int> ev_t0_, ev_t1_;  // timing: around the slot's classify
  std::vector<int> slot_n_;         // images of the slot's step (-1: no timing pending)
  double busy_ms_ = 0.0;
  int64_t busy_steps_ = 0, busy_images_ = 0;
  std::vector<bool> in_used_, out_used_;
  int ans_world_ = 0;
};

// Issue order for the ranks one thread drives (all in one comm group per
// phase): input(first); per step i: input(i+1), compute(i), output(i), then
// the coordinator collects step i-(slots-1) (with 2 slots one step behind,
// so the host never waits for the step it just issued). All ranks of one
// call must have the same slot count.
struct PipelineResult {
  int64_t steps = 0, images = 0;
  std::vector<double> step_ms;  // unpipelined runs: input issue -> answers collected, per step (coordinator)
  double busy_ms = 0.0;         // this rank's mean forward time per step (the first rank this thread drives)
};
using PlanFn = std::function<StepPlan(int64_t step, const Rank& r)>;
using ResultFn = std::function<void(const StepPlan& p, const int32_t* idx, const float* prob)>;
PipelineResult run_pipeline(const std::vector<Rank*>& ranks, int64_t first, int64_t n, const PlanFn& plan,
                            const ResultFn& on_result, int timeout_ms = -1, bool pipelined = true);

// One process owning several GPUs.
class Group {
 public:
  using CommFactory = std::function<std::vector<std::unique_ptr<Comm>>(const std::vector<int>& members)>;
  // workers[0] is the coordinator. make_comms(members) returns one
  // communicator per member (rank i = members[i]); it is called twice per
  // (re)build (shards and answers use separate communicators).
  Group(std::vector<Worker*> workers, CommFactory make_comms, int max_per_rank, size_t image_bytes,
        int timeout_ms = 30000);
  ~Group();

  struct Stats {
    int64_t images = 0, steps = 0;
    int recoveries = 0;
    int64_t redone_images = 0;  // images classified again after a loss
    std::vector<int64_t> per_worker;  // images answered by each worker (index into workers)
    int ranks_used = 0;               // most ranks one step used
  };
  // Classify n images stored contiguously at `src` (coordinator memory),
  // answers in input order. `src_event`: coordinator event after which src
  // is valid (-1: already valid).
  // commit_count (optional, n entries): +1 per image each time its answer is
  // committed (tests check exactly-once).
  Stats classify(const uint8_t* src, int64_t n, int32_t* idx, float* prob, int src_event = -1,
                 int32_t* commit_count = nullptr);
  // Fault injection: member `m` (index into workers, not the coordinator)
  // is lost before its next step; with after_steps > 0, once that many more
  // steps have been issued. The lost GPU is dropped without a communicator
  // error (the operations already posted complete), then the group rebuilds.
  // abrupt (host communicators only, a test hook): the member dies in the
  // middle of that step instead — its communicator operations fail and its
  // worker reports unhealthy — so the recovery runs from a CommError, as
  // after a real GPU loss.
  void fail(int m, int64_t after_steps = 0, bool abrupt = false);
  std::vector<int> members() const { return members_; }
  int size() const { return (int)members_.size(); }
  // A step of n images uses ceil(n / min_per_rank) ranks at most (small
  // query batches stay on few GPUs; default 1 = always all ranks).
  void set_min_per_rank(int m) { min_per_rank_ = std::max(1, m); }
  Worker* coordinator() const { return workers_.front(); }
  // The coordinator's share of a step relative to the other ranks (it drives
  // every scatter leg). With auto_balance (the default) each classify() of
  // two or more steps re-estimates it from the ranks' forward time per image
  // (smoothed), so the coordinator stops setting the pace of every step.
  double coord_weight() const { return coord_weight_; }
  void set_coord_weight(double w, bool auto_balance);

 private:
  void rebuild();
  std::vector<Worker*> workers_;
  CommFactory make_comms_;
  int max_;
  size_t ib_;
  int timeout_ms_;
  std::vector<int> members_;  // live workers, coordinator first
  std::vector<std::unique_ptr<Rank>> ranks_;  // one per worker (index = worker)
  std::vector<std::unique_ptr<Comm>> cin_, cout_;
  std::vector<bool> lost_;
  std::vector<bool> killed_;  // kill_now()ed: its communicator operations fail, whatever its worker says
  std::vector<int64_t> fail_at_;  // per worker: steps still to issue before it is lost (-1: never)
  std::vector<bool> fail_abrupt_;
  int min_per_rank_ = 1;
  double coord_weight_ = 1.0;
  bool auto_balance_ = true;
  void kill_now(int m);
  void rebalance_coord(const std::vector<Rank*>& rs);
};

}  // namespace dp
}  // namespace dmlc
