// The serving fleet of one node: the GPUs split between the node's models
// (jobs), each model's partition serving its queries.
//
// Reference counterparts:
//   * fair share (`assign` loop, src/services.rs:199-211): every 3 s the
//     sorted active members are split, the first floor(n/2) to ResNet18 and
//     the rest to AlexNet, so the two concurrent jobs (:146-151) run on
//     disjoint halves of the cluster. Here the unit is a GPU of the node:
//     partition_devices() applies the same rule to the live GPUs (generalised
//     to J jobs as the leader's assign_loop does), and the split is redone
//     whenever a GPU is lost.
//   * per-query routing (`run_job`, :414-421: every query goes to one member
//     of the job's set): a query of a few images goes to ONE GPU of the
//     model's partition, the one with the fewest queries outstanding, and
//     runs there on a free compute lane, so independent small queries spread
//     over the whole partition instead of queueing on one GPU.
//   * a batch large enough to shard (>= 2 x min_shard images) is scattered
//     over the partition with RCCL instead (dp::Group: grouped send/recv over
//     xGMI, elastic on the loss of a GPU).
//   * the reference serialises concurrent queries per model behind a mutex
//     and runs each as its own batch-1 forward (`Member::predict`,
//     src/services.rs:475-497). Here concurrent direct queries routed to the
//     same (model, GPU) instance are COALESCED: they queue on the instance,
//     and whichever caller finds a free compute lane and a ready queue (full
//     batch, or the oldest request waited batch_window_us) stages every queued
//     request into that lane's batch buffer back to back and runs ONE
//     forward for all of them (real batching). A query
//     larger than max_per_rank is cut into max_per_rank chunks that queue the
//     same way, so its chunks run on several lanes at once (issued together,
//     synchronised oldest first) instead of one lane with a host sync per
//     chunk. The batch size of a forward is rounded up to a bucket (1, 2, 4,
//     ..., 64, then multiples of 32 up to max_per_rank), so each lane replays
//     one captured hipGraph per bucket.
//
// Invariants:
//   * partitions are disjoint whenever there are at least as many live GPUs
//     as models; with fewer, each model gets ONE GPU (models share it). Only a
//     partition of two or more GPUs has communicators, so no two models ever
//     hold RCCL communicators on the same device, and only one group (one
//     thread) drives a partition's communicators at a time;
//   * every query's answers are committed exactly once: a direct query that
//     fails on a lost GPU is redone whole on the rebalanced fleet; a scattered
//     one is redone image-exactly by dp::Group;
//   * rebalancing (and a hot swap's weight broadcast) runs with no query in
//     flight (exclusive plan lock).
#pragma once
#include <atomic>
#include <condition_variable>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <shared_mutex>
#include <string>
#include <vector>

#include "dp.h"

namespace dmlc {
namespace dp {

// Reference rule (src/services.rs:199-211) over the live GPUs, sorted:
// job j of J gets [j*n/J, (j+1)*n/J); with n < J job j gets GPU j % n alone.
std::vector<std::vector<int>> partition_devices(std::vector<int> live, int jobs);

// Forward batch for b coalesced images (FleetOptions::bucket_batches).
int bucket_batch(int b, int max);

struct FleetOptions {
  int max_per_rank = 256;         // images per GPU per forward (= the CU count: one round of the big-batch kernels)
  size_t image_bytes = 224 * 224 * 3;
  int min_shard = 32;             // scatter only batches of >= 2*min_shard, >= min_shard per GPU
  size_t aux_bytes = 0;           // scratch PER IMAGE handed to the stage function (a lane holds max_per_rank x it)
  int timeout_ms = 30000;         // dp::Group step timeout
  // Coalescing of direct queries: a queued request waits at most this long
  // for more requests to join its forward (0: a free lane takes whatever is
  // queued at once).
  int batch_window_us = 200;
  // ... except on an idle instance (no forward running): the first request
  // goes at once, later ones batch while it runs.
  bool eager_when_idle = true;
  // Round a forward's batch up to a bucket (bucket_batch(): powers of two to
  // 64, then multiples of 32, max_per_rank at most): a bounded set of
  // captured graphs per lane.
  bool bucket_batches = true;
};

// Where the stage function puts a query's images for a chosen worker.
struct StageCtx {
  Worker* worker = nullptr;
  int device = -1;
  int stream = 0;             // Worker stream id: enqueue the stage here
  void* batch = nullptr;      // worker memory, room for `capacity` images
  int64_t capacity = 0;
  void* aux = nullptr;        // worker memory, FleetOptions::aux_bytes
  void* aux_host = nullptr;   // pinned host memory, aux_bytes (free again once the stream passed the stage)
};
// Make images [first, first + n) of the query available, contiguous u8
// [n, H, W, 3], in ctx.worker's memory (enqueued on ctx.stream); return
// their address (ctx.batch or any other worker-memory address).
using StageFn = std::function<const uint8_t*(const StageCtx& ctx, int64_t first, int64_t n)>;

class Fleet {
 public:
  // replica_of == nullptr: build `model` on `device` from the host copy of
  // its weights. Otherwise a replica of that (same-model, live) instance whose
  // weight arena the fleet fills by an RCCL broadcast.
  using WorkerFactory =
      std::function<std::unique_ptr<Worker>(const std::string& model, int device, Worker* replica_of)>;
  // Communicators for these devices (rank i on devices[i]).
  using CommFactory = std::function<std::vector<std::unique_ptr<Comm>>(const std::vector<int>& devices)>;

  Fleet(std::vector<int> devices, WorkerFactory wf, CommFactory cf, FleetOptions opt = {});
  ~Fleet();
  Fleet(const Fleet&) = delete;
  Fleet& operator=(const Fleet&) = delete;

  // Order of the jobs for the partition rule (models not listed follow in
  // load order). Only loaded models take GPUs.
  void set_jobs(const std::vector<std::string>& models);
  // Load `model` (first time: the partitions are recomputed), or hot-swap
  // its weights (`train`): new instances are built from the host weights
  // while queries run, then swapped in under the plan lock.
  void load(const std::string& model);
  bool has(const std::string& model) const;

  struct Route {
    int device = -1;        // direct: the GPU that served it (last chunk)
    int devices_used = 1;   // scattered: GPUs of the partition used
    bool scattered = false;
    int retries = 0;        // redone after a GPU loss
  };
  struct QueryOptions {
    int prefer_device = -1;     // data locality: this GPU if it is in the partition and no busier than the rest
    bool allow_scatter = true;  // false: always one GPU per query (data already spread over the GPUs)
  };
  Route classify(const std::string& model, int64_t n, const StageFn& stage, int32_t* idx, float* prob,
                 QueryOptions q);
  Route classify(const std::string& model, int64_t n, const StageFn& stage, int32_t* idx, float* prob) {
    return classify(model, n, stage, idx, prob, QueryOptions());
  }

  std::map<std::string, std::vector<int>> partitions() const;
  std::vector<int> live() const;
  // Declare a GPU lost (operator / health check) and rebalance now.
  void lose(int device);
  // Images served per device for `model` (direct and scattered).
  std::map<int, int64_t> served(const std::string& model) const;
  // Direct-path forwards run per device for `model` (each may carry several
  // coalesced queries).
  std::map<int, int64_t> forwards(const std::string& model) const;
  // Direct-path forwards by (bucketed) batch size, over the partition.
  std::map<int, int64_t> forward_sizes(const std::string& model) const;
  int rebalances() const { return rebalances_.load(); }
  // The instance of `model` on `device` (nullptr if none): tests, hooks.
  Worker* worker(const std::string& model, int device) const;

 private:
  struct Instance;
  struct Model;
  struct DeviceLost {
    int device;
  };
  Model& get(const std::string& model) const;
  Route direct(Model& m, int64_t n, const StageFn& stage, int32_t* idx, float* prob, int prefer);
  Route scattered(Model& m, int64_t n, const StageFn& stage, int32_t* idx, float* prob);
  void mark_lost(int device);
  void rebalance();                          // takes the plan lock
  void apply_locked(Model& m, const std::vector<int>& devs, std::vector<std::shared_ptr<Instance>> fresh = {});
  std::vector<std::vector<int>> plan_locked() const;
  std::vector<std::string> order_locked() const;
  void broadcast_weights(Instance& src, const std::vector<Instance*>& dst);
  std::shared_ptr<Instance> make_instance(const std::string& model, int device, Worker* replica_of);

  std::vector<int> devices_;
  WorkerFactory wf_;
  CommFactory cf_;
  FleetOptions opt_;
  mutable std::shared_mutex plan_mu_;  // queries: shared; rebalance / swap: exclusive
  std::map<std::string, std::unique_ptr<Model>> models_;
  std::vector<std::string> jobs_, loaded_;  // partition order
  mutable std::mutex lost_mu_;
  std::set<int> lost_;
  std::atomic<bool> dirty_{false};  // a loss was seen: rebalance before the next query
  std::atomic<int> rebalances_{0};
  std::mutex load_mu_;  // one load / hot swap at a time
};

}  // namespace dp
}  // namespace dmlc
