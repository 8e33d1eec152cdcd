// One rank of a multi-process data-parallel job (one process per GPU):
// bench.py's serving step. Rank 0 holds the image pool; every step its
// shards go to the ranks over RCCL (scatter mode) or were placed in each
// rank's HBM beforehand (staged mode, stage()), every rank classifies its
// shard, and the answers are gathered to rank 0 on a second communicator.
//
// The same class runs on host workers and the rendezvous host communicator
// in CPU tests (tests/test_dp_native_cpu.py::test_bench_protocol_*), so the
// exact call sequence bench.py issues (stage, prime run, warmup, timed run,
// unpipelined latency run) is exercised for world 2..8 without GPUs.
//
// Reference counterpart: the leader's fan-out of queries to members
// (src/services.rs:414-421) and the replies.
#pragma once
#include <functional>
#include <memory>
#include <vector>

#include "dp.h"

namespace dmlc {
namespace dp {

// Per-rank image counts of one step: every rank classifies `per_rank` images
// except rank 0 (the coordinator, which also drives every scatter leg), which
// takes round(coord_weight x per_rank) (coord_weight in (0, 1]; 1: an even
// split). The other ranks are never raised above per_rank: at per_rank = 256
// (the CU count) the one-workgroup-per-image kernels would run a second,
// nearly empty round.
std::vector<int> weighted_counts(int per_rank, int world, double coord_weight);

class Runner {
 public:
  // counts: images per rank per step (every rank passes the same vector);
  // max_per_rank >= every count.
  Runner(std::unique_ptr<Worker> w, std::unique_ptr<Comm> in, std::unique_ptr<Comm> out, int world, int rank,
         std::vector<int> counts, bool scatter, size_t image_bytes, int timeout_ms = -1, int slots = 0);
  ~Runner();

  // Steps [first, first + n). Scatter mode: the coordinator's pool holds
  // global batches back to back (sum(counts) images each). Staged/local
  // mode: this rank's pool holds per-rank batches at a stride of
  // max_per_rank() images (counts[rank] used per step).
  PipelineResult run(const uint8_t* pool, int64_t pool_images, int64_t first, int64_t n, bool pipelined = true);
  // Place one global batch's shards in the ranks' memory: the coordinator's
  // global batch at `src` (rank r's shard at its count offset) goes to `dst`
  // on rank r over the shard communicator (rank 0's own part by a device
  // copy). Blocks until done.
  void stage(const uint8_t* src, uint8_t* dst);

  // New per-rank counts between runs (every rank the same vector, each count
  // <= max_per_rank()): the coordinator share after a calibration.
  void set_counts(const std::vector<int>& counts);

  // Coordinator-share calibration (scatter mode, world > 1): up to `rounds`
  // runs of `steps` pipelined steps; after each, every rank's mean forward
  // time per step is all-gathered (allgather: this rank's value -> every
  // rank's, in rank order; every rank calls it the same number of times) and
  // the coordinator's count re-solved (next_coord_weight) until its forward
  // time is within `tol` of the slowest other rank's. Ends on the measured
  // weight with the best rate (best_coord_weight); every rank computes the
  // same decisions from the same gathered values.
  struct Calibration {
    double weight = 1.0;
    std::vector<CalibRound> rounds;
    int64_t steps = 0;
  };
  using AllGather = std::function<std::vector<double>(double)>;
  Calibration calibrate(const uint8_t* pool, int64_t pool_images, int64_t first, int64_t steps, int rounds,
                        double tol, const AllGather& allgather, double min_weight = 0.5);

  Worker* worker() const { return w_.get(); }
  int world() const { return world_; }
  int rank() const { return rank_; }
  int max_per_rank() const { return max_; }
  const std::vector<int>& counts() const { return counts_; }
  int64_t global_batch() const;
  const std::vector<int32_t>& last_idx() const { return last_idx_; }
  const std::vector<float>& last_prob() const { return last_prob_; }
  // Called on the coordinator with every step's gathered answers (step,
  // idx, prob, global batch) as run() commits them (tests: every step, not
  // only the last, is checked).
  using StepHook = std::function<void(int64_t step, const int32_t* idx, const float* prob, int64_t n)>;
  void set_step_hook(StepHook h) { hook_ = std::move(h); }

 private:
  std::unique_ptr<Worker> w_;
  std::unique_ptr<Comm> in_, out_;
  int world_, rank_;
  std::vector<int> counts_;
  int max_;
  bool scatter_;
  size_t ib_;
  int timeout_ms_;
  std::unique_ptr<Rank> r_;
  std::vector<int32_t> last_idx_;
  std::vector<float> last_prob_;
  StepHook hook_;
};

}  // namespace dp
}  // namespace dmlc
