#include "runner.h"

#include <cmath>
#include <numeric>
#include <stdexcept>

namespace dmlc {
namespace dp {

std::vector<int> weighted_counts(int per_rank, int world, double coord_weight) {
  if (world < 1 || per_rank < 1) throw std::invalid_argument("weighted_counts: need world >= 1 and per_rank >= 1");
  if (!(coord_weight > 0.0) || coord_weight > 1.0)
    throw std::invalid_argument("weighted_counts: coord_weight must be in (0, 1]");
  // the other ranks keep exactly per_rank: a batch above it would push the
  // one-workgroup-per-image kernels (per_rank = 256 = the CU count) into a
  // second, nearly empty round
  std::vector<int> c(world, per_rank);
  if (world > 1) c[0] = std::max(1, std::min(per_rank, (int)std::lround(per_rank * coord_weight)));
  return c;
}

Runner::Runner(std::unique_ptr<Worker> w, std::unique_ptr<Comm> in, std::unique_ptr<Comm> out, int world, int rank,
               std::vector<int> counts, bool scatter, size_t image_bytes, int timeout_ms, int slots)
    : w_(std::move(w)), in_(std::move(in)), out_(std::move(out)), world_(world), rank_(rank),
      counts_(std::move(counts)), scatter_(scatter), ib_(image_bytes), timeout_ms_(timeout_ms) {
  if ((int)counts_.size() != world_) throw std::invalid_argument("dp::Runner: one count per rank");
  max_ = 0;
  for (int c : counts_) {
    if (c < 0) throw std::invalid_argument("dp::Runner: negative count");
    max_ = std::max(max_, c);
  }
  if (max_ < 1) throw std::invalid_argument("dp::Runner: empty step");
  // Steps in flight (slots). Step i reuses slot i - slots, so its forward
  // waits for that step's answers to have left; with slots = 2 that was the
  // step just before on the same lane, and the answer copy's latency sat
  // between a lane's consecutive forwards (bench: 268k vs 276k img/s with 4
  // slots, the bare two-lane loop 276.7k: tools/pipeline_probe.py).
  if (slots <= 0) slots = 2 * std::max(2, w_->lanes());
  r_ = std::make_unique<Rank>(w_.get(), max_, ib_, scatter_, slots);
  if (world_ > 1) {
    if (!in_ || !out_ || in_->size() != world_ || in_->rank() != rank_)
      throw std::invalid_argument("dp::Runner: communicators do not match world/rank");
    r_->attach(in_.get(), out_.get());
  } else {
    r_->attach(nullptr, nullptr);
  }
}

Runner::~Runner() {
  r_.reset();
  w_->sync_all_noexcept();
  in_.reset();
  out_.reset();
  w_.reset();
}

int64_t Runner::global_batch() const { return std::accumulate(counts_.begin(), counts_.end(), (int64_t)0); }

PipelineResult Runner::run(const uint8_t* pool, int64_t pool_images, int64_t first, int64_t n, bool pipelined) {
  const int64_t G = global_batch();
  const int64_t per = scatter_ ? G : max_;  // pool stride of one step's images
  const bool has_pool = scatter_ ? rank_ == 0 : true;
  if (has_pool && (!pool || pool_images < (scatter_ ? G : counts_[rank_])))
    throw std::invalid_argument("dp::Runner::run: pool smaller than one batch");
  const int64_t nb = has_pool ? std::max<int64_t>(1, pool_images / per) : 1;
  auto plan = [&](int64_t step, const Rank&) {
    StepPlan p;
    p.step = step;
    p.counts = counts_;
    p.src = has_pool ? pool + (size_t)((step % nb) * per) * ib_ : nullptr;
    return p;
  };
  auto on_result = [&](const StepPlan& p, const int32_t* i, const float* pr) {
    last_idx_.assign(i, i + G);
    last_prob_.assign(pr, pr + G);
    if (hook_) hook_(p.step, i, pr, G);
  };
  return run_pipeline({r_.get()}, first, n, plan, on_result, timeout_ms_, pipelined);
}

void Runner::set_counts(const std::vector<int>& counts) {
  if ((int)counts.size() != world_) throw std::invalid_argument("dp::Runner::set_counts: one count per rank");
  int64_t total = 0;
  for (int c : counts) {
    if (c < 0 || c > max_) throw std::invalid_argument("dp::Runner::set_counts: count outside [0, max_per_rank]");
    total += c;
  }
  if (total < 1) throw std::invalid_argument("dp::Runner::set_counts: empty step");
  counts_ = counts;
}

Runner::Calibration Runner::calibrate(const uint8_t* pool, int64_t pool_images, int64_t first, int64_t steps,
                                      int rounds, double tol, const AllGather& allgather, double min_weight) {
  Calibration out;
  if (world_ < 2 || !scatter_ || steps < 1 || rounds < 1) {
    out.weight = world_ > 1 ? (double)counts_[0] / counts_[1] : 1.0;
    return out;
  }
  const int per = counts_[1];
  double w = (double)counts_[0] / per;
  for (int k = 0; k < rounds; ++k) {
    const PipelineResult res = run(pool, pool_images, first + out.steps, steps);
    out.steps += steps;
    const std::vector<double> b = allgather(res.busy_ms);
    if ((int)b.size() != world_) throw std::runtime_error("dp::Runner::calibrate: all-gather returned the wrong size");
    CalibRound r;
    r.weight = w;
    r.busy_coord = b[0];
    for (int i = 1; i < world_; ++i) r.busy_worker = std::max(r.busy_worker, b[i]);
    r.coord_count = counts_[0];
    r.per_rank = per;
    r.world = world_;
    out.rounds.push_back(r);
    if (r.busy_worker > 0.0 && std::fabs(r.busy_coord / r.busy_worker - 1.0) <= tol) break;
    const double nw = next_coord_weight(r, min_weight);
    if (weighted_counts(per, world_, nw) == counts_) break;  // the count would not change
    w = nw;
    set_counts(weighted_counts(per, world_, w));
  }
  out.weight = best_coord_weight(out.rounds);
  set_counts(weighted_counts(per, world_, out.weight));
  return out;
}

void Runner::stage(const uint8_t* src, uint8_t* dst) {
  w_->activate();
  const size_t mine = (size_t)counts_[rank_] * ib_;
  if (rank_ == 0 && mine) w_->copy(dst, src, mine, Worker::kIn);
  if (world_ > 1) {
    in_->group_start();
    try {
      if (rank_ == 0) {
        size_t off = (size_t)counts_[0] * ib_;
        for (int r = 1; r < world_; ++r) {
          const size_t b = (size_t)counts_[r] * ib_;
          if (b) in_->send(src + off, b, r, w_->stream(Worker::kIn));
          off += b;
        }
      } else if (mine) {
        in_->recv(dst, mine, 0, w_->stream(Worker::kIn));
      }
    } catch (...) {
      in_->group_end();
      throw;
    }
    in_->group_end();
  }
  w_->sync_all();
}

}  // namespace dp
}  // namespace dmlc
