#include "dp.h"

#include <map>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <mutex>
#include <cstdlib>
#include <cstring>
#include <thread>

namespace dmlc {
namespace dp {

// ------------------------------------------------------------------ host worker
namespace {

class HostWorker : public Worker {
 public:
  HostWorker(int device, int H, int W, int classes, int lanes, uint32_t seed, int delay_us, int us_per_image,
             int extra_us)
      : device_(device), bytes_((size_t)H * W * 3), classes_(classes), lanes_(std::max(1, lanes)),
        delay_us_(delay_us), us_per_image_(us_per_image), extra_us_(extra_us), busy_(lanes_) {
    for (auto& b : busy_) b = false;
    std::memcpy(arena_, &seed, 4);
  }
  ~HostWorker() override {
    for (void* p : live_) std::free(p);
  }
  int device() const override { return device_; }
  void* alloc(size_t bytes) override { return track(std::calloc(1, std::max<size_t>(bytes, 1))); }
  void dealloc(void* p) override { untrack(p); }
  void* alloc_host(size_t bytes) override { return alloc(bytes); }
  void dealloc_host(void* p) override { untrack(p); }
  Stream stream(int) override { return nullptr; }
  int new_event() override {
    std::lock_guard<std::mutex> g(mu_);
    stamps_.emplace_back();
    return n_events_++;
  }
  // synchronous "streams" with a synthetic device clock per stream: a
  // forward advances its compute stream's clock by its modelled cost
  // (delay_us + us_per_image * B + extra_us) and an event reads the clock of
  // the stream it is recorded on, so elapsed_ms() around a forward is exactly
  // that cost, whatever the host's sleep and wake-up jitter (the forward
  // still sleeps for it, so the protocol's real-time overlap is exercised).
  // The coordinator calibration that reads these times is then deterministic
  // (its tests used to assert on wall-clock stamps).
  void record(int ev, int stream) override {
    std::lock_guard<std::mutex> g(mu_);
    stamps_.at(ev) = clock_us_[stream];
  }
  double elapsed_ms(int a, int b) override {
    std::lock_guard<std::mutex> g(mu_);
    return (double)(stamps_.at(b) - stamps_.at(a)) / 1000.0;
  }
  void wait(int, int) override {}
  bool query(int) override { return true; }
  void sync(int) override {}
  void sync_all() override {}
  int lanes() const override { return lanes_; }
  void classify(const uint8_t* images, int B, int32_t* idx, float* prob, int lane) override {
    if (!healthy_) throw comm::CommError("host worker " + std::to_string(device_) + ": device lost");
    if (lane < 0 || lane >= lanes_) throw std::invalid_argument("host worker: no such lane");
    // a lane runs one forward at a time (a stream): concurrent use is a bug
    if (busy_[lane].exchange(true)) throw std::logic_error("host worker: lane used concurrently");
    uint32_t w;
    std::memcpy(&w, arena_, 4);
    const int64_t us = delay_us_ + (int64_t)us_per_image_ * B + extra_us_;
    if (us > 0) std::this_thread::sleep_for(std::chrono::microseconds(us));
    {
      std::lock_guard<std::mutex> g(mu_);
      clock_us_[compute_stream(lane)] += us;
    }
    for (int b = 0; b < B; ++b) {
      const uint8_t* img = images + (size_t)b * bytes_;
      idx[b] = (int32_t)(((uint64_t)host_class_of(img, bytes_, 1 << 30) + w) % (uint64_t)classes_);
      prob[b] = host_prob_of(img);
    }
    busy_[lane] = false;
  }
  void copy_d2h(void* dst, const void* src, size_t bytes, int) override { std::memmove(dst, src, bytes); }
  void copy(void* dst, const void* src, size_t bytes, int) override { std::memmove(dst, src, bytes); }
  bool healthy() override { return healthy_; }
  void* weight_arena() override { return arena_; }
  size_t weight_bytes() const override { return sizeof(arena_); }
  std::atomic<bool> healthy_{true};

 private:
  void* track(void* p) {
    if (!p) throw std::bad_alloc();
    std::lock_guard<std::mutex> g(mu_);
    live_.push_back(p);
    return p;
  }
  void untrack(void* p) {
    std::lock_guard<std::mutex> g(mu_);
    auto it = std::find(live_.begin(), live_.end(), p);
    if (it != live_.end()) {
      std::free(p);
      live_.erase(it);
    }
  }
  int device_;
  size_t bytes_;
  int classes_, lanes_, delay_us_, us_per_image_, extra_us_;
  std::vector<std::atomic<bool>> busy_;
  uint8_t arena_[16] = {};
  int n_events_ = 0;
  std::vector<int64_t> stamps_;             // synthetic µs, per event
  std::map<int, int64_t> clock_us_;         // synthetic µs, per stream
  std::mutex mu_;
  std::vector<void*> live_;
};

}  // namespace

std::unique_ptr<Worker> make_host_worker(int device, int H, int W, int classes, int lanes, uint32_t seed,
                                         int delay_us, int us_per_image, int extra_us) {
  return std::make_unique<HostWorker>(device, H, W, classes, lanes, seed, delay_us, us_per_image, extra_us);
}

void host_worker_set_healthy(Worker& w, bool healthy) {
  auto* h = dynamic_cast<HostWorker*>(&w);
  if (!h) throw std::invalid_argument("host_worker_set_healthy: not a host worker");
  h->healthy_ = healthy;
}

int host_class_of(const uint8_t* img, size_t bytes, int classes) {
  uint64_t s = 0;
  for (size_t i = 0; i < bytes; ++i) s += img[i];
  return (int)(s % (uint64_t)classes);
}

float host_prob_of(const uint8_t* img) { return (img[0] + 1) / 257.f; }

double CalibRound::rate() const {
  const double pace = std::max(busy_coord, busy_worker);
  const double images = coord_count + (double)per_rank * (world - 1);
  return pace > 0.0 ? images / pace : 0.0;
}

double next_coord_weight(const CalibRound& r, double min_weight) {
  if (!(r.busy_coord > 0.0) || !(r.busy_worker > 0.0)) return r.weight;
  const double w = r.weight * r.busy_worker / r.busy_coord;
  return std::max(min_weight, std::min(1.0, w));
}

double best_coord_weight(const std::vector<CalibRound>& rounds) {
  double best = 1.0, rate = -1.0;
  for (const auto& r : rounds) {
    const double x = r.rate();
    if (x > rate * 1.0005 || (x >= rate * 0.9995 && r.weight > best)) {
      rate = std::max(rate, x);
      best = r.weight;
    }
  }
  return best;
}

std::vector<int> weighted_shards(int64_t n, int world, int cap, double w0) {
  if (world <= 1 || w0 >= 1.0) return shard_counts(n, world, cap);
  if (!(w0 > 0.0)) throw std::invalid_argument("weighted_shards: w0 must be in (0, 1]");
  const int cap0 = std::max(1, std::min(cap, (int)std::lround(cap * w0)));
  const int64_t room = (int64_t)cap0 + (int64_t)cap * (world - 1);
  if (n < 0 || n > room) throw std::invalid_argument("weighted_shards: n exceeds the step's capacity");
  int64_t c0 = std::min<int64_t>(cap0, std::llround((double)n * w0 / (w0 + world - 1)));
  int64_t rest = n - c0;
  if (rest > (int64_t)cap * (world - 1)) {  // the others are full: the coordinator takes the overflow
    c0 += rest - (int64_t)cap * (world - 1);
    rest = (int64_t)cap * (world - 1);
  }
  std::vector<int> out{(int)c0};
  for (int c : shard_counts(rest, world - 1, cap)) out.push_back(c);
  return out;
}

std::vector<int> shard_counts(int64_t n, int world, int cap) {
  if (world < 1) throw std::invalid_argument("shard_counts: world < 1");
  if (n < 0 || n > (int64_t)world * cap) throw std::invalid_argument("shard_counts: n exceeds world * cap");
  std::vector<int> c(world, (int)(n / world));
  for (int r = 0; r < (int)(n % world); ++r) ++c[r];
  return c;
}

// ------------------------------------------------------------------ rank
Rank::Rank(Worker* w, int max_per_rank, size_t image_bytes, bool scatter, int slots)
    : w_(w), max_(max_per_rank), slots_(slots), ib_(image_bytes), scatter_(scatter) {
  if (max_ < 1 || slots_ < 2) throw std::invalid_argument("dp::Rank: need max_per_rank >= 1 and slots >= 2");
  w_->activate();
  for (int s = 0; s < slots_; ++s) {
    ev_in_.push_back(w_->new_event());
    ev_comp_.push_back(w_->new_event());
    ev_out_.push_back(w_->new_event());
    ev_t0_.push_back(w_->new_timing_event());
    ev_t1_.push_back(w_->new_timing_event());
  }
  slot_n_.assign(slots_, -1);
  inbuf_.assign(slots_, nullptr);
  ans_.assign(slots_, nullptr);
  host_ans_.assign(slots_, nullptr);
  reset();
}

Rank::~Rank() {
  // teardown never throws: the device may be the lost one
  try {
    w_->activate();
  } catch (...) {
  }
  w_->sync_all_noexcept();
  for (void* p : inbuf_)
    if (p) w_->dealloc(p);
  for (void* p : ans_)
    if (p) w_->dealloc(p);
  for (void* p : host_ans_)
    if (p) w_->dealloc_host(p);
}

void Rank::reset() {
  in_used_.assign(slots_, false);
  out_used_.assign(slots_, false);
  slot_n_.assign(slots_, -1);
}

void Rank::attach(Comm* in, Comm* out) {
  if ((in == nullptr) != (out == nullptr)) throw std::invalid_argument("dp::Rank::attach: both or no comms");
  if (in && (in->size() != out->size() || in->rank() != out->rank()))
    throw std::invalid_argument("dp::Rank::attach: shard and answer communicators disagree");
  w_->activate();
  w_->sync_all();  // nothing of the old binding may still be in flight
  in_ = in;
  out_ = out;
  reset();
  const int world = this->world();
  if (scatter_ && !root()) {
    for (auto& p : inbuf_)
      if (!p) p = w_->alloc((size_t)max_ * ib_);
  }
  const int blocks = root() ? world : 1;
  if (blocks > ans_world_) {
    for (auto& p : ans_) {
      if (p) w_->dealloc(p);
      p = w_->alloc((size_t)blocks * block_bytes());
    }
    for (auto& p : host_ans_) {
      if (p) w_->dealloc_host(p);
      p = root() ? w_->alloc_host((size_t)blocks * block_bytes()) : nullptr;
    }
    ans_world_ = blocks;
  }
  if (root())
    for (auto& p : host_ans_)
      if (!p) p = w_->alloc_host((size_t)ans_world_ * block_bytes());
}

void Rank::settle_busy() {
  for (int s = 0; s < slots_; ++s)
    if (slot_n_[s] > 0 && w_->query(ev_t1_[s])) {
      busy_ms_ += w_->elapsed_ms(ev_t0_[s], ev_t1_[s]);
      ++busy_steps_;
      busy_images_ += slot_n_[s];
      slot_n_[s] = -1;
    }
}

void Rank::post_input(const StepPlan& p) {
  if (!scatter_ || world() == 1) return;
  const int s = slot(p);
  if (root()) {
    if (p.src_event >= 0) w_->wait(Worker::kIn, p.src_event);
    size_t off = (size_t)p.counts[0];
    for (int r = 1; r < world(); ++r) {
      if (p.counts[r] > 0) in_->send(p.src + off * ib_, (size_t)p.counts[r] * ib_, r, w_->stream(Worker::kIn));
      off += (size_t)p.counts[r];
    }
  } else {
    if (in_used_[s]) w_->wait(Worker::kIn, ev_comp_[s]);  // compute(step - slots) has read this slot
    const int n = p.counts[rank()];
    if (n > 0) in_->recv(inbuf_[s], (size_t)n * ib_, 0, w_->stream(Worker::kIn));
  }
}

void Rank::after_input(const StepPlan& p) {
  if (!scatter_ || world() == 1 || root()) return;
  w_->record(ev_in_[slot(p)], Worker::kIn);
}

void Rank::compute(const StepPlan& p) {
  const int s = slot(p);
  const int n = p.counts.at(rank());
  if (n > max_) throw std::invalid_argument("dp::Rank::compute: shard larger than max_per_rank");
  const bool received = scatter_ && !root() && world() > 1;
  const uint8_t* img = received ? (const uint8_t*)inbuf_[s] : p.src;
  // consecutive steps alternate over the worker's compute lanes (whatever the
  // slot count)
  const int lane = (int)(p.step % w_->lanes());
  const int cs = Worker::compute_stream(lane);
  if (received) w_->wait(cs, ev_in_[s]);
  else if (root() && p.src_event >= 0) w_->wait(cs, p.src_event);
  if (out_used_[s]) w_->wait(cs, ev_out_[s]);  // gather(step - slots) has read the answers
  auto* blk = (uint8_t*)ans_[s];
  if (n > 0) {
    if (!img) throw std::invalid_argument("dp::Rank::compute: no images for this rank");
    w_->record(ev_t0_[s], cs);
    w_->classify(img, n, (int32_t*)blk, (float*)(blk + (size_t)max_ * 4), lane);
    w_->record(ev_t1_[s], cs);
  }
  slot_n_[s] = n > 0 ? n : -1;
  w_->record(ev_comp_[s], cs);
  in_used_[s] = true;
}

void Rank::post_output(const StepPlan& p) {
  const int s = slot(p);
  w_->wait(Worker::kOut, ev_comp_[s]);
  if (world() == 1) return;
  if (root()) {
    for (int r = 1; r < world(); ++r)
      if (p.counts[r] > 0)
        out_->recv((uint8_t*)ans_[s] + (size_t)r * block_bytes(), block_bytes(), r, w_->stream(Worker::kOut));
  } else if (p.counts[rank()] > 0) {
    out_->send(ans_[s], block_bytes(), 0, w_->stream(Worker::kOut));
  }
}

void Rank::after_output(const StepPlan& p) {
  const int s = slot(p);
  if (root()) w_->copy_d2h(host_ans_[s], ans_[s], (size_t)world() * block_bytes(), Worker::kOut);
  w_->record(ev_out_[s], Worker::kOut);
  out_used_[s] = true;
}

void Rank::wait_step(const StepPlan& p, int timeout_ms) {
  const int s = slot(p);
  const auto t0 = std::chrono::steady_clock::now();
  int spins = 0;
  while (!w_->query(ev_out_[s])) {
    if ((in_ && !in_->ok()) || (out_ && !out_->ok())) throw comm::CommError("dp: communicator error while waiting");
    if (timeout_ms >= 0 &&
        std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(timeout_ms))
      throw comm::CommError("dp: step " + std::to_string(p.step) + " timed out");
    if (++spins > 64) std::this_thread::sleep_for(std::chrono::microseconds(20));
  }
  if (slot_n_[s] > 0) {  // the step's forward is complete: account its time
    busy_ms_ += w_->elapsed_ms(ev_t0_[s], ev_t1_[s]);
    ++busy_steps_;
    busy_images_ += slot_n_[s];
    slot_n_[s] = -1;
  }
}

void Rank::collect(const StepPlan& p, int32_t* idx, float* prob, int timeout_ms) {
  if (!root()) throw std::logic_error("dp::Rank::collect on a non-coordinator rank");
  wait_step(p, timeout_ms);
  const int s = slot(p);
  const auto* h = (const uint8_t*)host_ans_[s];
  size_t off = 0;
  for (int r = 0; r < world(); ++r) {
    const int n = p.counts[r];
    const auto* blk = h + (size_t)r * block_bytes();
    if (n > 0) {
      std::memcpy(idx + off, blk, (size_t)n * 4);
      std::memcpy(prob + off, blk + (size_t)max_ * 4, (size_t)n * 4);
    }
    off += (size_t)n;
  }
}

// ------------------------------------------------------------------ pipeline
PipelineResult run_pipeline(const std::vector<Rank*>& ranks, int64_t first, int64_t n, const PlanFn& plan,
                            const ResultFn& on_result, int timeout_ms, bool pipelined) {
  PipelineResult res;
  if (n <= 0 || ranks.empty()) return res;
  Rank* timed = ranks.front();
  const double busy0 = timed->busy_ms();
  const int64_t bsteps0 = timed->busy_steps();
  auto busy_mean = [&]() {
    const int64_t k = timed->busy_steps() - bsteps0;
    return k > 0 ? (timed->busy_ms() - busy0) / (double)k : 0.0;
  };
  Comm* gcomm = ranks.front()->comm_in();  // null for a world of one
  size_t root_i = ranks.size();
  for (size_t i = 0; i < ranks.size(); ++i)
    if (ranks[i]->root()) root_i = i;

  // plans of the steps in flight (at most slots + 1)
  std::vector<std::pair<int64_t, std::vector<StepPlan>>> live;
  auto plans_of = [&](int64_t step) -> std::vector<StepPlan>& {
    for (auto& kv : live)
      if (kv.first == step) return kv.second;
    std::vector<StepPlan> ps;
    ps.reserve(ranks.size());
    for (Rank* r : ranks) ps.push_back(plan(step, *r));  // may throw: nothing of the step is posted yet
    live.emplace_back(step, std::move(ps));
    return live.back().second;
  };
  auto drop = [&](int64_t step) {
    live.erase(std::remove_if(live.begin(), live.end(), [&](const auto& kv) { return kv.first == step; }),
               live.end());
  };
  // Groups are thread-wide in both backends: bracketing through one rank's
  // communicator groups the operations of every rank this thread drives.
  auto phase = [&](const std::vector<StepPlan>& ps, bool input) {
    if (gcomm) gcomm->group_start();
    try {
      for (size_t i = 0; i < ranks.size(); ++i) input ? ranks[i]->post_input(ps[i]) : ranks[i]->post_output(ps[i]);
    } catch (...) {
      if (gcomm) gcomm->group_end();
      throw;
    }
    if (gcomm) gcomm->group_end();
    for (size_t i = 0; i < ranks.size(); ++i) input ? ranks[i]->after_input(ps[i]) : ranks[i]->after_output(ps[i]);
  };

  std::vector<int32_t> idx;
  std::vector<float> prob;
  auto finish = [&](int64_t step) {
    auto& ps = plans_of(step);
    if (root_i < ranks.size()) {
      const auto& p = ps[root_i];
      int64_t total = 0;
      for (int c : p.counts) total += c;
      idx.resize((size_t)total);
      prob.resize((size_t)total);
      ranks[root_i]->collect(p, idx.data(), prob.data(), timeout_ms);
      res.images += total;
      if (on_result) on_result(p, idx.data(), prob.data());
    } else {
      ranks.front()->wait_step(ps.front(), timeout_ms);  // keep the host one step ahead at most
    }
    ++res.steps;
    drop(step);
  };

  const int64_t end = first + n;
  if (!pipelined) {  // latency mode: one step in flight
    for (int64_t i = first; i < end; ++i) {
      const auto t0 = std::chrono::steady_clock::now();
      auto& ps = plans_of(i);
      phase(ps, true);
      for (size_t k = 0; k < ranks.size(); ++k) ranks[k]->compute(ps[k]);
      phase(ps, false);
      finish(i);
      res.step_ms.push_back(std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
    }
    res.busy_ms = busy_mean();
    return res;
  }
  // steps in flight = the ranks' slot count (2: the host collects step i-1
  // after issuing step i)
  const int64_t depth = ranks.front()->slots();
  phase(plans_of(first), true);
  for (int64_t i = first; i < end; ++i) {
    if (i + 1 < end) phase(plans_of(i + 1), true);
    auto& ps = plans_of(i);
    for (size_t k = 0; k < ranks.size(); ++k) ranks[k]->compute(ps[k]);
    phase(ps, false);
    if (i - first >= depth - 1) finish(i - (depth - 1));
  }
  for (int64_t j = std::max(first, end - (depth - 1)); j < end; ++j) finish(j);
  res.busy_ms = busy_mean();
  return res;
}

// ------------------------------------------------------------------ group

namespace {
// Thrown by the plan function when fault injection drops a member: nothing
// of the step being planned has been posted yet.
struct MemberLost {
  int member;
};
}  // namespace

Group::Group(std::vector<Worker*> workers, CommFactory make_comms, int max_per_rank, size_t image_bytes,
             int timeout_ms)
    : workers_(std::move(workers)), make_comms_(std::move(make_comms)), max_(max_per_rank), ib_(image_bytes),
      timeout_ms_(timeout_ms) {
  if (workers_.empty()) throw std::invalid_argument("dp::Group: no workers");
  lost_.assign(workers_.size(), false);
  killed_.assign(workers_.size(), false);
  fail_at_.assign(workers_.size(), -1);
  fail_abrupt_.assign(workers_.size(), false);
  for (size_t i = 0; i < workers_.size(); ++i) {
    members_.push_back((int)i);
    ranks_.push_back(std::make_unique<Rank>(workers_[i], max_, ib_, /*scatter=*/true));
  }
  rebuild();
}

Group::~Group() {
  // a lost member is skipped (its device may not answer), and nothing here
  // throws: the group is torn down after a GPU loss (fleet rebalance, hot swap)
  for (size_t i = 0; i < ranks_.size(); ++i)
    if (!lost_[i]) ranks_[i]->worker()->sync_all_noexcept();
  ranks_.clear();
  cin_.clear();
  cout_.clear();
}

void Group::rebuild() {
  cin_.clear();
  cout_.clear();
  if (members_.size() > 1) {
    cin_ = make_comms_(members_);
    cout_ = make_comms_(members_);
    if (cin_.size() != members_.size() || cout_.size() != members_.size())
      throw std::runtime_error("dp::Group: communicator factory returned the wrong number of ranks");
  }
  for (size_t i = 0; i < members_.size(); ++i) {
    Rank& r = *ranks_[members_[i]];
    if (members_.size() > 1) r.attach(cin_[i].get(), cout_[i].get());
    else r.attach(nullptr, nullptr);
  }
}

void Group::fail(int m, int64_t after_steps, bool abrupt) {
  if (m <= 0 || m >= (int)workers_.size()) throw std::invalid_argument("dp::Group::fail: bad member (0 is the coordinator)");
  fail_at_[m] = std::max<int64_t>(0, after_steps);
  fail_abrupt_[m] = abrupt;
}

void Group::kill_now(int m) {
  if (m <= 0 || m >= (int)workers_.size()) throw std::invalid_argument("dp::Group::kill_now: bad member");
  auto it = std::find(members_.begin(), members_.end(), m);
  if (it == members_.end()) return;
  // (a host worker also fails its forwards; a HIP worker on the device
  // loopback loses only its communicator operations)
  if (dynamic_cast<HostWorker*>(workers_[m])) host_worker_set_healthy(*workers_[m], false);
  killed_[m] = true;
  const int rank = (int)(it - members_.begin());
  if (!cin_.empty()) {
    comm::host_kill(*cin_[0], rank);
    comm::host_kill(*cout_[0], rank);
  }
}

void Group::set_coord_weight(double w, bool auto_balance) {
  if (!(w > 0.0) || w > 1.0) throw std::invalid_argument("dp::Group: coord_weight must be in (0, 1]");
  coord_weight_ = w;
  auto_balance_ = auto_balance;
}

// Per-image forward time of the coordinator vs the slowest other rank over
// the last run: the weight that equalises them under a time ~ images model,
// half-way from the current one (serving batches vary; a step's fixed costs
// are not linear in its images).
void Group::rebalance_coord(const std::vector<Rank*>& rs) {
  for (Rank* r : rs) r->settle_busy();
  auto per_image = [](const Rank* r) {
    return r->busy_images() > 0 ? r->busy_ms() / (double)r->busy_images() : 0.0;
  };
  const double t0 = per_image(rs.front());
  double tw = 0.0;
  for (size_t i = 1; i < rs.size(); ++i) tw = std::max(tw, per_image(rs[i]));
  if (t0 > 0.0 && tw > 0.0) {
    const double target = std::max(0.5, std::min(1.0, tw / t0));
    coord_weight_ = std::max(0.5, std::min(1.0, 0.5 * coord_weight_ + 0.5 * target));
  }
  for (Rank* r : rs) r->reset_busy();
}

Group::Stats Group::classify(const uint8_t* src, int64_t n, int32_t* idx, float* prob, int src_event,
                             int32_t* commit_count) {
  Stats st;
  st.per_worker.assign(workers_.size(), 0);
  int64_t committed = 0;  // answers [0, committed) are final
  int64_t issued = 0;     // images whose step was planned (posted) in the current attempt
  while (committed < n) {
    const int world = (int)members_.size();
    const double w0 = world > 1 ? coord_weight_ : 1.0;
    const int64_t G = (int64_t)max_ * (world - 1) + std::max(1, std::min(max_, (int)std::lround(max_ * w0)));
    const int64_t base = committed;
    const int64_t steps = (n - base + G - 1) / G;
    issued = base;
    std::vector<Rank*> rs;
    for (int m : members_) rs.push_back(ranks_[m].get());
    auto plan = [&](int64_t step, const Rank& r) {
      if (&r == rs.front()) {  // once per step, before anything of it is posted
        for (int m : members_) {
          if (fail_at_[m] == 0) {
            fail_at_[m] = -1;
            if (!fail_abrupt_[m]) throw MemberLost{m};
            kill_now(m);  // this step's operations with m fail
          } else if (fail_at_[m] > 0) {
            --fail_at_[m];
          }
        }
        issued = std::min<int64_t>(n, base + (step + 1) * G);
      }
      StepPlan p;
      p.step = step;
      const int64_t start = base + step * G;
      const int64_t nstep = std::min<int64_t>(G, n - start);
      // as many ranks as can each take min_per_rank images (at least enough
      // to stay under max_ per rank)
      const int64_t want = std::max<int64_t>(nstep / min_per_rank_, (nstep + max_ - 1) / max_);
      const int used = (int)std::min<int64_t>(world, std::max<int64_t>(1, want));
      // (with fewer ranks than the group, the step may not fit their caps
      // weighted: an even split then)
      const bool weighted = used == world && w0 < 1.0;
      p.counts = weighted ? weighted_shards(nstep, used, max_, w0) : shard_counts(nstep, used, max_);
      p.counts.resize(world, 0);
      p.src = src + (size_t)start * ib_;
      p.src_event = r.root() ? src_event : -1;
      return p;
    };
    auto on_result = [&](const StepPlan& p, const int32_t* i, const float* pr) {
      const int64_t start = base + p.step * G;
      int64_t total = 0;
      for (int c : p.counts) total += c;
      std::memcpy(idx + start, i, (size_t)total * 4);
      std::memcpy(prob + start, pr, (size_t)total * 4);
      if (commit_count)
        for (int64_t k = 0; k < total; ++k) ++commit_count[start + k];
      int used = 0;
      for (size_t i = 0; i < p.counts.size() && i < members_.size(); ++i) {
        st.per_worker[members_[i]] += p.counts[i];
        used += p.counts[i] > 0;
      }
      st.ranks_used = std::max(st.ranks_used, used);
      committed = start + total;
      ++st.steps;
    };
    std::vector<int> lost;
    try {
      run_pipeline(rs, 0, steps, plan, on_result, timeout_ms_);
      if (auto_balance_ && world > 1 && steps >= 2) rebalance_coord(rs);
      break;
    } catch (const MemberLost& e) {
      // injected: the GPU is in fact fine, so everything already posted
      // completes; drain it, then drop the member
      for (int m : members_) workers_[m]->sync_all();
      lost.push_back(e.member);
    } catch (const comm::CommError&) {
      for (int m : members_)
        if (!workers_[m]->healthy() || killed_[m]) lost.push_back(m);
      if (lost.empty()) throw;  // not attributable to a lost GPU
    }
    if (std::find(lost.begin(), lost.end(), members_.front()) != lost.end())
      throw comm::CommError("dp::Group: the coordinator GPU was lost");
    // abort the broken communicators (RCCL: also ends kernels blocked on
    // the lost peer), then rebuild over the survivors
    for (auto& c : cin_) c->abort();
    for (auto& c : cout_) c->abort();
    for (int m : members_)
      if (std::find(lost.begin(), lost.end(), m) == lost.end()) workers_[m]->sync_all();
      else if (killed_[m]) workers_[m]->sync_all_noexcept();  // a killed HIP worker's GPU is fine: drain it
    for (int m : lost) lost_[m] = true;
    members_.erase(std::remove_if(members_.begin(), members_.end(), [&](int m) { return lost_[m]; }),
                   members_.end());
    ++st.recoveries;
    st.redone_images += issued - committed;
    rebuild();
  }
  st.images = n;
  return st;
}

}  // namespace dp
}  // namespace dmlc
