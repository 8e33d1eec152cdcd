// Python bindings of the native data-parallel layer (csrc/comm):
//   rccl_unique_id()   bytes for bootstrapping a multi-process communicator
//   DpRunner           one rank of a multi-process job (bench.py: one
//                      process per GPU, RCCL over xGMI)
//   DpGroup            one process owning several GPUs (single-process
//                      multi-GPU serving, elastic on GPU loss)
//   dp_host_run        the same protocol over the host fake (CPU tests:
//                      shard order, exactly-once answers, rank loss)
#include <hip/hip_runtime.h>
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <thread>
#include <vector>

#include "../comm/comm.h"
#include "../comm/dp.h"
#include "../comm/fleet.h"
#include "../comm/runner.h"
#include <atomic>
#include <map>
#include <mutex>
#include <set>
#include <tuple>
#include "../runtime/engine.h"

namespace py = pybind11;
using namespace dmlc;

namespace {

// ------------------------------------------------------------------ runner
// bench.py's rank (csrc/comm/runner.h) on the HIP engine and RCCL.
class DpRunner {
 public:
  DpRunner(Engine* e, int world, int rank, const std::string& id_in, const std::string& id_out, int max_per_rank,
           bool scatter, int image_size, bool use_graph, int timeout_ms, int lanes, int slots, double coord_weight,
           std::vector<int> counts)
      : S_(image_size) {
    if (lanes < 1 || lanes > dp::Worker::kMaxLanes) throw std::invalid_argument("DpRunner: lanes must be 1..4");
    if (counts.empty()) counts = dp::weighted_counts(max_per_rank, world, coord_weight);
    int mx = 0;
    for (int c : counts) mx = std::max(mx, c);
    e->reserve(mx);
    std::vector<Engine*> more;
    for (int l = 1; l < lanes; ++l) {  // further instances of the model: consecutive steps overlap
      lanes_.push_back(std::make_unique<Engine>(*e, e->device()));
      lanes_.back()->copy_weights_from(*e);
      lanes_.back()->reserve(std::max(e->max_batch(), mx));
      more.push_back(lanes_.back().get());
    }
    std::unique_ptr<comm::Comm> cin, cout;
    if (world > 1) {
      cin = comm::rccl_init_rank(id_in, world, rank, e->device());
      // answers: 8 B per image, one CTA (comm::rccl_init_rank's max_ctas)
      cout = comm::rccl_init_rank(id_out, world, rank, e->device(), 1);
    }
    r_ = std::make_unique<dp::Runner>(dp::make_hip_worker(e, S_, S_, use_graph, more), std::move(cin),
                                      std::move(cout), world, rank, counts, scatter, (size_t)S_ * S_ * 3, timeout_ms,
                                      slots);
  }
  // bench.py --dry-run: the same rank on a host worker (a classify of B
  // images takes B x us_per_image (+ extra_us on the coordinator, the modelled
  // cost of its scatter legs) of synthetic device time, csrc/comm/dp.h) and
  // the cross-process socket communicator (comm::socket_init_rank), one
  // process per rank exactly as on the GPUs.
  DpRunner(int world, int rank, const std::string& id_in, const std::string& id_out, int max_per_rank, bool scatter,
           int image_size, int timeout_ms, int lanes, int slots, double coord_weight, int us_per_image,
           int coord_extra_us)
      : S_(image_size) {
    if (lanes < 1 || lanes > dp::Worker::kMaxLanes) throw std::invalid_argument("DpRunner: lanes must be 1..4");
    const auto counts = dp::weighted_counts(max_per_rank, world, coord_weight);
    std::unique_ptr<comm::Comm> cin, cout;
    if (world > 1) {
      const int to = timeout_ms > 0 ? timeout_ms : 20000;
      cin = comm::socket_init_rank(id_in, world, rank, to);
      cout = comm::socket_init_rank(id_out, world, rank, to);
    }
    r_ = std::make_unique<dp::Runner>(
        dp::make_host_worker(rank, S_, S_, 1000, lanes, 0, 0, us_per_image, rank == 0 ? coord_extra_us : 0),
        std::move(cin), std::move(cout), world, rank, counts, scatter, (size_t)S_ * S_ * 3, timeout_ms, slots);
  }
  ~DpRunner() {
    r_.reset();
    lanes_.clear();
  }
  py::dict run(uintptr_t pool, int64_t pool_images, int64_t first, int64_t n, bool pipelined) {
    dp::PipelineResult res;
    {
      py::gil_scoped_release nogil;
      res = r_->run((const uint8_t*)pool, pool_images, first, n, pipelined);
    }
    py::dict d;
    d["steps"] = res.steps;
    d["images"] = res.images;
    d["step_ms"] = res.step_ms;
    d["busy_ms"] = res.busy_ms;
    return d;
  }
  void set_counts(const std::vector<int>& c) { r_->set_counts(c); }
  // allgather: Python callable, float -> list of every rank's float (bench.py:
  // torch.distributed over gloo); called with the GIL held
  py::dict calibrate(uintptr_t pool, int64_t pool_images, int64_t first, int64_t steps, int rounds, double tol,
                     py::function allgather, double min_weight) {
    dp::Runner::AllGather ag = [&allgather](double x) {
      py::gil_scoped_acquire gil;
      return allgather(x).cast<std::vector<double>>();
    };
    dp::Runner::Calibration c;
    {
      py::gil_scoped_release nogil;
      c = r_->calibrate((const uint8_t*)pool, pool_images, first, steps, rounds, tol, ag, min_weight);
    }
    return calib_dict(c);
  }
  static py::dict calib_dict(const dp::Runner::Calibration& c) {
    py::dict d;
    d["weight"] = c.weight;
    d["steps"] = c.steps;
    py::list rs;
    for (const auto& r : c.rounds) {
      py::dict x;
      x["weight"] = r.weight;
      x["coord_count"] = r.coord_count;
      x["busy_coord_ms"] = r.busy_coord;
      x["busy_worker_ms"] = r.busy_worker;
      x["rate"] = r.rate();
      rs.append(x);
    }
    d["rounds"] = rs;
    return d;
  }
  py::tuple last_results() const { return py::make_tuple(r_->last_idx(), r_->last_prob()); }
  uintptr_t compute_stream() { return (uintptr_t)r_->worker()->stream(dp::Worker::kCompute); }
  void sync() {
    py::gil_scoped_release nogil;
    r_->worker()->sync_all();
  }
  // SDFS replicas placed where they are served: this global batch's shards
  // into every rank's HBM before a run (csrc/comm/runner.h stage()).
  void stage(uintptr_t src, uintptr_t dst) {
    py::gil_scoped_release nogil;
    r_->stage((const uint8_t*)src, (uint8_t*)dst);
  }
  int S_;
  std::vector<std::unique_ptr<Engine>> lanes_;
  std::unique_ptr<dp::Runner> r_;
};

// bench.py's exact per-rank call sequence (stage, prime, warmup, timed,
// unpipelined latency) on host workers and the rendezvous host
// communicator, one thread per rank (= one process per GPU). `pool`: two
// global batches on the coordinator. Returns per rank the steps of each run
// and on rank 0 whether the last step's answers match its images.
// All-gather of one double per thread-rank (the host stand-in for bench.py's
// gloo all_gather): every rank's call returns once all have contributed.
class ThreadAllGather {
 public:
  explicit ThreadAllGather(int world) : world_(world), vals_(world) {}
  std::vector<double> operator()(int rank, double x) {
    std::unique_lock<std::mutex> g(mu_);
    const int64_t gen = gen_;
    vals_[rank] = x;
    if (++arrived_ == world_) {
      out_ = vals_;
      arrived_ = 0;
      ++gen_;
      cv_.notify_all();
    } else {
      cv_.wait(g, [&] { return gen_ != gen; });
    }
    return out_;
  }

 private:
  int world_, arrived_ = 0;
  int64_t gen_ = 0;
  std::vector<double> vals_, out_;
  std::mutex mu_;
  std::condition_variable cv_;
};

py::dict dp_host_bench(py::array_t<uint8_t, py::array::c_style> pool, int world, int per_rank, double coord_weight,
                       const std::string& input_mode, int lanes, int prime, int warmup, int steps, int latency,
                       int us_per_image, int coord_extra_us, int calib_rounds, int calib_steps) {
  if (pool.ndim() != 4 || pool.shape(3) != 3) throw std::invalid_argument("pool must be u8 [n,H,W,3]");
  const int H = (int)pool.shape(1), W = (int)pool.shape(2);
  const size_t ib = (size_t)H * W * 3;
  const auto counts = dp::weighted_counts(per_rank, world, coord_weight);
  int64_t G = 0;
  for (int c : counts) G += c;
  if (pool.shape(0) != 2 * G) throw std::invalid_argument("pool must hold two global batches");
  const bool scatter = input_mode == "scatter";
  if (!scatter && input_mode != "staged") throw std::invalid_argument("input_mode: scatter | staged");
  const uint8_t* src = pool.data();
  auto cin = comm::host_world(world, 5000), cout = comm::host_world(world, 5000);
  std::vector<std::string> errs(world);
  std::vector<std::vector<int64_t>> done(world);
  std::vector<int32_t> last_idx;
  std::vector<float> last_prob;
  int64_t last_step = -1;
  std::vector<int> final_counts;
  dp::Runner::Calibration calib;
  ThreadAllGather ag(world);
  {
    py::gil_scoped_release nogil;
    std::vector<std::thread> ts;
    for (int r = 0; r < world; ++r)
      ts.emplace_back([&, r] {
        try {
          dp::Runner run(dp::make_host_worker(r, H, W, 1000, lanes, 0, 0, us_per_image, r == 0 ? coord_extra_us : 0),
                         world > 1 ? std::move(cin[r]) : nullptr, world > 1 ? std::move(cout[r]) : nullptr, world, r,
                         counts, scatter, ib, 5000);
          std::vector<uint8_t> mine;
          const uint8_t* p = r == 0 ? src : nullptr;
          int64_t np = r == 0 ? 2 * G : 0;
          if (!scatter) {  // staged: two per-rank batches at a stride of max_per_rank images
            mine.resize((size_t)2 * run.max_per_rank() * ib);
            for (int k = 0; k < 2; ++k)
              run.stage(r == 0 ? src + (size_t)k * G * ib : nullptr, mine.data() + (size_t)k * run.max_per_rank() * ib);
            p = mine.data();
            np = 2 * run.max_per_rank();
          }
          std::vector<int64_t> d;
          d.push_back(run.run(p, np, 0, prime).steps);
          if (calib_rounds > 0) {
            auto c = run.calibrate(p, np, prime, calib_steps, calib_rounds, 0.05,
                                   [&](double x) { return ag(r, x); });
            if (r == 0) calib = c;
          }
          d.push_back(run.run(p, np, 0, warmup).steps);
          d.push_back(run.run(p, np, warmup, steps).steps);
          d.push_back(run.run(p, np, warmup + steps, latency, /*pipelined=*/false).steps);
          done[r] = d;
          if (r == 0) {
            last_idx = run.last_idx();
            last_prob = run.last_prob();
            last_step = warmup + steps + latency - 1;
            final_counts = run.counts();
          }
        } catch (const std::exception& e) {
          errs[r] = e.what();
        }
      });
    for (auto& t : ts) t.join();
  }
  for (int r = 0; r < world; ++r)
    if (!errs[r].empty()) throw std::runtime_error("rank " + std::to_string(r) + ": " + errs[r]);
  // the last step read global batch (last_step % nb) at a stride of the
  // final counts' total (calibration may have lowered the coordinator's)
  int64_t Gf = 0;
  for (int c : final_counts) Gf += c;
  const int64_t nb = scatter ? std::max<int64_t>(1, 2 * G / std::max<int64_t>(1, Gf)) : 2;
  bool ok = (int64_t)last_idx.size() == Gf;
  const uint8_t* b = src + (size_t)(scatter ? (last_step % nb) * Gf : (last_step % 2) * G) * ib;
  for (int64_t i = 0; ok && i < Gf; ++i)
    ok = last_idx[i] == dp::host_class_of(b + i * ib, ib) && last_prob[i] == dp::host_prob_of(b + i * ib);
  py::dict out;
  out["steps"] = done;
  out["counts"] = final_counts;
  out["answers_ok"] = ok;
  out["calibration"] = DpRunner::calib_dict(calib);
  return out;
}

py::dict group_stats(const dp::Group::Stats& st) {
  py::dict d;
  d["images"] = st.images;
  d["steps"] = st.steps;
  d["recoveries"] = st.recoveries;
  d["redone_images"] = st.redone_images;
  return d;
}

// ------------------------------------------------------------------ loopback
// bench.py's per-rank call sequence (stage, prime, calibrate, timed runs,
// an unpipelined run) on `world` virtual ranks of ONE GPU: rank r is a
// dp::Runner over its own HIP worker (engines[r] + lanes - 1 copies, its own
// streams and slots) and the device-loopback communicators (stream-ordered
// device copies, comm::device_loopback_world), one thread per rank as one
// process per GPU would be. `pool`: the coordinator's device pool of two
// global batches. Returns every step's gathered answers from rank 0.
py::dict dp_loopback_bench(std::vector<Engine*> engines, uintptr_t pool, int per_rank, double coord_weight,
                           const std::string& input_mode, int lanes, int prime, int steps, int unpipelined,
                           int calib_rounds, int calib_steps, int image_size) {
  const int world = (int)engines.size();
  if (world < 1) throw std::invalid_argument("dp_loopback_bench: no engines");
  const bool scatter = input_mode == "scatter";
  if (!scatter && input_mode != "staged") throw std::invalid_argument("input_mode: scatter | staged");
  const int S = image_size;
  const size_t ib = (size_t)S * S * 3;
  const auto counts0 = dp::weighted_counts(per_rank, world, coord_weight);
  int64_t G = 0;
  for (int c : counts0) G += c;
  const uint8_t* src = (const uint8_t*)pool;
  auto cin = comm::device_loopback_world(world), cout = comm::device_loopback_world(world);
  // every rank's runner, built here (engine copies allocate), driven below by one thread each
  std::vector<std::vector<std::unique_ptr<Engine>>> lane_engines(world);
  std::vector<std::unique_ptr<dp::Runner>> runners;
  for (int r = 0; r < world; ++r) {
    Engine* e = engines[r];
    e->reserve(per_rank);
    std::vector<Engine*> more;
    for (int l = 1; l < lanes; ++l) {
      lane_engines[r].push_back(std::make_unique<Engine>(*e, e->device()));
      lane_engines[r].back()->copy_weights_from(*e);
      lane_engines[r].back()->reserve(std::max(e->max_batch(), per_rank));
      more.push_back(lane_engines[r].back().get());
    }
    runners.push_back(std::make_unique<dp::Runner>(dp::make_hip_worker(e, S, S, true, more),
                                                   world > 1 ? std::move(cin[r]) : nullptr,
                                                   world > 1 ? std::move(cout[r]) : nullptr, world, r, counts0,
                                                   scatter, ib, 20000));
  }
  std::vector<std::string> errs(world);
  std::vector<std::vector<int64_t>> done(world);
  std::vector<int64_t> ans_step;
  std::vector<std::vector<int32_t>> ans_idx;
  std::vector<std::vector<float>> ans_prob;
  std::vector<int> final_counts;
  dp::Runner::Calibration calib;
  ThreadAllGather ag(world);
  runners[0]->set_step_hook([&](int64_t step, const int32_t* i, const float* p, int64_t n) {
    ans_step.push_back(step);
    ans_idx.emplace_back(i, i + n);
    ans_prob.emplace_back(p, p + n);
  });
  {
    py::gil_scoped_release nogil;
    std::vector<std::thread> ts;
    for (int r = 0; r < world; ++r)
      ts.emplace_back([&, r] {
        uint8_t* mine = nullptr;
        try {
          dp::Runner& run = *runners[r];
          run.worker()->activate();
          const uint8_t* p = r == 0 ? src : nullptr;
          int64_t np = r == 0 ? 2 * G : 0;
          if (!scatter) {  // staged: two per-rank batches at a stride of max_per_rank images, in this rank's HBM
            DMLC_HIP_CHECK(hipMalloc(&mine, (size_t)2 * run.max_per_rank() * ib));
            for (int k = 0; k < 2; ++k)
              run.stage(r == 0 ? src + (size_t)k * G * ib : nullptr, mine + (size_t)k * run.max_per_rank() * ib);
            p = mine;
            np = 2 * run.max_per_rank();
          }
          std::vector<int64_t> d;
          d.push_back(run.run(p, np, 0, prime).steps);
          if (calib_rounds > 0) {
            auto c = run.calibrate(p, np, prime, calib_steps, calib_rounds, 0.05, [&](double x) { return ag(r, x); });
            if (r == 0) calib = c;
          }
          d.push_back(run.run(p, np, 1000, steps).steps);
          d.push_back(run.run(p, np, 1000 + steps, unpipelined, /*pipelined=*/false).steps);
          run.worker()->sync_all();
          done[r] = d;
          if (r == 0) final_counts = run.counts();
        } catch (const std::exception& e) {
          errs[r] = e.what();
        }
        if (mine) (void)hipFree(mine);
      });
    for (auto& t : ts) t.join();
  }
  for (int r = 0; r < world; ++r)
    if (!errs[r].empty()) throw std::runtime_error("rank " + std::to_string(r) + ": " + errs[r]);
  runners.clear();
  py::list steps_out;
  for (size_t k = 0; k < ans_step.size(); ++k) {
    steps_out.append(py::make_tuple(ans_step[k], py::array_t<int32_t>(ans_idx[k].size(), ans_idx[k].data()),
                                    py::array_t<float>(ans_prob[k].size(), ans_prob[k].data())));
  }
  py::dict out;
  out["runs"] = done;
  out["counts"] = final_counts;
  out["answers"] = steps_out;
  out["calibration"] = DpRunner::calib_dict(calib);
  return out;
}

// dp::Group (one process driving several GPUs: the serving fleet's scatter)
// over `engines` as its members on ONE GPU and device-loopback
// communicators; fail_member >= 1 is lost after fail_after steps (its
// communicator operations fail) and the group rebuilds over the survivors.
py::dict dp_loopback_group(std::vector<Engine*> engines, uintptr_t images, int64_t n, int max_per_rank,
                           int fail_member, int64_t fail_after, int repeats, int image_size) {
  const int S = image_size;
  std::vector<std::unique_ptr<dp::Worker>> owned;
  std::vector<dp::Worker*> ws;
  for (Engine* e : engines) {
    e->reserve(max_per_rank);
    owned.push_back(dp::make_hip_worker(e, S, S, true));
    ws.push_back(owned.back().get());
  }
  std::vector<std::vector<int>> builds;
  auto factory = [&builds](const std::vector<int>& members) {
    builds.push_back(members);
    return comm::device_loopback_world((int)members.size());
  };
  py::array_t<int32_t> idx(n), commits(n);
  py::array_t<float> prob(n);
  int32_t* pi = idx.mutable_data();
  float* pp = prob.mutable_data();
  int32_t* pc = commits.mutable_data();
  dp::Group::Stats st;
  std::vector<int> members;
  {
    py::gil_scoped_release nogil;
    dp::Group g(ws, factory, max_per_rank, (size_t)S * S * 3, 20000);
    if (fail_member >= 0) g.fail(fail_member, fail_after, /*abrupt=*/true);
    for (int k = 0; k < std::max(1, repeats); ++k) {
      std::fill(pi, pi + n, -1);
      std::fill(pc, pc + n, 0);
      st = g.classify((const uint8_t*)images, n, pi, pp, -1, pc);
    }
    members = g.members();
  }
  py::dict out;
  out["idx"] = idx;
  out["prob"] = prob;
  out["commits"] = commits;
  out["stats"] = group_stats(st);
  out["members"] = members;
  out["builds"] = builds;
  return out;
}

// ------------------------------------------------------------------ group
class DpGroupPy {
 public:
  DpGroupPy(std::vector<Engine*> engines, int max_per_rank, int image_size, bool use_graph, int timeout_ms)
      : S_(image_size) {
    std::vector<dp::Worker*> ws;
    std::vector<int> devices;
    for (Engine* e : engines) {
      workers_.push_back(dp::make_hip_worker(e, S_, S_, use_graph));
      ws.push_back(workers_.back().get());
      devices.push_back(e->device());
    }
    auto factory = [devices](const std::vector<int>& members) {
      std::vector<int> devs;
      for (int m : members) devs.push_back(devices.at(m));
      return comm::rccl_init_all(devs);
    };
    g_ = std::make_unique<dp::Group>(ws, factory, max_per_rank, (size_t)S_ * S_ * 3, timeout_ms);
  }
  py::tuple classify(uintptr_t src, int64_t n) {
    py::array_t<int32_t> idx(n);
    py::array_t<float> prob(n);
    dp::Group::Stats st;
    {
      int32_t* pi = idx.mutable_data();
      float* pp = prob.mutable_data();
      py::gil_scoped_release nogil;
      st = g_->classify((const uint8_t*)src, n, pi, pp);
    }
    return py::make_tuple(idx, prob, stats(st));
  }
  static py::dict stats(const dp::Group::Stats& st) {
    py::dict d;
    d["images"] = st.images;
    d["steps"] = st.steps;
    d["recoveries"] = st.recoveries;
    d["redone_images"] = st.redone_images;
    return d;
  }
  int S_;
  std::vector<std::unique_ptr<dp::Worker>> workers_;
  std::unique_ptr<dp::Group> g_;
};

// ------------------------------------------------------------------ host
py::dict dp_host_run(py::array_t<uint8_t, py::array::c_style> images, int world, int max_per_rank,
                     const std::string& mode, bool scatter, int fail_member, int64_t fail_after, bool abrupt,
                     bool pipelined, int slots, int us_per_image, int coord_extra_us, int repeats, bool auto_balance) {
  if (images.ndim() != 4 || images.shape(3) != 3) throw std::invalid_argument("images must be u8 [n,H,W,3]");
  const int64_t n = images.shape(0);
  const int H = (int)images.shape(1), W = (int)images.shape(2);
  const size_t ib = (size_t)H * W * 3;
  const uint8_t* src = images.data();
  py::array_t<int32_t> idx(n), commits(n);
  py::array_t<float> prob(n);
  int32_t* pi = idx.mutable_data();
  float* pp = prob.mutable_data();
  int32_t* pc = commits.mutable_data();
  std::fill(pi, pi + n, -1);
  std::fill(pp, pp + n, 0.f);
  std::fill(pc, pc + n, 0);
  py::dict out;
  if (mode == "group") {
    std::vector<std::unique_ptr<dp::Worker>> owned;
    std::vector<dp::Worker*> ws;
    for (int r = 0; r < world; ++r) {
      owned.push_back(dp::make_host_worker(r, H, W, 1000, 1, 0, 0, us_per_image, r == 0 ? coord_extra_us : 0));
      ws.push_back(owned.back().get());
    }
    std::vector<std::vector<int>> builds;
    auto factory = [&builds](const std::vector<int>& members) {
      builds.push_back(members);
      return comm::host_world((int)members.size(), 5000);
    };
    dp::Group::Stats st;
    std::vector<int> members;
    std::vector<double> weights;
    {
      py::gil_scoped_release nogil;
      dp::Group g(ws, factory, max_per_rank, ib, 5000);
      g.set_coord_weight(1.0, auto_balance);
      if (fail_member >= 0) g.fail(fail_member, fail_after, abrupt);
      for (int k = 0; k < std::max(1, repeats); ++k) {
        if (k > 0) std::fill(pc, pc + n, 0);
        st = g.classify(src, n, pi, pp, -1, pc);
        weights.push_back(g.coord_weight());
      }
      members = g.members();
    }
    out["coord_weights"] = weights;
    out["stats"] = DpGroupPy::stats(st);
    out["members"] = members;
    out["builds"] = builds;
  } else if (mode == "threads") {
    // one thread per rank: the multi-process issue order
    auto cin = comm::host_world(world, 5000), cout = comm::host_world(world, 5000);
    const int64_t G = (int64_t)max_per_rank * world;
    const int64_t steps = (n + G - 1) / G;
    std::vector<std::string> errs(world);
    std::vector<int64_t> steps_done(world, 0);
    {
      py::gil_scoped_release nogil;
      std::vector<std::thread> ts;
      for (int r = 0; r < world; ++r)
        ts.emplace_back([&, r] {
          try {
            auto w = dp::make_host_worker(r, H, W);
            dp::Rank rank(w.get(), max_per_rank, ib, scatter, slots);
            if (world > 1) rank.attach(cin[r].get(), cout[r].get());
            else rank.attach(nullptr, nullptr);
            auto plan = [&](int64_t step, const dp::Rank& rk) {
              dp::StepPlan p;
              p.step = step;
              p.counts = dp::shard_counts(std::min<int64_t>(G, n - step * G), world, max_per_rank);
              int64_t off = step * G;
              if (!scatter)
                for (int q = 0; q < rk.rank(); ++q) off += p.counts[q];
              // scatter: only the coordinator holds the images
              p.src = (scatter && rk.rank() != 0) ? nullptr : src + (size_t)off * ib;
              return p;
            };
            auto on_result = [&](const dp::StepPlan& p, const int32_t* i, const float* pr) {
              int64_t total = 0;
              for (int c : p.counts) total += c;
              const int64_t start = p.step * G;
              std::memcpy(pi + start, i, (size_t)total * 4);
              std::memcpy(pp + start, pr, (size_t)total * 4);
              for (int64_t k = 0; k < total; ++k) ++pc[start + k];
            };
            auto res = dp::run_pipeline({&rank}, 0, steps, plan, on_result, 5000, pipelined);
            steps_done[r] = res.steps;
          } catch (const std::exception& e) {
            errs[r] = e.what();
          }
        });
      for (auto& t : ts) t.join();
    }
    for (int r = 0; r < world; ++r)
      if (!errs[r].empty()) throw std::runtime_error("rank " + std::to_string(r) + ": " + errs[r]);
    out["steps"] = steps_done;
  } else {
    throw std::invalid_argument("mode must be 'group' or 'threads'");
  }
  out["idx"] = idx;
  out["prob"] = prob;
  out["commits"] = commits;
  return out;
}

// ------------------------------------------------------------------ host fleet
// The serving fleet (csrc/comm/fleet.h) over host workers and the rendezvous
// host communicator: the partition rule, rebalancing after a GPU loss, the
// weight broadcast into moved GPUs, per-query routing under concurrency and
// exactly-once answers, all on the CPU (tests/test_fleet_cpu.py).
// Every communicator world the fleet creates is tracked: worlds alive at the
// same time must cover identical or disjoint device sets (two models never
// hold communicators on one device).
class HostFleet {
 public:
  HostFleet(std::vector<int> devices, int H, int W, int lanes, int delay_us, int max_per_rank, int min_shard,
            std::map<std::string, uint32_t> seeds, int batch_window_us, bool eager_when_idle)
      : H_(H), W_(W), seeds_(std::move(seeds)) {
    dp::FleetOptions o;
    o.max_per_rank = max_per_rank;
    o.image_bytes = (size_t)H * W * 3;
    o.min_shard = min_shard;
    o.aux_bytes = 8;
    o.timeout_ms = 5000;
    o.batch_window_us = batch_window_us;
    o.eager_when_idle = eager_when_idle;
    auto wf = [this, lanes, delay_us](const std::string& m, int d, dp::Worker* rep) {
      std::lock_guard<std::mutex> g(mu_);
      if (fail_builds_ > 0) {  // fault injection: a worker build that fails (OOM, HIP error)
        --fail_builds_;
        throw std::runtime_error("HostFleet: injected worker build failure");
      }
      auto it = seeds_.find(m);
      if (it == seeds_.end()) throw std::runtime_error("HostFleet: unknown model " + m);
      builds_.push_back({m, d, rep != nullptr});
      // a replica starts with an empty arena: only the broadcast makes it right
      return dp::make_host_worker(d, H_, W_, 1000, lanes, rep ? 0u : it->second, delay_us);
    };
    auto cf = [this](const std::vector<int>& devs) {
      std::vector<std::unique_ptr<comm::Comm>> out;
      auto world = std::make_shared<int>(0);
      {
        std::lock_guard<std::mutex> g(mu_);
        for (auto& w : worlds_) {
          if (w.second.expired()) continue;
          std::set<int> a(w.first.begin(), w.first.end()), b(devs.begin(), devs.end());
          bool overlap = false;
          for (int x : b) overlap |= a.count(x) > 0;
          if (overlap && a != b) overlaps_.push_back(w.first), overlaps_.push_back(devs);
        }
        worlds_.emplace_back(devs, world);
        comm_builds_.push_back(devs);
      }
      for (auto& c : comm::host_world((int)devs.size(), 5000)) out.push_back(std::make_unique<Tracked>(std::move(c), world));
      return out;
    };
    f_ = std::make_unique<dp::Fleet>(devices, wf, cf, o);
  }
  void set_jobs(const std::vector<std::string>& j) {
    py::gil_scoped_release nogil;
    f_->set_jobs(j);
  }
  void load(const std::string& m) {
    py::gil_scoped_release nogil;
    f_->load(m);
  }
  void lose(int d) {
    py::gil_scoped_release nogil;
    f_->lose(d);
  }
  // new "host weights" for `model` (then load() = a hot swap, as `train`)
  void set_seed(const std::string& m, uint32_t seed) {
    std::lock_guard<std::mutex> g(mu_);
    seeds_[m] = seed;
  }
  // the next n worker builds throw
  void fail_next_builds(int n) {
    std::lock_guard<std::mutex> g(mu_);
    fail_builds_ = n;
  }
  // abrupt: every instance on `d` starts failing (found by the next query)
  void fail(int d) {
    for (const auto& kv : f_->partitions())
      if (dp::Worker* w = f_->worker(kv.first, d)) dp::host_worker_set_healthy(*w, false);
  }
  // queries: (model, first, count) over `images`; run by `threads` threads.
  // Queries listed in `bad` fail inside their stage function (as a JPEG of
  // a bad size does in the GPU executor's stage): only they get an error.
  py::dict run(py::array_t<uint8_t, py::array::c_style> images, std::vector<std::tuple<std::string, int64_t, int64_t>> qs,
               int threads, std::vector<int> bad) {
    const std::set<int> bad_q(bad.begin(), bad.end());
    const size_t ib = (size_t)H_ * W_ * 3;
    const uint8_t* src = images.data();
    const int64_t total = images.shape(0);
    std::vector<std::vector<int32_t>> idx(qs.size());
    std::vector<std::vector<float>> prob(qs.size());
    std::vector<dp::Fleet::Route> routes(qs.size());
    std::vector<std::string> errs(qs.size());
    {
      py::gil_scoped_release nogil;
      std::atomic<size_t> next{0};
      std::vector<std::thread> ts;
      for (int t = 0; t < std::max(1, threads); ++t)
        ts.emplace_back([&] {
          for (size_t q = next++; q < qs.size(); q = next++) {
            const auto& [model, first, count] = qs[q];
            try {
              if (first < 0 || first + count > total) throw std::invalid_argument("query out of range");
              idx[q].assign(count, -1);
              prob[q].assign(count, 0.f);
              const bool fails = bad_q.count((int)q) > 0;
              auto stage = [&, first = first, fails](const dp::StageCtx& c, int64_t off, int64_t n) -> const uint8_t* {
                if (fails) throw std::runtime_error("stage: bad image size");
                if (n > c.capacity) throw std::logic_error("stage: more images than the batch holds");
                std::memcpy(c.batch, src + (size_t)(first + off) * ib, (size_t)n * ib);
                return (const uint8_t*)c.batch;
              };
              routes[q] = f_->classify(model, count, stage, idx[q].data(), prob[q].data());
            } catch (const std::exception& e) {
              errs[q] = e.what();
            }
          }
        });
      for (auto& t : ts) t.join();
    }
    py::list out_idx, out_prob, out_route;
    for (size_t q = 0; q < qs.size(); ++q) {
      out_idx.append(py::array_t<int32_t>(idx[q].size(), idx[q].data()));
      out_prob.append(py::array_t<float>(prob[q].size(), prob[q].data()));
      py::dict r;
      r["device"] = routes[q].device;
      r["scattered"] = routes[q].scattered;
      r["devices_used"] = routes[q].devices_used;
      r["retries"] = routes[q].retries;
      out_route.append(r);
    }
    py::dict d;
    d["idx"] = out_idx;
    d["prob"] = out_prob;
    d["routes"] = out_route;
    d["errors"] = errs;
    return d;
  }
  py::dict state() {
    py::dict d;
    d["partitions"] = f_->partitions();
    d["live"] = f_->live();
    d["rebalances"] = f_->rebalances();
    std::map<std::string, std::map<int, int64_t>> served;
    for (const auto& kv : f_->partitions()) served[kv.first] = f_->served(kv.first);
    d["served"] = served;
    std::map<std::string, std::map<int, int64_t>> fwd;
    for (const auto& kv : f_->partitions()) fwd[kv.first] = f_->forwards(kv.first);
    d["forwards"] = fwd;
    std::map<std::string, std::map<int, int64_t>> sizes;
    for (const auto& kv : f_->partitions()) sizes[kv.first] = f_->forward_sizes(kv.first);
    d["forward_sizes"] = sizes;
    std::lock_guard<std::mutex> g(mu_);
    d["comm_builds"] = comm_builds_;
    d["overlapping_worlds"] = overlaps_;
    py::list b;
    for (const auto& x : builds_) b.append(py::make_tuple(std::get<0>(x), std::get<1>(x), std::get<2>(x)));
    d["worker_builds"] = b;
    return d;
  }

 private:
  // a host communicator that keeps its world's liveness token alive
  struct Tracked : comm::Comm {
    Tracked(std::unique_ptr<comm::Comm> c, std::shared_ptr<int> t) : c_(std::move(c)), t_(std::move(t)) {}
    int rank() const override { return c_->rank(); }
    int size() const override { return c_->size(); }
    std::string backend() const override { return c_->backend(); }
    void group_start() override { c_->group_start(); }
    void group_end() override { c_->group_end(); }
    void send(const void* b, size_t n, int p, comm::Stream s) override { c_->send(b, n, p, s); }
    void recv(void* b, size_t n, int p, comm::Stream s) override { c_->recv(b, n, p, s); }
    void broadcast(const void* sb, void* rb, size_t n, int root, comm::Stream s) override {
      c_->broadcast(sb, rb, n, root, s);
    }
    bool ok() override { return c_->ok(); }
    void abort() override { c_->abort(); }
    std::unique_ptr<comm::Comm> c_;
    std::shared_ptr<int> t_;
  };
  int H_, W_;
  std::map<std::string, uint32_t> seeds_;
  int fail_builds_ = 0;
  std::unique_ptr<dp::Fleet> f_;
  std::mutex mu_;
  std::vector<std::pair<std::vector<int>, std::weak_ptr<int>>> worlds_;
  std::vector<std::vector<int>> comm_builds_, overlaps_;
  std::vector<std::tuple<std::string, int, bool>> builds_;
};

// A deliberately mis-ordered exchange on the host fake: with `bad`, both
// ranks send before they receive (each in its own group); RCCL would hang,
// the rendezvous fake must time out. Without it, the well-ordered exchange
// completes and nothing is left pending.
py::dict host_order_probe(bool bad, int timeout_ms) {
  auto cs = comm::host_world(2, timeout_ms);
  std::vector<uint8_t> a(64, 1), b(64, 2), ra(64, 0), rb(64, 0);
  std::string e0, e1;
  {
    py::gil_scoped_release nogil;
    std::thread t1([&] {
      try {
        if (bad) {
          cs[1]->send(b.data(), 64, 0, nullptr);
          cs[1]->recv(rb.data(), 64, 0, nullptr);
        } else {
          cs[1]->recv(rb.data(), 64, 0, nullptr);
          cs[1]->send(b.data(), 64, 0, nullptr);
        }
      } catch (const std::exception& e) {
        e1 = e.what();
      }
    });
    try {
      cs[0]->send(a.data(), 64, 1, nullptr);
      cs[0]->recv(ra.data(), 64, 1, nullptr);
    } catch (const std::exception& e) {
      e0 = e.what();
    }
    t1.join();
  }
  py::dict d;
  d["err0"] = e0;
  d["err1"] = e1;
  d["ok"] = ra == b && rb == a;
  d["pending"] = comm::host_pending(*cs[0]);
  return d;
}

// One group spanning two communicators, posted by the two ranks in opposite
// communicator order (rank 0: send on A, recv on B; rank 1: send on B, recv
// on A): valid for RCCL, so the host fake must complete it too.
py::dict host_multi_world_probe(int timeout_ms) {
  auto A = comm::host_world(2, timeout_ms), B = comm::host_world(2, timeout_ms);
  std::vector<uint8_t> a(64, 1), b(64, 2), ra(64, 0), rb(64, 0);
  std::string e0, e1;
  {
    py::gil_scoped_release nogil;
    std::thread t1([&] {
      try {
        A[1]->group_start();
        B[1]->send(b.data(), 64, 0, nullptr);
        A[1]->recv(rb.data(), 64, 0, nullptr);
        A[1]->group_end();
      } catch (const std::exception& e) {
        e1 = e.what();
      }
    });
    try {
      A[0]->group_start();
      A[0]->send(a.data(), 64, 1, nullptr);
      B[0]->recv(ra.data(), 64, 1, nullptr);
      A[0]->group_end();
    } catch (const std::exception& e) {
      e0 = e.what();
    }
    t1.join();
  }
  py::dict d;
  d["err0"] = e0;
  d["err1"] = e1;
  d["ok"] = ra == b && rb == a;
  d["pending"] = comm::host_pending(*A[0]) + comm::host_pending(*B[0]);
  return d;
}

// One-rank RCCL communicator on `device` (optionally CTA-capped) moving
// `bytes` to itself with a grouped send/recv and a broadcast: exercises the
// RcclComm wrapper and librccl on a one-GPU box (tests/test_dp_native_gpu.py).
bool rccl_loopback(int device, size_t bytes, int max_ctas) {
  if (hipSetDevice(device) != hipSuccess) throw std::runtime_error("rccl_loopback: hipSetDevice");
  auto c = comm::rccl_init_rank(comm::rccl_unique_id(), 1, 0, device, max_ctas);
  hipStream_t s;
  uint8_t *a, *b, *d;
  if (hipStreamCreate(&s) != hipSuccess || hipMalloc(&a, bytes) != hipSuccess || hipMalloc(&b, bytes) != hipSuccess ||
      hipMalloc(&d, bytes) != hipSuccess)
    throw std::runtime_error("rccl_loopback: allocation");
  std::vector<uint8_t> h(bytes), g(bytes), g2(bytes);
  for (size_t i = 0; i < bytes; ++i) h[i] = (uint8_t)(i * 131 + 7);
  bool ok = hipMemcpy(a, h.data(), bytes, hipMemcpyHostToDevice) == hipSuccess &&
            hipMemset(b, 0, bytes) == hipSuccess && hipMemset(d, 0, bytes) == hipSuccess;
  c->group_start();
  c->send(a, bytes, 0, s);
  c->recv(b, bytes, 0, s);
  c->group_end();
  c->broadcast(a, d, bytes, 0, s);
  ok = ok && hipStreamSynchronize(s) == hipSuccess && c->ok();
  ok = ok && hipMemcpy(g.data(), b, bytes, hipMemcpyDeviceToHost) == hipSuccess &&
       hipMemcpy(g2.data(), d, bytes, hipMemcpyDeviceToHost) == hipSuccess;
  ok = ok && g == h && g2 == h;
  c.reset();
  (void)hipFree(a);
  (void)hipFree(b);
  (void)hipFree(d);
  (void)hipStreamDestroy(s);
  return ok;
}

// A one-rank RCCL communicator that issues self send/recv groups on a given
// stream without waiting: real RCCL kernels (their CTAs, LDS and register
// footprint) next to the forward on one GPU, for tools/interference_probe.py
// (what the coordinator's scatter does to its own compute at N > 1).
class RcclLoop {
 public:
  RcclLoop(int device, int max_ctas) : c_(comm::rccl_init_rank(comm::rccl_unique_id(), 1, 0, device, max_ctas)) {}
  // `legs` grouped send/recv pairs of `bytes` each, src -> dst + i * bytes
  void issue(uintptr_t stream, uintptr_t src, uintptr_t dst, size_t bytes, int legs) {
    c_->group_start();
    for (int i = 0; i < legs; ++i) {
      c_->send((const void*)(src + i * bytes), bytes, 0, (comm::Stream)stream);
      c_->recv((void*)(dst + i * bytes), bytes, 0, (comm::Stream)stream);
    }
    c_->group_end();
  }

 private:
  std::unique_ptr<comm::Comm> c_;
};

}  // namespace

void bind_dp(py::module& m) {
  m.def("dp_partition_devices", &dp::partition_devices, py::arg("live"), py::arg("jobs"));
  m.def("fleet_bucket_batch", &dp::bucket_batch, py::arg("b"), py::arg("max"));
  m.def("dp_loopback_bench", &dp_loopback_bench, py::arg("engines"), py::arg("pool"), py::arg("per_rank"),
        py::arg("coord_weight") = 1.0, py::arg("input_mode") = "scatter", py::arg("lanes") = 2, py::arg("prime") = 4,
        py::arg("steps") = 50, py::arg("unpipelined") = 4, py::arg("calib_rounds") = 0, py::arg("calib_steps") = 4,
        py::arg("image_size") = 224);
  m.def("dp_loopback_group", &dp_loopback_group, py::arg("engines"), py::arg("images"), py::arg("n"),
        py::arg("max_per_rank"), py::arg("fail_member") = -1, py::arg("fail_after") = 0, py::arg("repeats") = 1,
        py::arg("image_size") = 224);
  m.def("host_order_probe", &host_order_probe, py::arg("bad"), py::arg("timeout_ms") = 500);
  m.def("host_multi_world_probe", &host_multi_world_probe, py::arg("timeout_ms") = 2000);
  py::class_<HostFleet>(m, "HostFleet")
      .def(py::init<std::vector<int>, int, int, int, int, int, int, std::map<std::string, uint32_t>, int, bool>(),
           py::arg("devices"), py::arg("H"), py::arg("W"), py::arg("lanes"), py::arg("delay_us"),
           py::arg("max_per_rank"), py::arg("min_shard"), py::arg("seeds"), py::arg("batch_window_us") = 200,
           py::arg("eager_when_idle") = true)
      .def("set_jobs", &HostFleet::set_jobs)
      .def("load", &HostFleet::load)
      .def("lose", &HostFleet::lose)
      .def("fail", &HostFleet::fail)
      .def("set_seed", &HostFleet::set_seed)
      .def("fail_next_builds", &HostFleet::fail_next_builds)
      .def("run", &HostFleet::run, py::arg("images"), py::arg("queries"), py::arg("threads") = 1,
           py::arg("bad") = std::vector<int>{})
      .def("state", &HostFleet::state);
  py::class_<RcclLoop>(m, "RcclLoop")
      .def(py::init<int, int>(), py::arg("device") = 0, py::arg("max_ctas") = 0)
      .def("issue", &RcclLoop::issue, py::arg("stream"), py::arg("src"), py::arg("dst"), py::arg("bytes"),
           py::arg("legs") = 7);
  m.def("rccl_loopback", &rccl_loopback, py::arg("device") = 0, py::arg("bytes") = 1 << 20, py::arg("max_ctas") = 0);
  m.def("rccl_unique_id", []() { return py::bytes(comm::rccl_unique_id()); });
  m.def("socket_unique_id", []() { return py::bytes(comm::socket_unique_id()); });
  m.def("dp_shard_counts", &dp::shard_counts);
  m.def("dp_weighted_counts", &dp::weighted_counts, py::arg("per_rank"), py::arg("world"), py::arg("coord_weight"));
  m.def("dp_host_bench", &dp_host_bench, py::arg("pool"), py::arg("world"), py::arg("per_rank"),
        py::arg("coord_weight") = 1.0, py::arg("input_mode") = "scatter", py::arg("lanes") = 2, py::arg("prime") = 3,
        py::arg("warmup") = 2, py::arg("steps") = 5, py::arg("latency") = 3, py::arg("us_per_image") = 0,
        py::arg("coord_extra_us") = 0, py::arg("calib_rounds") = 0, py::arg("calib_steps") = 4);
  m.def("dp_weighted_shards", &dp::weighted_shards, py::arg("n"), py::arg("world"), py::arg("cap"), py::arg("w0"));
  m.def("dp_next_coord_weight",
        [](double w, double b0, double bw, int c0, int per, int world, double min_w) {
          dp::CalibRound r;
          r.weight = w, r.busy_coord = b0, r.busy_worker = bw, r.coord_count = c0, r.per_rank = per, r.world = world;
          return dp::next_coord_weight(r, min_w);
        },
        py::arg("weight"), py::arg("busy_coord"), py::arg("busy_worker"), py::arg("coord_count"), py::arg("per_rank"),
        py::arg("world"), py::arg("min_weight") = 0.5);
  m.def("dp_host_run", &dp_host_run, py::arg("images"), py::arg("world"), py::arg("max_per_rank"),
        py::arg("mode") = "group", py::arg("scatter") = true, py::arg("fail_member") = -1,
        py::arg("fail_after") = 0, py::arg("abrupt") = false, py::arg("pipelined") = true, py::arg("slots") = 2,
        py::arg("us_per_image") = 0, py::arg("coord_extra_us") = 0, py::arg("repeats") = 1,
        py::arg("auto_balance") = true);
  py::class_<DpRunner>(m, "DpRunner")
      .def(py::init([](Engine* e, int world, int rank, py::bytes id_in, py::bytes id_out, int max_per_rank,
                       bool scatter, int image_size, bool use_graph, int timeout_ms, int lanes, int slots,
                       double coord_weight, std::vector<int> counts) {
             return new DpRunner(e, world, rank, std::string(id_in), std::string(id_out), max_per_rank, scatter,
                                 image_size, use_graph, timeout_ms, lanes, slots, coord_weight, counts);
           }),
           py::arg("engine"), py::arg("world"), py::arg("rank"), py::arg("id_in"), py::arg("id_out"),
           py::arg("max_per_rank"), py::arg("scatter") = true, py::arg("image_size") = 224,
           py::arg("use_graph") = true, py::arg("timeout_ms") = -1, py::arg("lanes") = 1, py::arg("slots") = 0,
           py::arg("coord_weight") = 1.0, py::arg("counts") = std::vector<int>{}, py::keep_alive<1, 2>())
      .def_static("host",
                  [](int world, int rank, py::bytes id_in, py::bytes id_out, int max_per_rank, bool scatter,
                     int image_size, int timeout_ms, int lanes, int slots, double coord_weight, int us_per_image,
                     int coord_extra_us) {
                    return std::unique_ptr<DpRunner>(new DpRunner(world, rank, std::string(id_in), std::string(id_out),
                                                                  max_per_rank, scatter, image_size, timeout_ms, lanes,
                                                                  slots, coord_weight, us_per_image, coord_extra_us));
                  },
                  py::arg("world"), py::arg("rank"), py::arg("id_in"), py::arg("id_out"), py::arg("max_per_rank"),
                  py::arg("scatter") = true, py::arg("image_size") = 224, py::arg("timeout_ms") = 60000,
                  py::arg("lanes") = 2, py::arg("slots") = 0, py::arg("coord_weight") = 1.0,
                  py::arg("us_per_image") = 4, py::arg("coord_extra_us") = 0)
      .def("run", &DpRunner::run, py::arg("pool"), py::arg("pool_images"), py::arg("first"), py::arg("n"),
           py::arg("pipelined") = true)
      .def("last_results", &DpRunner::last_results)
      .def("compute_stream", &DpRunner::compute_stream)
      .def("sync", &DpRunner::sync)
      .def("stage", &DpRunner::stage, py::arg("src"), py::arg("dst"))
      .def("set_counts", &DpRunner::set_counts, py::arg("counts"))
      .def("calibrate", &DpRunner::calibrate, py::arg("pool"), py::arg("pool_images"), py::arg("first"),
           py::arg("steps"), py::arg("rounds"), py::arg("tol"), py::arg("allgather"), py::arg("min_weight") = 0.5)
      .def_property_readonly("counts", [](const DpRunner& r) { return r.r_->counts(); })
      .def_property_readonly("max_per_rank", [](const DpRunner& r) { return r.r_->max_per_rank(); });
  py::class_<DpGroupPy>(m, "DpGroup")
      .def(py::init([](std::vector<Engine*> engines, int max_per_rank, int image_size, bool use_graph,
                       int timeout_ms) { return new DpGroupPy(engines, max_per_rank, image_size, use_graph, timeout_ms); }),
           py::arg("engines"), py::arg("max_per_rank"), py::arg("image_size") = 224, py::arg("use_graph") = true,
           py::arg("timeout_ms") = 30000, py::keep_alive<1, 2>())
      .def("classify", &DpGroupPy::classify, py::arg("src"), py::arg("n"))
      .def("fail", [](DpGroupPy& g, int m, int64_t after) { g.g_->fail(m, after, false); }, py::arg("member"),
           py::arg("after_steps") = 0)
      .def_property_readonly("members", [](const DpGroupPy& g) { return g.g_->members(); });
}
