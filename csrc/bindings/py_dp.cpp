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
#include "../runtime/engine.h"

namespace py = pybind11;
using namespace dmlc;

namespace {

// ------------------------------------------------------------------ runner
class DpRunner {
 public:
  DpRunner(Engine* e, int world, int rank, const std::string& id_in, const std::string& id_out, int max_per_rank,
           bool scatter, int image_size, bool use_graph, int timeout_ms, int lanes, int slots)
      : world_(world), rank_(rank), max_(max_per_rank), scatter_(scatter), S_(image_size), timeout_ms_(timeout_ms) {
    if (lanes < 1 || lanes > dp::Worker::kMaxLanes) throw std::invalid_argument("DpRunner: lanes must be 1..4");
    std::vector<Engine*> more;
    for (int l = 1; l < lanes; ++l) {  // further instances of the model: consecutive steps overlap
      lanes_.push_back(std::make_unique<Engine>(*e, e->device()));
      lanes_.back()->copy_weights_from(*e);
      lanes_.back()->reserve(std::max(e->max_batch(), max_per_rank));
      more.push_back(lanes_.back().get());
    }
    w_ = dp::make_hip_worker(e, S_, S_, use_graph, more);
    // one slot per lane (>= 2): that many steps in flight
    // Steps in flight (slots). Step i reuses slot i - slots, so its forward
    // waits for that step's answers to have left; with slots = 2 that was the
    // step just before on the same lane, and the answer copy's latency sat
    // between a lane's consecutive forwards (bench: 268k vs 276k img/s with 4
    // slots, the bare two-lane loop 276.7k: tools/pipeline_probe.py).
    if (slots <= 0) slots = 2 * std::max(2, lanes);
    if (slots < 2) throw std::invalid_argument("DpRunner: slots must be >= 2");
    r_ = std::make_unique<dp::Rank>(w_.get(), max_, ib(), scatter_, slots);
    if (world_ > 1) {
      cin_ = comm::rccl_init_rank(id_in, world_, rank_, e->device());
      // answers: 8 B per image, one CTA (comm::rccl_init_rank's max_ctas)
      cout_ = comm::rccl_init_rank(id_out, world_, rank_, e->device(), 1);
      r_->attach(cin_.get(), cout_.get());
    } else {
      r_->attach(nullptr, nullptr);
    }
  }
  ~DpRunner() {
    r_.reset();
    w_.reset();
    lanes_.clear();
    cin_.reset();
    cout_.reset();
  }
  size_t ib() const { return (size_t)S_ * S_ * 3; }

  // Steps [first, first+n) over a staged pool: scatter mode reads global
  // batches (max*world images) from the coordinator's pool; local mode reads
  // per-rank batches from this rank's own pool.
  py::dict run(uintptr_t pool, int64_t pool_images, int64_t first, int64_t n, bool pipelined) {
    const int64_t G = (int64_t)max_ * world_;
    const int64_t per = scatter_ ? G : max_;
    const bool has_pool = scatter_ ? rank_ == 0 : true;
    if (has_pool && pool_images < per) throw std::invalid_argument("DpRunner.run: pool smaller than one batch");
    const int64_t nb = has_pool ? pool_images / per : 1;
    auto counts = dp::shard_counts(G, world_, max_);
    auto plan = [&](int64_t step, const dp::Rank&) {
      dp::StepPlan p;
      p.step = step;
      p.counts = counts;
      p.src = has_pool ? (const uint8_t*)pool + (size_t)((step % nb) * per) * ib() : nullptr;
      return p;
    };
    auto on_result = [&](const dp::StepPlan&, const int32_t* i, const float* pr) {
      last_idx_.assign(i, i + G);
      last_prob_.assign(pr, pr + G);
    };
    dp::PipelineResult res;
    {
      py::gil_scoped_release nogil;
      res = dp::run_pipeline({r_.get()}, first, n, plan, on_result, timeout_ms_, pipelined);
    }
    py::dict d;
    d["steps"] = res.steps;
    d["images"] = res.images;
    d["step_ms"] = res.step_ms;
    return d;
  }
  py::tuple last_results() const { return py::make_tuple(last_idx_, last_prob_); }
  uintptr_t compute_stream() { return (uintptr_t)w_->stream(dp::Worker::kCompute); }
  void sync() {
    py::gil_scoped_release nogil;
    w_->sync_all();
  }
  // Stage shards into every rank's HBM before a run (SDFS replicas placed
  // where they are served): the coordinator's `images` images per rank at
  // src (rank r's at image offset r * images) go to dst on rank r over the
  // shard communicator (its own part by a device copy); blocks until done.
  void stage(uintptr_t src, uintptr_t dst, int64_t images) {
    const size_t bytes = (size_t)images * ib();
    py::gil_scoped_release nogil;
    w_->activate();
    if (rank_ == 0) w_->copy((void*)dst, (const void*)src, bytes, dp::Worker::kIn);
    if (world_ > 1) {
      cin_->group_start();
      if (rank_ == 0) {
        for (int r = 1; r < world_; ++r) cin_->send((const void*)(src + r * bytes), bytes, r, w_->stream(dp::Worker::kIn));
      } else {
        cin_->recv((void*)dst, bytes, 0, w_->stream(dp::Worker::kIn));
      }
      cin_->group_end();
    }
    w_->sync_all();
  }

  int world_, rank_, max_;
  bool scatter_;
  int S_, timeout_ms_;
  std::vector<std::unique_ptr<Engine>> lanes_;
  std::unique_ptr<dp::Worker> w_;
  std::unique_ptr<dp::Rank> r_;
  std::unique_ptr<comm::Comm> cin_, cout_;
  std::vector<int32_t> last_idx_;
  std::vector<float> last_prob_;
};

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
                     bool pipelined, int slots) {
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
      owned.push_back(dp::make_host_worker(r, H, W));
      ws.push_back(owned.back().get());
    }
    std::vector<std::vector<int>> builds;
    auto factory = [&builds](const std::vector<int>& members) {
      builds.push_back(members);
      return comm::host_world((int)members.size(), 5000);
    };
    dp::Group::Stats st;
    std::vector<int> members;
    {
      py::gil_scoped_release nogil;
      dp::Group g(ws, factory, max_per_rank, ib, 5000);
      if (fail_member >= 0) g.fail(fail_member, fail_after, abrupt);
      st = g.classify(src, n, pi, pp, -1, pc);
      members = g.members();
    }
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
  py::class_<RcclLoop>(m, "RcclLoop")
      .def(py::init<int, int>(), py::arg("device") = 0, py::arg("max_ctas") = 0)
      .def("issue", &RcclLoop::issue, py::arg("stream"), py::arg("src"), py::arg("dst"), py::arg("bytes"),
           py::arg("legs") = 7);
  m.def("rccl_loopback", &rccl_loopback, py::arg("device") = 0, py::arg("bytes") = 1 << 20, py::arg("max_ctas") = 0);
  m.def("rccl_unique_id", []() { return py::bytes(comm::rccl_unique_id()); });
  m.def("dp_shard_counts", &dp::shard_counts);
  m.def("dp_host_run", &dp_host_run, py::arg("images"), py::arg("world"), py::arg("max_per_rank"),
        py::arg("mode") = "group", py::arg("scatter") = true, py::arg("fail_member") = -1,
        py::arg("fail_after") = 0, py::arg("abrupt") = false, py::arg("pipelined") = true, py::arg("slots") = 2);
  py::class_<DpRunner>(m, "DpRunner")
      .def(py::init([](Engine* e, int world, int rank, py::bytes id_in, py::bytes id_out, int max_per_rank,
                       bool scatter, int image_size, bool use_graph, int timeout_ms, int lanes, int slots) {
             return new DpRunner(e, world, rank, std::string(id_in), std::string(id_out), max_per_rank, scatter,
                                 image_size, use_graph, timeout_ms, lanes, slots);
           }),
           py::arg("engine"), py::arg("world"), py::arg("rank"), py::arg("id_in"), py::arg("id_out"),
           py::arg("max_per_rank"), py::arg("scatter") = true, py::arg("image_size") = 224,
           py::arg("use_graph") = true, py::arg("timeout_ms") = -1, py::arg("lanes") = 1, py::arg("slots") = 0,
           py::keep_alive<1, 2>())
      .def("run", &DpRunner::run, py::arg("pool"), py::arg("pool_images"), py::arg("first"), py::arg("n"),
           py::arg("pipelined") = true)
      .def("last_results", &DpRunner::last_results)
      .def("compute_stream", &DpRunner::compute_stream)
      .def("sync", &DpRunner::sync)
      .def("stage", &DpRunner::stage, py::arg("src"), py::arg("dst"), py::arg("images"));
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
