#include "fleet.h"

#include "cv_wait.h"

#include <algorithm>
#include <chrono>
#include <climits>
#include <deque>
#include <cstring>
#include <stdexcept>

namespace dmlc {
namespace dp {

std::vector<std::vector<int>> partition_devices(std::vector<int> live, int jobs) {
  std::vector<std::vector<int>> out(std::max(0, jobs));
  std::sort(live.begin(), live.end());
  live.erase(std::unique(live.begin(), live.end()), live.end());
  const int n = (int)live.size();
  if (jobs <= 0 || n == 0) return out;
  for (int j = 0; j < jobs; ++j) {
    if (n >= jobs) {
      out[j].assign(live.begin() + (size_t)j * n / jobs, live.begin() + (size_t)(j + 1) * n / jobs);
    } else {
      out[j] = {live[j % n]};  // fewer GPUs than jobs: one GPU each, shared
    }
  }
  return out;
}

// ------------------------------------------------------------------ instance
// One model on one GPU: its worker, and per compute lane a staging batch,
// scratch and answer buffers. Direct queries queue here as requests and are
// coalesced into forwards (one lane each); a scattered query claims every
// lane of every instance of the partition for one group step at a time.
struct Fleet::Instance {
  struct Lane {
    void* batch = nullptr;
    void* aux = nullptr;
    void* aux_host = nullptr;
    void* ans = nullptr;       // [idx int32 x max][prob f32 x max]
    void* ans_host = nullptr;
    int ev = -1;
  };
  // A chunk (<= max images) of one direct query, queued for a forward.
  struct Req {
    const StageFn* stage = nullptr;
    int64_t first = 0;         // images [first, first + n) of its query
    int n = 0;
    int32_t* idx = nullptr;    // the caller's answers for this chunk
    float* prob = nullptr;
    std::chrono::steady_clock::time_point t0;
    int state = 0;             // 0 queued, 1 in a forward, 2 answered, 3 failed
    bool lost = false;         // failed because the device is lost (the query is redone)
    std::exception_ptr err;    // failed for another reason (rethrown to the caller)
    int off = 0;               // its first image's slot in the forward's batch
  };
  std::string model;
  int device;
  int max;
  size_t ib, aux_pi;
  std::unique_ptr<Worker> w;
  std::vector<Lane> lanes;
  std::mutex mu;
  std::condition_variable cv;
  std::vector<int> free;
  int claims = 0;
  std::deque<Req*> q;        // queued direct requests, oldest first (under mu)
  int64_t q_images = 0;
  int busy = 0;              // lanes running a direct forward (under mu)
  bool dead = false;         // a forward failed on an unhealthy device (under mu)
  std::atomic<int> outstanding{0};
  std::atomic<int64_t> served{0};
  std::atomic<int64_t> forwards{0};
  std::mutex sizes_mu;
  std::map<int, int64_t> sizes;  // direct forwards by (bucketed) batch size

  Instance(std::string m, int d, std::unique_ptr<Worker> worker, const FleetOptions& o)
      : model(std::move(m)), device(d), max(o.max_per_rank), ib(o.image_bytes), aux_pi(o.aux_bytes),
        w(std::move(worker)) {
    w->activate();
    for (int l = 0; l < w->lanes(); ++l) {
      Lane L;
      L.batch = w->alloc((size_t)max * o.image_bytes);
      if (o.aux_bytes) {
        L.aux = w->alloc(o.aux_bytes * max);
        L.aux_host = w->alloc_host(o.aux_bytes * max);
      }
      L.ans = w->alloc((size_t)max * 8);
      L.ans_host = w->alloc_host((size_t)max * 8);
      L.ev = w->new_event();
      lanes.push_back(L);
      free.push_back(l);
    }
  }
  ~Instance() {
    try {
      w->activate();
    } catch (...) {
    }
    w->sync_all_noexcept();
    for (auto& L : lanes) {
      w->dealloc(L.batch);
      if (L.aux) w->dealloc(L.aux);
      if (L.aux_host) w->dealloc_host(L.aux_host);
      w->dealloc(L.ans);
      w->dealloc_host(L.ans_host);
    }
  }
  // Scatter steps: queued direct requests go first (bounded, so a steady
  // stream of small queries cannot starve a scatter), then every lane.
  void claim_all() {
    std::unique_lock<std::mutex> g(mu);
    const auto until = std::chrono::steady_clock::now() + std::chrono::milliseconds(5);
    while (!(q.empty() || dead) && cv_wait_until(cv, g, until) != std::cv_status::timeout) {
    }
    ++claims;  // no new direct forward starts from here on
    cv.wait(g, [&] { return free.size() == lanes.size(); });
  }
  void release_all() {
    std::lock_guard<std::mutex> g(mu);
    --claims;
    cv.notify_all();
  }
};

struct Fleet::Model {
  std::string name;
  std::vector<int> devices;
  std::vector<std::shared_ptr<Instance>> inst;  // parallel to devices
  std::unique_ptr<Group> group;                 // partitions of >= 2 GPUs
  std::mutex group_mu;                          // one scattered query at a time
  // coordinator (inst[0]) staging of a scattered query
  void* gbatch = nullptr;
  void* gaux = nullptr;
  void* gaux_host = nullptr;
  int gev = -1;
  int64_t gcap = 0;
  std::atomic<uint32_t> rr{0};
  std::map<int, int64_t> retired;  // served by instances since dropped

  void drop_group(const FleetOptions& o) {
    if (!group) return;
    group.reset();
    Worker* w = inst.front()->w.get();
    w->sync_all_noexcept();
    w->dealloc(gbatch);
    if (gaux) w->dealloc(gaux);
    if (gaux_host) w->dealloc_host(gaux_host);
    gbatch = gaux = gaux_host = nullptr;
    gcap = 0;
    (void)o;
  }
};

// ------------------------------------------------------------------ fleet
Fleet::Fleet(std::vector<int> devices, WorkerFactory wf, CommFactory cf, FleetOptions opt)
    : devices_(std::move(devices)), wf_(std::move(wf)), cf_(std::move(cf)), opt_(opt) {
  if (devices_.empty()) throw std::invalid_argument("dp::Fleet: no devices");
  std::vector<int> s = devices_;
  std::sort(s.begin(), s.end());
  if (std::adjacent_find(s.begin(), s.end()) != s.end()) throw std::invalid_argument("dp::Fleet: duplicate device");
  if (opt_.max_per_rank < 1 || opt_.min_shard < 1) throw std::invalid_argument("dp::Fleet: bad options");
}

Fleet::~Fleet() {
  std::unique_lock<std::shared_mutex> lk(plan_mu_);
  for (auto& kv : models_) {
    Model& m = *kv.second;
    if (!m.inst.empty()) m.drop_group(opt_);
    m.inst.clear();
  }
  models_.clear();
}

void Fleet::set_jobs(const std::vector<std::string>& models) {
  {
    std::unique_lock<std::shared_mutex> lk(plan_mu_);
    jobs_ = models;
  }
  dirty_ = true;
  rebalance();
}

bool Fleet::has(const std::string& model) const {
  std::shared_lock<std::shared_mutex> lk(plan_mu_);
  return models_.count(model) > 0;
}

Fleet::Model& Fleet::get(const std::string& model) const {
  auto it = models_.find(model);
  if (it == models_.end()) throw std::runtime_error("model not loaded: " + model);
  return *it->second;
}

std::vector<std::string> Fleet::order_locked() const {
  std::vector<std::string> o;
  for (const auto& m : jobs_)
    if (models_.count(m) && std::find(o.begin(), o.end(), m) == o.end()) o.push_back(m);
  for (const auto& m : loaded_)
    if (models_.count(m) && std::find(o.begin(), o.end(), m) == o.end()) o.push_back(m);
  return o;
}

std::vector<int> Fleet::live() const {
  std::lock_guard<std::mutex> g(lost_mu_);
  std::vector<int> l;
  for (int d : devices_)
    if (!lost_.count(d)) l.push_back(d);
  return l;
}

std::vector<std::vector<int>> Fleet::plan_locked() const {
  return partition_devices(live(), (int)order_locked().size());
}

std::map<std::string, std::vector<int>> Fleet::partitions() const {
  std::shared_lock<std::shared_mutex> lk(plan_mu_);
  std::map<std::string, std::vector<int>> out;
  for (const auto& kv : models_) out[kv.first] = kv.second->devices;
  return out;
}

std::map<int, int64_t> Fleet::forwards(const std::string& model) const {
  std::shared_lock<std::shared_mutex> lk(plan_mu_);
  const Model& m = get(model);
  std::map<int, int64_t> out;
  for (const auto& i : m.inst) out[i->device] += i->forwards.load();
  return out;
}

std::map<int, int64_t> Fleet::forward_sizes(const std::string& model) const {
  std::shared_lock<std::shared_mutex> lk(plan_mu_);
  const Model& m = get(model);
  std::map<int, int64_t> out;
  for (const auto& i : m.inst) {
    std::lock_guard<std::mutex> g(i->sizes_mu);
    for (const auto& kv : i->sizes) out[kv.first] += kv.second;
  }
  return out;
}

std::map<int, int64_t> Fleet::served(const std::string& model) const {
  std::shared_lock<std::shared_mutex> lk(plan_mu_);
  const Model& m = get(model);
  std::map<int, int64_t> out = m.retired;
  for (const auto& i : m.inst) out[i->device] += i->served.load();
  return out;
}

Worker* Fleet::worker(const std::string& model, int device) const {
  std::shared_lock<std::shared_mutex> lk(plan_mu_);
  const Model& m = get(model);
  for (const auto& i : m.inst)
    if (i->device == device) return i->w.get();
  return nullptr;
}

std::shared_ptr<Fleet::Instance> Fleet::make_instance(const std::string& model, int device, Worker* replica_of) {
  auto w = wf_(model, device, replica_of);
  if (!w) throw std::runtime_error("dp::Fleet: worker factory returned nothing for " + model);
  if (w->device() != device) throw std::runtime_error("dp::Fleet: worker on the wrong device");
  return std::make_shared<Instance>(model, device, std::move(w), opt_);
}

// `train`'s weight distribution: one RCCL broadcast of
// the packed arena from a live instance into the new replicas over xGMI.
void Fleet::broadcast_weights(Instance& src, const std::vector<Instance*>& dst) {
  if (dst.empty()) return;
  const size_t bytes = src.w->weight_bytes();
  std::vector<int> devs{src.device};
  for (Instance* d : dst) {
    if (d->w->weight_bytes() != bytes) throw std::runtime_error("dp::Fleet: replica weight size differs");
    devs.push_back(d->device);
  }
  if (bytes == 0) return;
  auto comms = cf_(devs);
  if (comms.size() != devs.size()) throw std::runtime_error("dp::Fleet: communicator factory returned the wrong size");
  comms[0]->group_start();
  try {
    for (size_t k = 0; k < devs.size(); ++k) {
      Worker* w = k == 0 ? src.w.get() : dst[k - 1]->w.get();
      w->activate();
      comms[k]->broadcast(src.w->weight_arena(), w->weight_arena(), bytes, 0, w->stream(Worker::kIn));
    }
  } catch (...) {
    comms[0]->group_end();
    throw;
  }
  comms[0]->group_end();
  src.w->sync_all();
  for (Instance* d : dst) {
    d->w->sync_all();
    d->w->weights_updated();
    d->w->sync_all();
  }
}

void Fleet::apply_locked(Model& m, const std::vector<int>& devs, std::vector<std::shared_ptr<Instance>> fresh) {
  std::set<int> lost;
  {
    std::lock_guard<std::mutex> g(lost_mu_);
    lost = lost_;
  }
  bool same = fresh.empty() && devs == m.devices && m.inst.size() == devs.size() &&
              (devs.size() < 2 || (m.group && m.gcap > 0));
  for (const auto& i : m.inst) same = same && !lost.count(i->device);
  if (same) return;

  // Nothing of `m` changes until the new instances exist (a failed build or
  // broadcast leaves the old plan in place, marked dirty by rebalance()).
  if (!m.inst.empty()) m.drop_group(opt_);
  std::vector<std::shared_ptr<Instance>> next(devs.size());
  if (!fresh.empty()) {
    next = std::move(fresh);
  } else {
    std::map<int, std::shared_ptr<Instance>> kept;
    for (auto& i : m.inst)
      if (!lost.count(i->device) && std::find(devs.begin(), devs.end(), i->device) != devs.end())
        kept[i->device] = i;
    std::shared_ptr<Instance> src = kept.empty() ? nullptr : kept.begin()->second;
    std::vector<Instance*> need;
    for (size_t k = 0; k < devs.size(); ++k) {
      auto it = kept.find(devs[k]);
      if (it != kept.end()) {
        next[k] = it->second;
      } else if (!src) {
        next[k] = make_instance(m.name, devs[k], nullptr);  // from the host weights
        src = next[k];
      } else {
        next[k] = make_instance(m.name, devs[k], src->w.get());
        need.push_back(next[k].get());
      }
    }
    if (src) broadcast_weights(*src, need);
  }
  for (auto& i : m.inst)  // keep the per-device counts of dropped instances
    if (std::find(next.begin(), next.end(), i) == next.end()) m.retired[i->device] += i->served.load();
  m.inst = std::move(next);  // dropped instances are destroyed here (nothing in flight)
  m.devices = devs;
  if (devs.size() > 1) {
    std::vector<Worker*> ws;
    for (auto& i : m.inst) ws.push_back(i->w.get());
    auto cf = cf_;
    auto d = devs;
    auto factory = [cf, d](const std::vector<int>& members) {
      std::vector<int> sub;
      for (int x : members) sub.push_back(d.at(x));
      return cf(sub);
    };
    m.group = std::make_unique<Group>(ws, factory, opt_.max_per_rank, opt_.image_bytes, opt_.timeout_ms);
    m.group->set_min_per_rank(opt_.min_shard);
    Worker* w = ws.front();
    w->activate();
    m.gcap = (int64_t)opt_.max_per_rank * (int64_t)devs.size();
    m.gbatch = w->alloc((size_t)m.gcap * opt_.image_bytes);
    if (opt_.aux_bytes) {
      m.gaux = w->alloc(opt_.aux_bytes * (size_t)m.gcap);
      m.gaux_host = w->alloc_host(opt_.aux_bytes * (size_t)m.gcap);
    }
    m.gev = w->new_event();
  }
}

void Fleet::rebalance() {
  std::unique_lock<std::shared_mutex> lk(plan_mu_);
  dirty_ = false;
  try {
    const auto order = order_locked();
    const auto plan = partition_devices(live(), (int)order.size());
    // every group whose partition changes goes first, so the broadcast of a
    // moved GPU's new weights never shares a device with a live group of
    // another model
    for (size_t j = 0; j < order.size(); ++j) {
      Model& m = *models_.at(order[j]);
      if (m.devices != plan[j] && !m.inst.empty()) m.drop_group(opt_);
    }
    for (size_t j = 0; j < order.size(); ++j) apply_locked(*models_.at(order[j]), plan[j]);
  } catch (...) {
    // a model whose instances or group could not be (re)built keeps its old
    // instances without a group (queries run direct); the next query retries
    dirty_ = true;
    throw;
  }
  ++rebalances_;
}

void Fleet::mark_lost(int device) {
  {
    std::lock_guard<std::mutex> g(lost_mu_);
    lost_.insert(device);
  }
  dirty_ = true;
}

void Fleet::lose(int device) {
  if (std::find(devices_.begin(), devices_.end(), device) == devices_.end())
    throw std::invalid_argument("dp::Fleet::lose: not a device of this fleet");
  mark_lost(device);
  rebalance();
}

void Fleet::load(const std::string& model) {
  std::lock_guard<std::mutex> lg(load_mu_);
  std::vector<int> devs;
  bool exists;
  {
    std::shared_lock<std::shared_mutex> lk(plan_mu_);
    exists = models_.count(model) > 0;
    if (exists) devs = models_.at(model)->devices;
  }
  if (!exists) {  // a new job: every partition is recomputed
    {
      std::unique_lock<std::shared_mutex> lk(plan_mu_);
      auto m = std::make_unique<Model>();
      m->name = model;
      models_[model] = std::move(m);
      loaded_.push_back(model);
    }
    dirty_ = true;
    rebalance();
    return;
  }
  // Hot swap: the new instances are built (host weights on the first GPU,
  // replicas on the others) while queries still run on the old ones.
  std::vector<std::shared_ptr<Instance>> fresh;
  for (size_t k = 0; k < devs.size(); ++k) fresh.push_back(make_instance(model, devs[k], k ? fresh[0]->w.get() : nullptr));
  std::unique_lock<std::shared_mutex> lk(plan_mu_);
  Model& m = *models_.at(model);
  bool ok = m.devices == devs && !fresh.empty();
  {
    std::lock_guard<std::mutex> g(lost_mu_);
    for (int d : devs) ok = ok && !lost_.count(d);
  }
  if (ok) {
    std::vector<Instance*> rep;
    for (size_t k = 1; k < fresh.size(); ++k) rep.push_back(fresh[k].get());
    broadcast_weights(*fresh[0], rep);
    apply_locked(m, devs, std::move(fresh));
  } else {
    // the partition moved meanwhile: rebuild it from the host weights
    fresh.clear();
    if (!m.inst.empty()) m.drop_group(opt_);
    for (auto& i : m.inst) m.retired[i->device] += i->served.load();
    m.inst.clear();
    m.devices.clear();
    const auto order = order_locked();
    const auto plan = partition_devices(live(), (int)order.size());
    for (size_t j = 0; j < order.size(); ++j)
      if (order[j] == model) apply_locked(m, plan[j]);
  }
}

// ------------------------------------------------------------------ queries
Fleet::Route Fleet::classify(const std::string& model, int64_t n, const StageFn& stage, int32_t* idx, float* prob,
                             QueryOptions q) {
  Route r;
  if (n <= 0) return r;
  int retries = 0;
  for (;;) {
    if (dirty_.load()) rebalance();
    try {
      std::shared_lock<std::shared_mutex> lk(plan_mu_);
      Model& m = get(model);
      if (m.inst.empty()) throw std::runtime_error("fleet: no live GPU serves " + model);
      const bool scatter =
          q.allow_scatter && m.inst.size() > 1 && m.group && m.gcap > 0 && n >= 2 * (int64_t)opt_.min_shard;
      r = scatter ? scattered(m, n, stage, idx, prob) : direct(m, n, stage, idx, prob, q.prefer_device);
    } catch (const DeviceLost&) {
      if (++retries > (int)devices_.size()) throw std::runtime_error("fleet: query failed on every GPU");
      continue;  // redo the whole query on the rebalanced fleet
    }
    r.retries = retries;
    if (dirty_.load()) rebalance();  // a scattered query dropped a GPU: rebalance now
    return r;
  }
}

// Forward batch of b coalesced images: the next power of two up to 64, then
// the next multiple of 32 (at most max). A bounded set of captured graphs per
// lane (7 + (max - 64) / 32), and above 64 images a forward pads at most 31
// (a 129-image forward runs 160, not 256).
int bucket_batch(int b, int max) {
  int p = 1;
  while (p < b && p < 64) p <<= 1;
  if (b > 64) p = (b + 31) / 32 * 32;
  return std::min(p, max);
}

Fleet::Route Fleet::direct(Model& m, int64_t n, const StageFn& stage, int32_t* idx, float* prob, int prefer) {
  // least outstanding queries; ties rotate so equal load spreads evenly; the
  // GPU holding the query's data wins a tie
  const size_t k0 = m.rr.fetch_add(1) % m.inst.size();
  Instance* best = nullptr;
  int bq = INT_MAX;
  for (size_t i = 0; i < m.inst.size(); ++i) {
    Instance* c = m.inst[(k0 + i) % m.inst.size()].get();
    const int q = c->outstanding.load();
    if (q < bq) {
      bq = q;
      best = c;
    }
  }
  for (auto& c : m.inst)
    if (c->device == prefer && c->outstanding.load() <= bq) best = c.get();
  Instance& in = *best;
  ++in.outstanding;
  struct Dec {
    std::atomic<int>& a;
    ~Dec() { --a; }
  } dec{in.outstanding};
  Worker* w = in.w.get();
  const int max = in.max;
  const auto window = std::chrono::microseconds(std::max(0, opt_.batch_window_us));

  using Req = Instance::Req;
  std::vector<Req> reqs((size_t)((n + max - 1) / max));
  const auto now0 = std::chrono::steady_clock::now();
  for (size_t k = 0; k < reqs.size(); ++k) {
    Req& r = reqs[k];
    r.stage = &stage;
    r.first = (int64_t)k * max;
    r.n = (int)std::min<int64_t>(max, n - r.first);
    r.idx = idx + r.first;
    r.prob = prob + r.first;
    r.t0 = now0;
  }
  struct Flight {
    int lane;
    std::vector<Req*> batch;
  };
  std::deque<Flight> mine;  // forwards this caller issued, oldest first; it finishes every one of them

  std::unique_lock<std::mutex> g(in.mu);
  for (Req& r : reqs) {
    in.q.push_back(&r);
    in.q_images += r.n;
  }
  in.cv.notify_all();
  auto fail_queue = [&]() {  // the device is gone: every queued request is redone elsewhere
    for (Req* r : in.q) {
      r->state = 3;
      r->lost = true;
    }
    in.q.clear();
    in.q_images = 0;
    in.cv.notify_all();
  };
  auto ready = [&]() {
    if (in.q.empty() || in.claims > 0 || in.free.empty() || in.dead) return false;
    return in.q_images >= max || window.count() == 0 || (opt_.eager_when_idle && in.busy == 0) ||
           std::chrono::steady_clock::now() >= in.q.front()->t0 + window;
  };
  auto all_done = [&]() {
    for (const Req& r : reqs)
      if (r.state < 2) return false;
    return true;
  };

  for (;;) {
    if (in.dead) fail_queue();
    // issue every ready forward, each on its own free lane
    while (ready()) {
      Flight f;
      f.lane = in.free.back();
      in.free.pop_back();
      ++in.busy;
      int B = 0;
      while (!in.q.empty() && B + in.q.front()->n <= max) {
        Req* r = in.q.front();
        in.q.pop_front();
        in.q_images -= r->n;
        r->state = 1;
        r->off = B;
        B += r->n;
        f.batch.push_back(r);
      }
      g.unlock();
      // stage every request into the lane's batch back to back, then one
      // forward and one answer copy for all of them
      auto& L = in.lanes[f.lane];
      const int cs = Worker::compute_stream(f.lane);
      bool issued = false;
      std::vector<std::pair<Req*, std::exception_ptr>> failed;  // stage errors, published under in.mu
      auto publish_failed = [&]() {  // holds in.mu
        for (auto& fr : failed) {
          fr.first->err = fr.second;
          fr.first->state = 3;
        }
        failed.clear();
      };
      try {
        w->activate();
        int off = 0;
        std::vector<Req*> kept;
        kept.reserve(f.batch.size());
        for (Req* r : f.batch) {
          StageCtx ctx;
          ctx.worker = w;
          ctx.device = in.device;
          ctx.stream = cs;
          ctx.batch = (uint8_t*)L.batch + (size_t)off * in.ib;
          ctx.capacity = max - off;
          ctx.aux = L.aux ? (uint8_t*)L.aux + (size_t)off * in.aux_pi : nullptr;
          ctx.aux_host = L.aux_host ? (uint8_t*)L.aux_host + (size_t)off * in.aux_pi : nullptr;
          const uint8_t* p = nullptr;
          try {
            p = (*r->stage)(ctx, r->first, r->n);
          } catch (...) {
            if (!w->healthy()) throw;
            // this request only. Its owner may return (and free it) as soon
            // as it sees state 3, so the failure is published under in.mu
            // below and the request leaves this forward's batch now: nothing
            // here touches it after the publish.
            failed.emplace_back(r, std::current_exception());
            continue;
          }
          // the lane's own buffer, so the graph key (batch address, bucket) is fixed per lane
          if (p != ctx.batch) w->copy(ctx.batch, p, (size_t)r->n * in.ib, cs);
          r->off = off;
          off += r->n;
          kept.push_back(r);
        }
        f.batch.swap(kept);
        if (off > 0) {
          const int Bf = opt_.bucket_batches ? bucket_batch(off, max) : off;
          auto* a = (uint8_t*)L.ans;
          w->classify((const uint8_t*)L.batch, Bf, (int32_t*)a, (float*)(a + (size_t)max * 4), f.lane);
          w->copy_d2h(L.ans_host, L.ans, (size_t)max * 8, cs);
          in.forwards++;
          std::lock_guard<std::mutex> sg(in.sizes_mu);
          in.sizes[Bf]++;
        }
        w->record(L.ev, cs);
        issued = true;
      } catch (...) {
        const bool lost = !w->healthy();
        const auto err = std::current_exception();
        g.lock();
        publish_failed();
        for (Req* r : f.batch)
          if (r->state == 1) {
            r->state = 3;
            r->lost = lost;
            if (!lost) r->err = err;
          }
        if (lost) in.dead = true;
        in.free.push_back(f.lane);
        --in.busy;
        in.cv.notify_all();
        continue;
      }
      g.lock();
      publish_failed();
      in.cv.notify_all();  // owners of failed requests
      if (issued) mine.push_back(std::move(f));
    }
    if (!mine.empty()) {  // finish my oldest forward
      Flight f = std::move(mine.front());
      mine.pop_front();
      g.unlock();
      auto& L = in.lanes[f.lane];
      bool lost = false;
      std::exception_ptr err;
      try {
        w->sync(L.ev);
        const auto* h = (const uint8_t*)L.ans_host;
        for (Req* r : f.batch)
          if (r->state == 1) {
            std::memcpy(r->idx, h + (size_t)r->off * 4, (size_t)r->n * 4);
            std::memcpy(r->prob, h + (size_t)max * 4 + (size_t)r->off * 4, (size_t)r->n * 4);
          }
      } catch (...) {
        lost = !w->healthy();
        err = std::current_exception();
      }
      g.lock();
      int64_t answered = 0;
      for (Req* r : f.batch)
        if (r->state == 1) {
          if (err) {
            r->state = 3;
            r->lost = lost;
            if (!lost) r->err = err;
          } else {
            r->state = 2;
            answered += r->n;
          }
        }
      in.served += answered;
      if (lost) in.dead = true;
      in.free.push_back(f.lane);
      --in.busy;
      in.cv.notify_all();
      continue;
    }
    if (all_done()) break;
    // wait for: a lane, my requests answered by another caller's forward, or
    // the batching window of the oldest queued request
    if (!in.q.empty() && in.claims == 0 && !in.free.empty() && !in.dead)
      cv_wait_until(in.cv, g, in.q.front()->t0 + window);
    else
      in.cv.wait(g);
  }
  g.unlock();
  for (const Req& r : reqs)
    if (r.lost) {
      mark_lost(in.device);
      throw DeviceLost{in.device};
    }
  for (const Req& r : reqs)
    if (r.err) std::rethrow_exception(r.err);
  Route r;
  r.device = in.device;
  return r;
}

Fleet::Route Fleet::scattered(Model& m, int64_t n, const StageFn& stage, int32_t* idx, float* prob) {
  std::lock_guard<std::mutex> g(m.group_mu);
  Instance& c = *m.inst.front();
  Worker* w = c.w.get();
  Route r;
  r.scattered = true;
  r.device = c.device;
  r.devices_used = 0;
  try {
    // one group classify (<= gcap images: one step per lane of each GPU) at
    // a time, every lane claimed only for it: direct queries queued
    // meanwhile run between the steps of a long scatter
    for (int64_t first = 0; first < n; first += m.gcap) {
      for (auto& i : m.inst) i->claim_all();
      struct Release {
        Model& m;
        ~Release() {
          for (auto& i : m.inst) i->release_all();
        }
      } rel{m};
      const int64_t cnt = std::min<int64_t>(m.gcap, n - first);
      w->activate();
      StageCtx ctx;
      ctx.worker = w;
      ctx.device = c.device;
      ctx.stream = Worker::kCompute;
      ctx.batch = m.gbatch;
      ctx.capacity = m.gcap;
      ctx.aux = m.gaux;
      ctx.aux_host = m.gaux_host;
      const uint8_t* img = stage(ctx, first, cnt);
      w->record(m.gev, Worker::kCompute);
      // returns once every answer is on the host (so the stage has run)
      const Group::Stats st = m.group->classify(img, cnt, idx + first, prob + first, m.gev);
      for (size_t k = 0; k < st.per_worker.size() && k < m.inst.size(); ++k) {
        m.inst[k]->served += st.per_worker[k];
        r.devices_used = std::max(r.devices_used, st.ranks_used);
      }
    }
  } catch (const comm::CommError&) {
    // dp::Group recovers from a lost member itself; it throws when the
    // coordinator is gone (or on an error no member explains)
    if (!w->healthy()) {
      mark_lost(c.device);
      throw DeviceLost{c.device};
    }
    throw;
  }
  const auto mem = m.group->members();  // members it dropped are lost GPUs
  for (size_t i = 0; i < m.inst.size(); ++i)
    if (std::find(mem.begin(), mem.end(), (int)i) == mem.end()) mark_lost(m.inst[i]->device);
  return r;
}

}  // namespace dp
}  // namespace dmlc
