#include "leader.h"

#include "../runtime/trace.h"

#include <climits>
#include <optional>

#include "../control/common.h"

namespace dmlc {
namespace ctl {

LeaderService::LeaderService(LeaderConfig cfg, MembershipService* ms, MemberService* member, Labels labels)
    : cfg_(std::move(cfg)), ms_(ms), member_(member), labels_(std::move(labels)) {
  for (const auto& m : cfg_.job_models) {
    Job j;
    j.model_name = m;
    jobs_.push_back(j);
  }
  running_.assign(jobs_.size(), false);
  retry_.resize(jobs_.size());
  segs_.resize(jobs_.size());
  job_inflight_.reset(new std::atomic<int>[jobs_.size()]);
  for (size_t j = 0; j < jobs_.size(); ++j) job_inflight_[j] = 0;
}

Id LeaderService::pick_target(const std::vector<Id>& all) {
  std::lock_guard<std::mutex> g(rng_mu_);
  // members benched after a failure sit out unless nobody else is left
  std::vector<Id> pool;
  for (const auto& id : all)
    if (!benched(id.address)) pool.push_back(id);
  if (pool.empty()) pool = all;
  if (cfg_.adaptive_window <= 0)  // reference: a random member (src/services.rs:414-416)
    return pool[std::uniform_int_distribution<size_t>(0, pool.size() - 1)(rng_)];
  // least outstanding queries; ties broken at random so load spreads evenly
  int best = INT_MAX;
  std::vector<size_t> ties;
  for (size_t i = 0; i < pool.size(); ++i) {
    auto it = member_inflight_.find(pool[i].address);
    const int q = it == member_inflight_.end() ? 0 : it->second;
    if (q < best) {
      best = q;
      ties.assign(1, i);
    } else if (q == best) {
      ties.push_back(i);
    }
  }
  return pool[ties[std::uniform_int_distribution<size_t>(0, ties.size() - 1)(rng_)]];
}

LeaderService::~LeaderService() { stop(); }

void LeaderService::start(int base_port) {
  self_ = ms_->id().address;
  server_ = std::make_unique<RpcServer>("leader", cfg_.bind_host, leader_port(base_port));
  register_handlers();
  server_->start();
  loops_.emplace_back([this] { rereplicate_loop(); });
  loops_.emplace_back([this] { assign_loop(); });
  loops_.emplace_back([this] { succession_loop(); });
  loops_.emplace_back([this] { standby_copy_loop(); });
}

void LeaderService::stop() {
  if (stop_.exchange(true)) return;
  for (auto& t : loops_)
    if (t.joinable()) t.join();
  {
    std::lock_guard<std::mutex> g(runners_mu_);
    for (auto& t : runners_)
      if (t.joinable()) t.join();
  }
  {
    std::lock_guard<std::mutex> g(pool_mu_);
    pool_stop_ = true;
  }
  pool_cv_.notify_all();
  for (auto& t : workers_)
    if (t.joinable()) t.join();
  if (server_) server_->stop();
}

bool LeaderService::is_leader() const { return member_->leader_address() == self_; }

void LeaderService::sleep_bg() {
  for (int slept = 0; slept < cfg_.bg_ms && !stop_.load(); slept += 50)
    std::this_thread::sleep_for(std::chrono::milliseconds(50));
}

int LeaderService::latest_version(const std::string& f) const {
  std::lock_guard<std::mutex> g(mu_);
  auto it = dir_.find(f);
  int v = 0;
  if (it == dir_.end()) return 0;
  for (const auto& r : it->second)
    if (!r.second.empty()) v = std::max(v, *r.second.rbegin());
  return v;
}

bool LeaderService::copy_to(const Id& src, const std::string& src_spec, const Id& dest, const std::string& dest_spec) {
  try {
    Writer w;
    w.str(src.host()).i32(member_port(src.port())).str(src_spec).str(dest_spec);
    const std::string resp =
        RpcClient::shared().call(dest.host(), member_port(dest.port()), M_FETCH, w.data(), 3600 * 1000);
    Reader r(resp);
    const bool ok = r.boolean();
    DMLC_LOG_INFO("copy " << src.address << ":" << src_spec << " -> " << dest.address << ":" << dest_spec << ": "
                          << (ok ? "ok" : "failed"));
    return ok;
  } catch (const std::exception& e) {
    DMLC_LOG_WARN("copy " << src.address << ":" << src_spec << " -> " << dest.address << ":" << dest_spec
                          << ": " << e.what());
    return false;
  }
}

std::set<Id> LeaderService::put_version(const Id* src_id, const std::string* src_spec, const std::string& filename,
                                        int version) {
  if (version == 0) return {};
  const std::set<Id> active = ms_->active_ids();
  if (active.empty()) return {};
  std::set<Id> current;
  {
    std::lock_guard<std::mutex> g(mu_);
    auto it = dir_.find(filename);
    if (it != dir_.end())
      for (const auto& r : it->second)
        if (active.count(r.first) && r.second.count(version)) current.insert(r.first);
  }
  if ((int)current.size() >= cfg_.replication) return current;
  Id sid;
  std::string sspec;
  if (src_id) {
    sid = *src_id;
    sspec = *src_spec;
  } else if (!current.empty()) {
    sid = *current.begin();
    sspec = "storage:" + storage_filename(filename, version);
  } else {
    DMLC_LOG_WARN("put_version: no source and no live replica of " << filename << " v" << version
                                                                   << "; the file may be lost");
    return current;
  }
  std::vector<Id> candidates;
  for (const auto& id : active)
    if (!current.count(id)) candidates.push_back(id);
  if (candidates.empty()) return current;
  const std::set<Id> targets = choose_replicas(filename, candidates, cfg_.replication - (int)current.size());
  const std::string dest_spec = "storage:" + storage_filename(filename, version);
  std::mutex rmu;
  std::set<Id> received;
  std::vector<std::thread> ts;
  for (const Id& d : targets) {
    ts.emplace_back([&, d] {
      if (!copy_to(sid, sspec, d, dest_spec)) return;
      try {
        Writer w;
        w.str(filename).i32(version);
        RpcClient::shared().call(d.host(), member_port(d.port()), M_RECEIVE, w.data(), 10000);
        std::lock_guard<std::mutex> g(rmu);
        received.insert(d);
      } catch (const std::exception& e) {
        DMLC_LOG_WARN("put_version: receive on " << d.address << " failed: " << e.what());
      }
    });
  }
  for (auto& t : ts) t.join();
  {
    std::lock_guard<std::mutex> g(mu_);
    auto& m = dir_[filename];
    for (const auto& id : received) m[id].insert(version);
  }
  std::set<Id> all = current;
  all.insert(received.begin(), received.end());
  return all;
}

std::set<Id> LeaderService::put(const Id& src, const std::string& src_path, const std::string& filename) {
  const int version = latest_version(filename) + 1;
  return put_version(&src, &src_path, filename, version);
}

std::optional<Id> LeaderService::get_version(const std::string& filename, int version, const Id& dest,
                                             const std::string& dest_spec) {
  if (version == 0) return std::nullopt;
  std::vector<Id> srcs;
  {
    std::lock_guard<std::mutex> g(mu_);
    auto it = dir_.find(filename);
    if (it != dir_.end())
      for (const auto& r : it->second)
        if (r.second.count(version)) srcs.push_back(r.first);
  }
  for (const auto& s : srcs)
    if (copy_to(s, "storage:" + storage_filename(filename, version), dest, dest_spec)) return s;
  return std::nullopt;
}

int LeaderService::get(const std::string& filename, const Id& dest, const std::string& dest_path) {
  const int v = latest_version(filename);
  return get_version(filename, v, dest, dest_path) ? v : 0;
}

std::set<int> LeaderService::get_versions(const std::string& filename, int count, const Id& dest,
                                          const std::string& dest_path) {
  const int latest = latest_version(filename);
  std::set<int> out;
  if (latest == 0 || count <= 0) return out;
  std::mutex omu;
  std::vector<std::thread> ts;
  for (int v = latest; v >= 1 && v > latest - count; --v) {
    ts.emplace_back([&, v] {
      if (get_version(filename, v, dest, versioned_sibling(dest_path, v))) {
        std::lock_guard<std::mutex> g(omu);
        out.insert(v);
      }
    });
  }
  for (auto& t : ts) t.join();
  return out;
}

void LeaderService::del(const std::string& filename) {
  std::set<Id> holders;
  {
    std::lock_guard<std::mutex> g(mu_);
    auto it = dir_.find(filename);
    if (it != dir_.end())
      for (const auto& r : it->second) holders.insert(r.first);
    dir_.erase(filename);
  }
  for (const auto& id : holders) {  // also drop the replica files (reference kept them)
    try {
      Writer w;
      w.str(filename);
      RpcClient::shared().call(id.host(), member_port(id.port()), M_DELETE_FILE, w.data(), 5000);
    } catch (const std::exception&) {
    }
  }
}

std::vector<std::pair<Id, std::vector<int>>> LeaderService::ls(const std::string& filename) {
  const std::set<Id> active = ms_->active_ids();
  std::vector<std::pair<Id, std::vector<int>>> out;
  std::lock_guard<std::mutex> g(mu_);
  auto it = dir_.find(filename);
  if (it == dir_.end()) return out;
  for (const auto& r : it->second)
    if (active.count(r.first)) out.emplace_back(r.first, std::vector<int>(r.second.begin(), r.second.end()));
  return out;
}

void LeaderService::train(const std::string& filename, const std::string& model_name) {
  const int v = latest_version(filename);
  if (v == 0) throw std::runtime_error("file not found: " + filename);
  const std::string spec = "models:" + model_name + ".ot";
  std::vector<std::thread> ts;
  std::mutex emu;
  std::vector<std::string> errors;
  for (const Id& id : ms_->active_ids()) {
    ts.emplace_back([&, id] {
      std::string err;
      if (!get_version(filename, v, id, spec)) {
        err = id.address + ": copy failed";
      } else {
        try {
          Writer w;
          w.str(model_name).str(spec);
          Reader r(RpcClient::shared().call(id.host(), member_port(id.port()), M_LOAD_MODEL, w.data(), 600000));
          if (!r.boolean()) err = id.address + ": " + r.str();
        } catch (const std::exception& e) {
          err = id.address + ": " + e.what();
        }
      }
      if (!err.empty()) {
        std::lock_guard<std::mutex> g(emu);
        errors.push_back(err);
      }
    });
  }
  for (auto& t : ts) t.join();
  if (!errors.empty()) {
    std::string s;
    for (const auto& e : errors) s += (s.empty() ? "" : "; ") + e;
    throw std::runtime_error(s);
  }
  // New weights: that model's job starts over, so the next `predict`
  // classifies the dataset with them (the reference never reloaded models
  // after `train`, src/services.rs:139-144 vs :513-524).
  std::lock_guard<std::mutex> g(mu_);
  for (size_t j = 0; j < jobs_.size(); ++j)
    if (jobs_[j].model_name == model_name && !running_[j]) {
      Job fresh;
      fresh.model_name = model_name;
      fresh.assigned = jobs_[j].assigned;
      jobs_[j] = std::move(fresh);
    }
}

std::vector<std::string> LeaderService::predict(const std::vector<std::string>* shards) {
  std::lock_guard<std::mutex> g(runners_mu_);
  std::vector<std::string> notes;
  for (size_t j = 0; j < jobs_.size(); ++j) {
    {
      std::lock_guard<std::mutex> g2(mu_);
      if (running_[j]) {
        if (shards && jobs_[j].source != *shards)
          notes.push_back("job " + jobs_[j].model_name + " is still running on its previous source; it keeps it");
        continue;
      }
      if (shards && jobs_[j].source != *shards) {  // another data source: the job starts over
        Job fresh;
        fresh.model_name = jobs_[j].model_name;
        fresh.assigned = jobs_[j].assigned;
        fresh.source = *shards;
        jobs_[j] = std::move(fresh);
      }
      running_[j] = true;
    }
    runners_.emplace_back([this, j] { run_job(j); });
  }
  return notes;
}

std::vector<Id> LeaderService::shard_holders(const std::string& file) {
  const int v = latest_version(file);
  const auto active = ms_->active_ids();
  std::vector<Id> out;
  std::lock_guard<std::mutex> g(mu_);
  auto it = dir_.find(file);
  if (it == dir_.end()) return out;
  for (const auto& rep : it->second)
    if (rep.second.count(v) && active.count(rep.first)) out.push_back(rep.first);
  return out;
}

// The job's shards: size and first label of each, from a live replica holder
// (M_SHARD_INFO); the job's index space is the shards back to back.
bool LeaderService::load_segments(size_t j, const std::vector<std::string>& source) {
  std::vector<Seg> segs;
  size_t start = 0;
  for (const auto& f : source) {
    bool got = false;
    std::string why = "no live replica holder";
    for (const Id& h : shard_holders(f)) {
      try {
        Writer w;
        w.str(f);
        Reader r(RpcClient::shared().call(h.host(), member_port(h.port()), M_SHARD_INFO, w.data(), 10000));
        (void)r.i32();  // version
        Seg sg;
        sg.file = f;
        sg.start = start;
        sg.n = r.u32();
        (void)r.u32();
        (void)r.u32();
        sg.label0 = r.u32();
        if (!r.boolean()) {
          why = "not a labelled shard";
          break;
        }
        if ((size_t)sg.label0 + sg.n > labels_.entries.size()) {
          why = "labels beyond the label table";
          break;
        }
        start += sg.n;
        segs.push_back(sg);
        got = true;
        break;
      } catch (const std::exception& e) {
        why = h.address + ": " + e.what();
      }
    }
    if (!got) {
      DMLC_LOG_WARN("job over shards: " << f << ": " << why);
      out_line("predict: shard " + f + ": " + why);
      return false;
    }
  }
  std::lock_guard<std::mutex> g(mu_);
  segs_[j] = std::move(segs);
  return true;
}

std::vector<Job> LeaderService::jobs() const {
  std::lock_guard<std::mutex> g(mu_);
  return jobs_;
}

// Fixed pool of query workers (instead of one detached thread per query).
void LeaderService::submit(std::function<void()> task) {
  std::unique_lock<std::mutex> g(pool_mu_);
  if (workers_.empty()) {
    const int n = std::max(1, std::min(cfg_.max_inflight, 256));
    for (int i = 0; i < n; ++i)
      workers_.emplace_back([this] {
        for (;;) {
          std::function<void()> t;
          {
            std::unique_lock<std::mutex> lk(pool_mu_);
            pool_cv_.wait(lk, [&] { return pool_stop_ || !tasks_.empty(); });
            if (tasks_.empty()) return;  // stopping and drained
            t = std::move(tasks_.front());
            tasks_.pop_front();
          }
          t();
        }
      });
  }
  tasks_.push_back(std::move(task));
  pool_cv_.notify_one();
}

bool LeaderService::benched(const std::string& addr) {  // under rng_mu_
  auto it = bench_until_.find(addr);
  if (it == bench_until_.end()) return false;
  if (steady_us() >= it->second) {
    bench_until_.erase(it);
    return false;
  }
  return true;
}

std::optional<Id> LeaderService::retry_target(size_t j, const std::set<std::string>& tried,
                                               const std::vector<Id>* only) {
  std::vector<Id> pool;
  {
    std::lock_guard<std::mutex> g(mu_);
    pool = jobs_[j].assigned;  // the job's own members first
  }
  if (only) {  // shard queries: replica holders only, the job's own first
    std::vector<Id> mine;
    for (const auto& id : *only)
      if (std::find(pool.begin(), pool.end(), id) != pool.end()) mine.push_back(id);
    pool = mine;
  }
  for (int pass = 0; pass < 2; ++pass) {
    if (pass == 1) {
      if (only) {
        pool = *only;
      } else {
        auto a = ms_->active_ids();
        pool.assign(a.begin(), a.end());
      }
    }
    std::vector<Id> cand;
    {
      std::lock_guard<std::mutex> g(rng_mu_);
      for (const auto& id : pool)
        if (!tried.count(id.address) && !benched(id.address)) cand.push_back(id);
    }
    if (!cand.empty()) return pick_target(cand);
  }
  return std::nullopt;
}

void LeaderService::run_job(size_t j) {
  std::string model;
  size_t idx;
  int64_t elapsed0;
  std::vector<std::string> source;
  {
    std::lock_guard<std::mutex> g(mu_);
    model = jobs_[j].model_name;
    // resume point (src/services.rs:410-411): queries answered or dropped
    idx = (size_t)jobs_[j].finished + (size_t)jobs_[j].failed;
    elapsed0 = jobs_[j].elapsed_us;
    source = jobs_[j].source;
    retry_[j].clear();
    segs_[j].clear();
  }
  if (!source.empty() && !load_segments(j, source)) {
    std::lock_guard<std::mutex> g(mu_);
    running_[j] = false;
    return;
  }
  std::vector<Seg> segs;
  {
    std::lock_guard<std::mutex> g(mu_);
    segs = segs_[j];
  }
  const int64_t run0 = steady_us();
  const auto& L = labels_.entries;
  size_t total = L.size();
  if (!source.empty()) total = segs.empty() ? 0 : segs.back().start + segs.back().n;
  // a label job stops after the label table (the reference's 1,000 queries);
  // a shard job's --job-limit may exceed its shards' images: it loops over
  // them (sustained throughput runs, tools/bench_jobs.py --job-limit)
  const size_t limit = cfg_.job_limit > 0 ? (source.empty() ? std::min(total, (size_t)cfg_.job_limit)
                                                            : (total ? (size_t)cfg_.job_limit : 0))
                                          : total;
  auto next_tick = std::chrono::steady_clock::now();
  for (;;) {
    if (stop_.load()) break;
    Range range;  // a failed query again, else the next labels / shard images
    {
      std::lock_guard<std::mutex> g(mu_);
      if (!retry_[j].empty()) {
        range = retry_[j].front();
        retry_[j].pop_front();
      }
    }
    if (range.n == 0) {
      if (idx >= limit) {
        // all issued: wait for the stragglers, which may hand a query back
        if (job_inflight_[j].load() == 0) {
          std::lock_guard<std::mutex> g(mu_);
          if (retry_[j].empty()) break;
        }
        std::this_thread::sleep_for(std::chrono::milliseconds(1));
        continue;
      }
      range.first = idx;
      range.n = std::min((size_t)cfg_.query_batch, limit - idx);
      const size_t di = total ? idx % total : idx;  // data index (a looping shard job wraps)
      for (const auto& sg : segs)  // a shard query never spans two shards
        if (di >= sg.start && di < sg.start + sg.n) range.n = std::min(range.n, sg.start + sg.n - di);
      idx += range.n;
    }
    if (cfg_.adaptive_window <= 0) {
      next_tick += std::chrono::milliseconds(cfg_.query_interval_ms);
      std::this_thread::sleep_until(next_tick);
    }
    if (!is_leader()) break;  // leadership moved: the new leader resumes
    std::vector<Id> pool;
    {
      std::lock_guard<std::mutex> g(mu_);
      pool = jobs_[j].assigned;
    }
    if (!segs.empty()) {
      // a shard query goes to a replica holder (its bytes are resident there),
      // one of the job's own members when it can
      const Seg* sg = nullptr;
      const size_t di = range.first % total;
      for (const auto& x : segs)
        if (di >= x.start && di < x.start + x.n) sg = &x;
      const std::vector<Id> holders = sg ? shard_holders(sg->file) : std::vector<Id>{};
      std::vector<Id> mine;
      for (const auto& h : holders)
        if (std::find(pool.begin(), pool.end(), h) != pool.end()) mine.push_back(h);
      pool = mine.empty() ? holders : mine;
    } else if (pool.empty()) {
      auto a = ms_->active_ids();
      pool.assign(a.begin(), a.end());
    }
    if (pool.empty()) {
      std::lock_guard<std::mutex> g(mu_);
      if (segs.empty()) {
        retry_[j].push_front(range);  // no member at all: not an attempt
      } else if (range.attempts + 1 >= std::max(1, cfg_.max_attempts)) {
        // a shard with no live replica holder: an attempt like a failed query
        // (it used to be requeued forever and the job never finished: ADVICE r3)
        jobs_[j].failed += (int32_t)range.n;
        DMLC_LOG_WARN("job " << jobs_[j].model_name << ": images " << range.first << "+" << range.n
                             << ": no live replica holder; dropped");
      } else {
        range.attempts += 1;
        retry_[j].push_back(range);
      }
      if (cfg_.adaptive_window > 0 || !segs.empty()) std::this_thread::sleep_for(std::chrono::milliseconds(50));
      continue;
    }
    if (cfg_.adaptive_window > 0) {
      // closed loop: wait for a free slot in this job's window
      const int window = cfg_.adaptive_window * (int)pool.size();
      while (job_inflight_[j].load() >= window && !stop_.load())
        std::this_thread::sleep_for(std::chrono::microseconds(200));
      if (stop_.load()) break;
    }
    const Id target = pick_target(pool);
    while (inflight_.load() >= cfg_.max_inflight && !stop_.load())
      std::this_thread::sleep_for(std::chrono::microseconds(200));
    {
      std::lock_guard<std::mutex> g(mu_);
      if (jobs_[j].started_us == 0) jobs_[j].started_us = wall_us();
    }
    inflight_++;
    job_inflight_[j]++;
    {
      std::lock_guard<std::mutex> g(rng_mu_);
      member_inflight_[target.address]++;
    }
    submit([this, j, model, target, range, run0, elapsed0] { query(j, model, target, range, run0, elapsed0); });
  }
  std::lock_guard<std::mutex> g(mu_);
  running_[j] = false;
}

// One query (a batch of `n` labels / shard images from `first`). A member
// that fails (no answer, or ok=false: e.g. it has no such model) is benched
// for a background period and the query moves to another member of the
// job's pool (then any live member; for a shard query, any live replica
// holder), with its in-flight count; latency is end to end, retries
// included. A query no member could answer goes back to the job, with a
// back-off, at most max_attempts times in all; then it is dropped (the
// reference dropped failed queries) and counted as unanswered.
void LeaderService::query(size_t j, const std::string& model, Id target, Range range, int64_t run0,
                          int64_t elapsed0) {
  const auto& L = labels_.entries;
  const size_t n = range.n;
  const Seg* sg = nullptr;
  std::vector<Seg> segs;
  {
    std::lock_guard<std::mutex> g(mu_);
    segs = segs_[j];
  }
  // data index of the query's first image (a shard job may loop over its shards)
  const size_t total = segs.empty() ? 0 : segs.back().start + segs.back().n;
  const size_t first = total ? range.first % total : range.first;
  for (const auto& x : segs)
    if (first >= x.start && first < x.start + x.n) sg = &x;
  if (range.attempts > 0)  // a requeued query: back off before sending it again
    std::this_thread::sleep_for(std::chrono::milliseconds(std::min(cfg_.bg_ms, 50 * range.attempts)));
  Writer w;
  std::vector<Id> holders;
  if (sg) {
    w.str(model).str(sg->file).u64(first - sg->start).u32((uint32_t)n);
    holders = shard_holders(sg->file);
  } else {
    w.str(model).u32((uint32_t)n);
    for (size_t i = 0; i < n; ++i) w.str(L[first + i].first);
  }
  // truth of image i: its label index
  auto truth_of = [&](size_t i) -> size_t { return sg ? sg->label0 + (first - sg->start) + i : first + i; };
  const int64_t t0 = steady_us();
  Id tgt = target;
  std::vector<std::pair<double, std::string>> res;
  std::vector<int> cls;
  bool got = false;
  std::set<std::string> tried;
  DMLC_TRACE("leader.query");
  for (int attempt = 0; attempt < 4 && !stop_.load(); ++attempt) {
    bool transport = false;
    std::string why;
    int deadline = 0;
    try {
      // the reference connects anew for every query (src/services.rs:420); by
      // default the pooled connection is reused (--new-conn-per-query: fresh)
      {
        std::lock_guard<std::mutex> g(mu_);
        deadline = query_timeout(j);
      }
      // (a member the failure detector declares dead ends the wait early:
      // before the job has a latency history its deadline is the ceiling)
      const std::string resp = RpcClient::shared().call(
          tgt.host(), member_port(tgt.port()), sg ? M_PREDICT_RANGE : M_PREDICT, w.data(), deadline,
          cfg_.new_conn_per_query, [this, &tgt] { return ms_->active_ids().count(tgt) > 0; });
      Reader r(resp);
      if (r.boolean()) {
        const uint32_t m = r.u32();
        for (uint32_t i = 0; i < m; ++i) {
          if (sg) {
            const int c = r.i32();
            const double p = r.f64();
            cls.push_back(c);
            res.emplace_back(p, labels_.text(c));
          } else {
            const double p = r.f64();
            res.emplace_back(p, r.str());
          }
        }
        got = true;
        break;
      }
      why = "cannot serve " + model;
    } catch (const std::exception& e) {
      transport = true;
      why = e.what();
    }
    DMLC_LOG_WARN("predict " << model << " on " << tgt.address << " failed: " << why << " (deadline " << deadline
                             << " ms); benched");
    tried.insert(tgt.address);
    {
      std::lock_guard<std::mutex> g(rng_mu_);
      bench_until_[tgt.address] = steady_us() + (int64_t)cfg_.bg_ms * 1000;
    }
    if (transport) std::this_thread::sleep_for(std::chrono::milliseconds(std::min(cfg_.bg_ms, 200)));
    auto next = retry_target(j, tried, sg ? &holders : nullptr);
    if (!next) break;
    {
      std::lock_guard<std::mutex> g(rng_mu_);
      if (--member_inflight_[tgt.address] <= 0) member_inflight_.erase(tgt.address);
      member_inflight_[next->address]++;
    }
    tgt = *next;
  }
  const int64_t dur = steady_us() - t0;
  std::vector<std::string> lines;
  bool dropped = false;
  {
    std::lock_guard<std::mutex> g(mu_);
    if (got) {
      const int64_t now = wall_us();
      if (jobs_[j].first_done_us == 0) jobs_[j].first_done_us = now;
      for (size_t i = 0; i < n; ++i) {
        const size_t t = truth_of(i);
        const std::string& truth = L[t].second;
        const bool have = i < res.size() && res[i].first >= 0;
        const bool ok = have && (sg ? cls[i] == (int)t : res[i].second == truth);
        jobs_[j].add_result(ok, dur, now);
        if (!have) {
          lines.push_back(model + " - " + L[t].first + ": no image");
        } else if (cfg_.print_predictions) {
          char buf[64];
          snprintf(buf, sizeof(buf), " (%.2f%%)", res[i].first * 100.0);
          lines.push_back(model + " - " + L[t].first + ": " + res[i].second + buf +
                          (ok ? "" : " (should be " + truth + ")"));
        }
      }
      jobs_[j].elapsed_us = std::max(jobs_[j].elapsed_us, elapsed0 + (steady_us() - run0));
    } else if (range.attempts + 1 >= std::max(1, cfg_.max_attempts)) {
      jobs_[j].failed += (int32_t)n;
      dropped = true;
    } else {
      retry_[j].push_back({first, n, range.attempts + 1});
    }
  }
  if (!got)
    DMLC_LOG_WARN("predict " << model << " " << L[truth_of(0)].first << "+" << n << ": no member answered; "
                             << (dropped ? "dropped" : "requeued"));
  for (const auto& l : lines) out_line(l);
  {
    std::lock_guard<std::mutex> g(rng_mu_);
    if (--member_inflight_[tgt.address] <= 0) member_inflight_.erase(tgt.address);
  }
  job_inflight_[j]--;
  inflight_--;
}

void LeaderService::rereplicate_loop() {
  while (!stop_.load()) {
    sleep_bg();
    if (stop_.load()) break;
    if (!is_leader()) continue;
    std::vector<std::string> files;
    {
      std::lock_guard<std::mutex> g(mu_);
      for (const auto& kv : dir_) files.push_back(kv.first);
    }
    for (const auto& f : files) put_version(nullptr, nullptr, f, latest_version(f));
  }
}

void LeaderService::assign_loop() {
  while (!stop_.load()) {
    sleep_bg();
    if (stop_.load()) break;
    const std::vector<Id> active = ms_->active_sorted();
    std::lock_guard<std::mutex> g(mu_);
    const size_t J = jobs_.size(), n = active.size();
    for (size_t j = 0; j < J; ++j) {
      const size_t b = j * n / J, e = (j + 1) * n / J;
      jobs_[j].assigned.assign(active.begin() + b, active.begin() + e);
    }
  }
}

void LeaderService::succession_loop() {
  // The member's leader check (every bg period, src/services.rs:527-545, or at
  // once when its heartbeat sees the leader miss) moves the leader pointer; a
  // standby that finds itself pointed at takes over at once (the pointer is a
  // local read, polled every 50 ms) instead of at its own next bg tick, which
  // added up to a whole further period to a coordinator fail-over (5.5 s mean
  // with the reference's periods, trials of 3.3-6.8 s:
  // profiles/r5_recovery_refperiods_leader_before.json). The job-state copy
  // runs in its own loop (standby_copy_loop), so a copy call stuck on a hung
  // leader never delays the take-over.
  std::string last = member_->leader_address();
  while (!stop_.load()) {
    std::this_thread::sleep_for(std::chrono::milliseconds(50));
    if (stop_.load()) break;
    const std::string leader = member_->leader_address();
    if (last != self_ && leader == self_) {
      bool resume;
      {
        std::lock_guard<std::mutex> g(mu_);
        leading_ = true;
        // resume when the copy shows the jobs running: any job that issued or
        // finished a query (not only job 0's completions: a copy taken before
        // the first job's first answer would otherwise leave both jobs stopped)
        resume = jobs_running(jobs_);
      }
      {
        // the previous leader's node was unreachable (that is what moved the
        // pointer): no queries to its member until membership has decided
        std::lock_guard<std::mutex> g(rng_mu_);
        bench_until_[last] = steady_us() + (int64_t)cfg_.bg_ms * 1000;
      }
      DMLC_LOG_WARN("became leader" << (resume ? "; resuming jobs" : ""));
      if (resume) predict();
    } else if (leader != self_) {
      std::lock_guard<std::mutex> g(mu_);
      leading_ = false;
    }
    last = leader;
  }
}

void LeaderService::standby_copy_loop() {
  // A standby copies the leader's job progress every standby_copy_ms
  // (incremental: only the queries completed since the last copy move; the
  // per-query vectors grow with every query, so re-sending them all each
  // period made the copy cost grow with the job) and the SDFS directory every
  // bg period (the reference's copy period; it changes only on put / delete /
  // re-replication, so copying it at the job-progress rate was 12x the state
  // traffic and leader-mutex time for nothing: ADVICE r5).
  const auto copy_period = std::chrono::milliseconds(std::max(50, cfg_.standby_copy_ms));
  const auto dir_period = std::chrono::milliseconds(std::max(cfg_.bg_ms, cfg_.standby_copy_ms));
  auto next_dir = std::chrono::steady_clock::now();
  while (!stop_.load()) {
    const auto t0 = std::chrono::steady_clock::now();
    for (auto t = t0; !stop_.load() && t < t0 + copy_period; t = std::chrono::steady_clock::now())
      std::this_thread::sleep_for(std::chrono::milliseconds(std::min<int64_t>(50, cfg_.standby_copy_ms)));
    if (stop_.load()) break;
    const std::string leader = member_->leader_address();
    if (leader == self_) continue;
    const bool want_dir = std::chrono::steady_clock::now() >= next_dir;
    try {
      Writer req;
      {
        std::lock_guard<std::mutex> g(mu_);
        req.u32((uint32_t)jobs_.size());
        for (const auto& j : jobs_) req.u32((uint32_t)std::min(j.durations_us.size(), j.done_us.size()));
      }
      req.boolean(want_dir);
      // (a copy waits at most one copy period: a hung leader stalls only this loop)
      const std::string resp = RpcClient::shared().call(host_of(leader), leader_port(port_of(leader)), L_STATE,
                                                        req.data(), std::max(1000, cfg_.standby_copy_ms));
      Reader r(resp);
      const uint32_t nj = r.u32();
      std::lock_guard<std::mutex> g(mu_);
      if (leading_) continue;  // took over meanwhile: this node's own progress is the truth now
      std::vector<Job> js = jobs_;
      bool aligned = nj == js.size();
      for (uint32_t i = 0; i < nj; ++i) {
        Job tmp;
        Job& dst = aligned ? js[i] : tmp;
        if (!read_job_delta(r, dst)) aligned = false;
      }
      const bool has_dir = r.boolean();
      if (has_dir) {
        dir_ = read_directory(r);
        next_dir = std::chrono::steady_clock::now() + dir_period;
      }
      if (aligned) jobs_ = std::move(js);
      else for (auto& j : jobs_) j.durations_us.clear(), j.done_us.clear();  // full copy next time
    } catch (const std::exception&) {
    }
  }
}

int LeaderService::query_timeout(size_t j) const {
  const auto& d = jobs_[j].durations_us;
  if (d.size() < 20) return cfg_.query_timeout_ms;
  std::vector<int64_t> recent(d.end() - (ptrdiff_t)std::min<size_t>(d.size(), 256), d.end());
  const size_t k = recent.size() * 99 / 100;
  std::nth_element(recent.begin(), recent.begin() + (ptrdiff_t)k, recent.end());
  const int64_t ms = recent[k] / 100;  // 10 x p99 (us -> ms)
  return (int)std::max<int64_t>(cfg_.query_timeout_min_ms, std::min<int64_t>(cfg_.query_timeout_ms, ms));
}

void LeaderService::register_handlers() {
  server_->handle(L_ALIVE, [](Reader&) {
    Writer w;
    w.boolean(true);
    return w.take();
  });
  server_->handle(L_PUT, [this](Reader& r) {
    const Id src = read_id(r);
    const std::string path = r.str(), fname = r.str();
    const auto ids = put(src, path, fname);
    Writer w;
    w.u32((uint32_t)ids.size());
    for (const auto& id : ids) write_id(w, id);
    return w.take();
  });
  server_->handle(L_GET, [this](Reader& r) {
    const std::string fname = r.str();
    const Id dest = read_id(r);
    const std::string path = r.str();
    const int v = get(fname, dest, path);
    Writer w;
    w.boolean(v > 0).i32(v);
    return w.take();
  });
  server_->handle(L_GET_VERSIONS, [this](Reader& r) {
    const std::string fname = r.str();
    const int count = r.i32();
    const Id dest = read_id(r);
    const std::string path = r.str();
    const auto vs = get_versions(fname, count, dest, path);
    Writer w;
    w.u32((uint32_t)vs.size());
    for (int v : vs) w.i32(v);
    return w.take();
  });
  server_->handle(L_DELETE, [this](Reader& r) {
    del(r.str());
    return std::string();
  });
  server_->handle(L_LS, [this](Reader& r) {
    const auto res = ls(r.str());
    Writer w;
    w.u32((uint32_t)res.size());
    for (const auto& e : res) {
      write_id(w, e.first);
      w.u32((uint32_t)e.second.size());
      for (int v : e.second) w.i32(v);
    }
    return w.take();
  });
  server_->handle(L_TRAIN, [this](Reader& r) {
    const std::string fname = r.str(), model = r.str();
    Writer w;
    try {
      train(fname, model);
      w.boolean(true).str("");
    } catch (const std::exception& e) {
      w.boolean(false).str(e.what());
    }
    return w.take();
  });
  server_->handle(L_PREDICT_SHARD, [this](Reader& r) {
    // a replica holder of the latest version classifies its (HBM-resident)
    // copy: the shard's bytes never move
    const std::string f = r.str(), model = r.str();
    const int v = latest_version(f);
    if (v == 0) throw std::runtime_error("file not found: " + f);
    std::vector<Id> holders;
    {
      std::lock_guard<std::mutex> g(mu_);
      for (const auto& rep : dir_[f])
        if (rep.second.count(v)) holders.push_back(rep.first);
    }
    const auto active = ms_->active_ids();
    std::string last_err = "no live holder";
    for (const Id& h : holders) {
      if (!active.count(h)) continue;
      try {
        Writer w;
        w.str(f).str(model);
        const std::string resp = RpcClient::shared().call(h.host(), member_port(h.port()), M_PREDICT_SHARD, w.data(),
                                                          600000);
        Writer out;
        out.str(h.address);
        return out.take() + resp;
      } catch (const std::exception& e) {
        last_err = h.address + ": " + e.what();
      }
    }
    throw std::runtime_error("predict-shard " + f + ": " + last_err);
  });
  server_->handle(L_PREDICT, [this](Reader& r) {
    std::vector<std::string> notes;
    if (r.left() >= 4) {  // `predict <shard>...` / `predict dataset`
      const uint32_t k = r.u32();
      if (k > 4096) throw std::runtime_error("predict: too many shards");
      std::vector<std::string> shards;
      for (uint32_t i = 0; i < k; ++i) shards.push_back(r.str());
      notes = predict(&shards);
    } else {
      notes = predict();
    }
    Writer w;
    w.u32((uint32_t)notes.size());
    for (const auto& x : notes) w.str(x);
    return w.take();
  });
  server_->handle(L_JOBS, [this](Reader&) {
    const auto js = jobs();
    Writer w;
    w.u32((uint32_t)js.size());
    for (const auto& j : js) write_job(w, j);
    return w.take();
  });
  server_->handle(L_STATE, [this](Reader& r) {
    std::vector<uint32_t> have;
    if (r.left() >= 4) {
      const uint32_t n = r.u32();
      for (uint32_t i = 0; i < n; ++i) have.push_back(r.u32());
    }
    const bool want_dir = r.left() >= 1 ? r.boolean() : true;
    Writer w;
    std::lock_guard<std::mutex> g(mu_);
    w.u32((uint32_t)jobs_.size());
    for (size_t i = 0; i < jobs_.size(); ++i) write_job_delta(w, jobs_[i], i < have.size() ? have[i] : 0);
    w.boolean(want_dir);
    if (want_dir) write_directory(w, dir_);
    return w.take();
  });
}

}  // namespace ctl
}  // namespace dmlc
