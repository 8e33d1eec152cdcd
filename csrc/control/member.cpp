#include "member.h"

#include "../runtime/trace.h"

#include <dirent.h>
#include <poll.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <fstream>
#include "../serve/shard.h"

#include "common.h"
#include "../comm/cv_wait.h"

namespace dmlc {
namespace ctl {

namespace {

void rm_rf(const std::string& path) {
  DIR* d = opendir(path.c_str());
  if (d) {
    while (dirent* e = readdir(d)) {
      const std::string n = e->d_name;
      if (n == "." || n == "..") continue;
      const std::string p = path + "/" + n;
      struct stat st;
      if (lstat(p.c_str(), &st) == 0 && S_ISDIR(st.st_mode))
        rm_rf(p);
      else
        unlink(p.c_str());
    }
    closedir(d);
  }
  rmdir(path.c_str());
}

void mkdir_p(const std::string& path) {
  std::string cur;
  for (const auto& part : split(path, '/')) {
    cur += part + "/";
    if (!part.empty()) mkdir(cur.c_str(), 0755);
  }
}

std::vector<std::string> list_dir_sorted(const std::string& path) {
  std::vector<std::string> out;
  DIR* d = opendir(path.c_str());
  if (!d) return out;
  while (dirent* e = readdir(d)) {
    const std::string n = e->d_name;
    if (n != "." && n != "..") out.push_back(n);
  }
  closedir(d);
  std::sort(out.begin(), out.end());
  return out;
}

}  // namespace

Labels Labels::load(const std::string& path) {
  Labels l;
  std::ifstream f(path);
  std::string line;
  while (std::getline(f, line)) {
    line = trim(line);
    if (line.empty()) continue;
    const auto sp = line.find(' ');
    std::string wnid = sp == std::string::npos ? line : line.substr(0, sp);
    std::string text = sp == std::string::npos ? "" : trim(line.substr(sp + 1));
    l.index[wnid] = (int)l.entries.size();
    l.entries.emplace_back(wnid, text);
  }
  return l;
}

std::string Labels::text(int idx) const {
  if (idx >= 0 && idx < (int)entries.size()) return entries[idx].second;
  return "class " + std::to_string(idx);
}

MemberService::MemberService(MemberConfig cfg, MembershipService* ms, std::unique_ptr<Executor> exec, Labels labels)
    : cfg_(std::move(cfg)), ms_(ms), exec_(std::move(exec)), labels_(std::move(labels)) {
  if (cfg_.storage_dir.empty()) cfg_.storage_dir = cfg_.workdir + "/storage";
  if (cfg_.models_dir.empty()) cfg_.models_dir = cfg_.workdir + "/models";
  if (!cfg_.leader_candidates.empty()) leader_ = cfg_.leader_candidates[0];
}

MemberService::~MemberService() { stop(); }

void MemberService::start(int base_port) {
  rm_rf(cfg_.storage_dir);  // storage is recreated empty at start-up (src/services.rs:504-507)
  mkdir_p(cfg_.storage_dir);
  mkdir_p(cfg_.models_dir);
  server_ = std::make_unique<RpcServer>("member", cfg_.bind_host, member_port(base_port));
  register_handlers();
  server_->start();
  checker_ = std::thread([this] { leader_check_loop(); });
  if (!cfg_.leader_candidates.empty() && cfg_.watch_ms > 0) watcher_ = std::thread([this] { leader_watch_loop(); });
  replicator_ = std::thread([this] { replica_loop(); });
}

namespace {
std::string replica_key(const std::string& file, int v) { return file + "@v" + std::to_string(v); }
}  // namespace

void MemberService::stage_replica(const std::string& file, int version) {
  if (!exec_) return;
  const std::string path = cfg_.storage_dir + "/" + storage_filename(file, version);
  {
    std::ifstream f(path, std::ios::binary);
    char magic[8] = {};
    if (!f.read(magic, 8) || std::memcmp(magic, kShardMagic, 8) != 0) return;  // only u8 shards live in HBM
  }
  const std::string key = replica_key(file, version);
  {
    std::ifstream f(path, std::ios::binary | std::ios::ate);
    const size_t bytes = (size_t)f.tellg();
    f.seekg(0);
    uint8_t head[kShardHeader] = {};
    if (!f.read((char*)head, kShardHeader)) throw std::runtime_error(path + ": short shard");
    ShardMeta m;
    m.version = version;
    m.info = parse_shard(head, bytes);  // validates the header before anything is staged
    std::lock_guard<std::mutex> g(mu_);
    shard_meta_[file] = m;
  }
  exec_->stage_blob(key, path);
  for (const auto& k : exec_->blob_keys())  // older versions of the same file leave HBM
    if (k != key && k.rfind(file + "@v", 0) == 0) exec_->drop_blob(k);
  DMLC_LOG_INFO("staged replica " << key << " in " << exec_->blob_location());
}

void MemberService::replica_loop() {
  while (!stop_.load()) {
    std::pair<std::string, int> item;
    {
      std::unique_lock<std::mutex> g(rq_mu_);
      // untimed wait: GCC 11's ThreadSanitizer does not intercept the
      // pthread_cond_clockwait behind wait_for (false double-lock reports)
      rq_cv_.wait(g, [&] { return !rq_.empty() || stop_.load(); });
      if (rq_.empty()) continue;
      item = rq_.front();
      rq_.pop_front();
    }
    try {
      stage_replica(item.first, item.second);
    } catch (const std::exception& e) {
      DMLC_LOG_WARN("staging replica " << item.first << " v" << item.second << " failed: " << e.what());
    }
  }
}

std::vector<std::string> MemberService::staged_replicas() const {
  return exec_ ? exec_->blob_keys() : std::vector<std::string>{};
}

MemberService::ShardResult MemberService::predict_shard(const std::string& file, const std::string& model) {
  if (!exec_) throw std::runtime_error("no executor");
  int v = 0;
  {
    std::lock_guard<std::mutex> g(mu_);
    auto it = files_.find(file);
    if (it == files_.end() || it->second.empty()) throw std::runtime_error("no replica of " + file + " here");
    v = *it->second.rbegin();
  }
  const std::string key = replica_key(file, v);
  const auto keys = exec_->blob_keys();
  if (std::find(keys.begin(), keys.end(), key) == keys.end()) stage_replica(file, v);
  ShardResult r;
  r.version = v;
  r.location = exec_->blob_location() + " -> " + exec_->backend();
  const int64_t t0 = steady_us();
  r.preds = exec_->predict_blob(model, key);
  r.elapsed_us = steady_us() - t0;
  return r;
}

MemberService::ShardMeta MemberService::shard_meta(const std::string& file) {
  int v = 0;
  {
    std::lock_guard<std::mutex> g(mu_);
    auto it = files_.find(file);
    if (it == files_.end() || it->second.empty()) throw std::runtime_error("no replica of " + file + " here");
    v = *it->second.rbegin();
    auto m = shard_meta_.find(file);
    if (m != shard_meta_.end() && m->second.version == v) return m->second;
  }
  const std::string path = cfg_.storage_dir + "/" + storage_filename(file, v);
  std::ifstream f(path, std::ios::binary | std::ios::ate);
  if (!f) throw std::runtime_error("replica of " + file + " v" + std::to_string(v) + " is neither staged nor on disk");
  const size_t bytes = (size_t)f.tellg();
  f.seekg(0);
  uint8_t head[kShardHeader] = {};
  if (!f.read((char*)head, kShardHeader)) throw std::runtime_error(file + " is not a u8 shard");
  ShardMeta m;
  m.version = v;
  m.info = parse_shard(head, bytes);
  std::lock_guard<std::mutex> g(mu_);
  shard_meta_[file] = m;
  return m;
}

std::vector<Prediction> MemberService::predict_range(const std::string& file, const std::string& model, int64_t first,
                                                     int64_t n) {
  if (!exec_) throw std::runtime_error("no executor");
  const ShardMeta m = shard_meta(file);
  if (first < 0 || n < 0 || first + n > (int64_t)m.info.n) throw std::runtime_error(file + ": range out of bounds");
  const std::string key = replica_key(file, m.version);
  const auto keys = exec_->blob_keys();
  if (std::find(keys.begin(), keys.end(), key) == keys.end()) stage_replica(file, m.version);
  DMLC_TRACE("member.predict_range");
  return exec_->predict_blob_range(model, key, first, n);
}

void MemberService::stop() {
  if (stop_.exchange(true)) return;
  { std::lock_guard<std::mutex> g(rq_mu_); }  // a waiter is past its predicate check or asleep: no lost wakeup
  rq_cv_.notify_all();
  { std::lock_guard<std::mutex> g(wake_mu_); }
  wake_cv_.notify_all();
  if (watcher_.joinable()) watcher_.join();
  if (replicator_.joinable()) replicator_.join();
  if (checker_.joinable()) checker_.join();
  if (prefetcher_.joinable()) prefetcher_.join();
  if (server_) server_->stop();
}

std::string MemberService::leader_address() const {
  std::lock_guard<std::mutex> g(mu_);
  return leader_;
}

std::map<std::string, std::set<int>> MemberService::files() const {
  std::lock_guard<std::mutex> g(mu_);
  return files_;
}

std::string MemberService::resolve_spec(const std::string& spec) const {
  if (starts_with(spec, "storage:")) return cfg_.storage_dir + "/" + sanitize_filename(spec.substr(8));
  if (starts_with(spec, "models:")) return cfg_.models_dir + "/" + sanitize_filename(spec.substr(7));
  if (!spec.empty() && spec[0] == '/') return spec;
  return cfg_.workdir + "/" + spec;
}

void MemberService::allow_read(const std::string& p, bool on) {
  std::lock_guard<std::mutex> g(mu_);
  if (on) readable_.insert(p);
  else if (readable_.count(p)) readable_.erase(readable_.find(p));
}

void MemberService::allow_write(const std::string& p, bool on) {
  std::lock_guard<std::mutex> g(mu_);
  if (on) writable_.insert(p);
  else if (writable_.count(p)) writable_.erase(writable_.find(p));
}

namespace {
bool managed_spec(const std::string& spec) { return starts_with(spec, "storage:") || starts_with(spec, "models:"); }
}  // namespace

std::string MemberService::readable_path(const std::string& spec) const {
  if (managed_spec(spec)) return resolve_spec(spec);
  std::lock_guard<std::mutex> g(mu_);
  if (!spec.empty() && spec[0] == '/' && readable_.count(spec)) return spec;
  throw std::runtime_error("refused: " + spec + " is not exported by this node");
}

std::string MemberService::writable_path(const std::string& spec) const {
  if (managed_spec(spec)) return resolve_spec(spec);
  std::lock_guard<std::mutex> g(mu_);
  if (!spec.empty() && spec[0] == '/') {
    if (writable_.count(spec)) return spec;
    // get-versions writes v<N>.<name> next to the requested destination
    const auto slash = spec.rfind('/');
    const std::string dir = spec.substr(0, slash + 1), base = spec.substr(slash + 1);
    size_t i = 1;
    if (base.size() > 2 && base[0] == 'v') {
      while (i < base.size() && isdigit((unsigned char)base[i])) ++i;
      if (i > 1 && i < base.size() && base[i] == '.' && writable_.count(dir + base.substr(i + 1))) return spec;
    }
  }
  throw std::runtime_error("refused: " + spec + " is not an expected destination on this node");
}

std::vector<std::pair<double, std::string>> MemberService::predict(const std::string& model,
                                                                   const std::vector<std::string>& ids, bool* ok) {
  *ok = false;
  std::vector<std::pair<double, std::string>> out;
  if (!exec_ || !exec_->has_model(model)) return out;
  DMLC_TRACE("member.predict");
  // One answer per requested id, in order: an id without an image (the
  // reference's read_dir would fail) answers (-1, "") so the leader never
  // shifts later answers onto the wrong labels.
  std::vector<std::string> paths;
  std::vector<size_t> where;
  for (size_t i = 0; i < ids.size(); ++i) {
    std::string p = query_image(ids[i]);
    if (!p.empty()) {
      paths.push_back(std::move(p));
      where.push_back(i);
    }
  }
  out.assign(ids.size(), {-1.0, std::string()});
  const auto preds = exec_->predict_files(model, paths);
  for (size_t k = 0; k < preds.size() && k < where.size(); ++k)
    out[where[k]] = {preds[k].prob, labels_.text(preds[k].class_idx)};
  *ok = true;
  return out;
}

std::string MemberService::query_image(const std::string& id) const {
  // src/services.rs:485-490: the first file of test_files/imagenet_1k/train/<id>/
  const std::string dir = cfg_.dataset_dir + "/" + sanitize_filename(id);
  const auto files = list_dir_sorted(dir);
  return files.empty() ? std::string() : dir + "/" + files[0];
}

bool MemberService::start_prefetch() {
  if (!exec_ || prefetching_.exchange(true)) return false;
  if (prefetcher_.joinable()) prefetcher_.join();
  prefetcher_ = std::thread([this] {
    for (size_t i = 0; i < labels_.entries.size() && !stop_; ++i) {
      const std::string p = query_image(labels_.entries[i].first);
      if (p.empty()) continue;
      try {
        if (!exec_->stage(p)) break;
        ++prefetched_;
      } catch (const std::exception& e) {
        DMLC_LOG_WARN("prefetch of " << p << " failed: " << e.what());
      }
    }
    prefetching_ = false;
  });
  return true;
}

bool MemberService::fetch(const std::string& src_host, int src_port, const std::string& src_spec,
                          const std::string& dest_spec) {
  std::string dest, tmp;
  try {
    dest = writable_path(dest_spec);
    tmp = dest + ".part" + std::to_string(getpid());
    std::ofstream out(tmp, std::ios::binary | std::ios::trunc);
    if (!out) throw std::runtime_error("cannot open " + tmp);
    uint64_t off = 0;
    while (true) {
      Writer w;
      w.str(src_spec).u64(off).u32((uint32_t)cfg_.chunk_bytes);
      const std::string resp = RpcClient::shared().call(src_host, src_port, M_READ_CHUNK, w.data(), 60000);
      Reader r(resp);
      const uint64_t total = r.u64();
      const std::string data = r.str();
      out.write(data.data(), (std::streamsize)data.size());
      off += data.size();
      if (off >= total || data.empty()) break;
    }
    out.close();
    if (rename(tmp.c_str(), dest.c_str()) != 0) throw std::runtime_error("rename failed");
    DMLC_LOG_INFO("fetch " << src_host << ":" << src_port << ":" << src_spec << " -> " << dest << ": ok (" << off
                           << " B)");
    return true;
  } catch (const std::exception& e) {
    if (!tmp.empty()) unlink(tmp.c_str());
    DMLC_LOG_WARN("fetch " << src_host << ":" << src_port << ":" << src_spec << " -> " << dest
                           << ": failed: " << e.what());
    return false;
  }
}

void MemberService::register_handlers() {
  server_->handle(M_GET_LATEST_VERSION, [this](Reader& r) {
    const std::string f = r.str();
    Writer w;
    std::lock_guard<std::mutex> g(mu_);
    auto it = files_.find(f);
    if (it == files_.end() || it->second.empty()) {
      w.boolean(false).i32(0);
    } else {
      w.boolean(true).i32(*it->second.rbegin());
    }
    return w.take();
  });
  server_->handle(M_RECEIVE, [this](Reader& r) {
    const std::string f = r.str();
    const int v = r.i32();
    {
      std::lock_guard<std::mutex> g(mu_);
      files_[f].insert(v);
    }
    if (cfg_.hbm_replicas && exec_) {  // a u8 shard replica goes resident into HBM
      std::lock_guard<std::mutex> g(rq_mu_);
      rq_.emplace_back(f, v);
      rq_cv_.notify_one();
    }
    return std::string();
  });
  server_->handle(M_PREDICT_SHARD, [this](Reader& r) {
    const std::string f = r.str(), model = r.str();
    const ShardResult res = predict_shard(f, model);
    Writer w;
    w.i32(res.version).str(res.location).i64(res.elapsed_us).u32((uint32_t)res.preds.size());
    for (const auto& p : res.preds) w.i32(p.class_idx).f64(p.prob);
    return w.take();
  });
  server_->handle(M_SHARD_INFO, [this](Reader& r) {
    const ShardMeta m = shard_meta(r.str());
    Writer w;
    w.i32(m.version).u32(m.info.n).u32(m.info.h).u32(m.info.w).u32(m.info.label0).boolean(m.info.labelled);
    return w.take();
  });
  server_->handle(M_PREDICT_RANGE, [this](Reader& r) {
    const std::string model = r.str(), file = r.str();
    const int64_t first = (int64_t)r.u64();
    const uint32_t n = r.u32();
    Writer w;
    if (!exec_ || !exec_->has_model(model)) {
      w.boolean(false).u32(0);
      return w.take();
    }
    const auto preds = predict_range(file, model, first, n);
    w.boolean(true).u32((uint32_t)preds.size());
    for (const auto& p : preds) w.i32(p.class_idx).f64(p.prob);
    return w.take();
  });
  server_->handle(M_PREDICT, [this](Reader& r) {
    const std::string model = r.str();
    const uint32_t n = r.u32();
    std::vector<std::string> ids(n);
    for (auto& s : ids) s = r.str();
    bool ok = false;
    const auto res = predict(model, ids, &ok);
    Writer w;
    w.boolean(ok).u32((uint32_t)res.size());
    for (const auto& p : res) w.f64(p.first).str(p.second);
    return w.take();
  });
  server_->handle(M_FETCH, [this](Reader& r) {
    const std::string host = r.str();
    const int port = r.i32();
    const std::string src = r.str(), dest = r.str();
    Writer w;
    w.boolean(fetch(host, port, src, dest));
    return w.take();
  });
  server_->handle(M_READ_CHUNK, [this](Reader& r) {
    const std::string spec = r.str();
    const uint64_t off = r.u64();
    const uint32_t len = std::min<uint32_t>(r.u32(), 64u << 20);
    const std::string path = readable_path(spec);
    std::ifstream f(path, std::ios::binary);
    if (!f) throw std::runtime_error("no such file: " + spec);
    f.seekg(0, std::ios::end);
    const uint64_t total = (uint64_t)f.tellg();
    std::string data;
    if (off < total) {
      data.resize((size_t)std::min<uint64_t>(len, total - off));
      f.seekg((std::streamoff)off);
      f.read(&data[0], (std::streamsize)data.size());
    }
    Writer w;
    w.u64(total).str(data);
    return w.take();
  });
  server_->handle(M_DELETE_FILE, [this](Reader& r) {
    const std::string f = r.str();
    std::set<int> versions;
    {
      std::lock_guard<std::mutex> g(mu_);
      auto it = files_.find(f);
      if (it != files_.end()) versions = it->second;
      files_.erase(f);
    }
    for (int v : versions) {
      unlink((cfg_.storage_dir + "/" + storage_filename(f, v)).c_str());
      if (exec_) exec_->drop_blob(replica_key(f, v));
    }
    return std::string();
  });
  server_->handle(M_LOAD_MODEL, [this](Reader& r) {
    const std::string model = r.str();
    const std::string spec = r.str();
    Writer w;
    try {
      if (!exec_) throw std::runtime_error("no executor");
      if (!managed_spec(spec)) throw std::runtime_error("refused: models load from storage:/models: specs only");
      exec_->load_model(model, resolve_spec(spec));
      DMLC_LOG_INFO("loaded model " << model << " from " << resolve_spec(spec));
      w.boolean(true).str("");
    } catch (const std::exception& e) {
      w.boolean(false).str(e.what());
    }
    return w.take();
  });
  server_->handle(M_INFO, [this](Reader&) {
    Writer w;
    w.str(exec_ ? exec_->backend() : "none");
    std::lock_guard<std::mutex> g(mu_);
    w.u32((uint32_t)files_.size());
    return w.take();
  });
}

bool MemberService::check_leader(const std::string& addr, int timeout_ms) {
  try {
    const std::string resp =
        RpcClient::shared().call(host_of(addr), leader_port(port_of(addr)), L_ALIVE, "", timeout_ms);
    Reader r(resp);
    return r.boolean();
  } catch (const std::exception&) {
    return false;
  }
}

void MemberService::leader_check_loop() {
  while (!stop_.load()) {
    bool woken;
    {
      // one check period, or earlier when the heartbeat saw the leader fail
      std::unique_lock<std::mutex> lk(wake_mu_);
      const auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(cfg_.check_ms);
      while (!wake_ && !stop_.load() && cv_wait_until(wake_cv_, lk, deadline) != std::cv_status::timeout) {
      }
      woken = wake_;
      wake_ = false;
    }
    if (stop_.load() || cfg_.leader_candidates.empty()) break;
    std::string cur = leader_address();
    // (woken: the heartbeat has already seen this leader miss: confirm with
    // the heartbeat's timeout; with the heartbeat on, the periodic check
    // waits at most 1 s, so it never holds the checker past a wake for long)
    if (check_leader(cur, woken || cfg_.watch_ms > 0 ? std::max(woken ? 100 : 1000, 3 * cfg_.watch_ms) : 2000))
      continue;
    // Advance through the candidate list (wrapping, unlike the reference),
    // at most one full round per check period.
    const auto& c = cfg_.leader_candidates;
    size_t idx = std::find(c.begin(), c.end(), cur) - c.begin();
    for (size_t step = 1; step <= c.size(); ++step) {
      const std::string next = c[(idx + step) % c.size()];
      if (next == cur) continue;
      if (check_leader(next)) {
        {
          std::lock_guard<std::mutex> g(mu_);
          leader_ = next;
        }
        DMLC_LOG_WARN("leader " << cur << " unreachable; switched to " << next);
        break;
      }
    }
  }
}

void MemberService::leader_watch_loop() {
  // The reference finds a dead leader only by its periodic check
  // (src/services.rs:527-545: one check period of detection on average, a
  // whole one at worst). The check stays; this heartbeat shortens detection:
  // an L_ALIVE probe every watch_ms on the pooled connection. A refused or
  // closed connection (a crashed process: its kernel sent a FIN or RST) wakes
  // the checker at once, a hung leader (sockets open, nothing answers) once a
  // probe times out; the checker confirms with a probe of its own before it
  // moves the pointer. Only a probe failure after one that succeeded counts
  // (a leader still coming up is left to the periodic check, as in the
  // reference), and wakes are at most one per second: a busy leader that
  // drops a probe costs one extra check (2 s timeout), never a storm.
  using clock = std::chrono::steady_clock;
  const int timeout = std::max(100, 3 * cfg_.watch_ms);
  std::string cur;
  bool seen_up = false;
  int missed = 0;
  auto last_wake = clock::now() - std::chrono::seconds(10);
  while (!stop_.load()) {
    const std::string now_leader = leader_address();
    if (now_leader != cur) {  // a new leader: start over
      cur = now_leader;
      seen_up = false;
      missed = 0;
    }
    const auto t0 = clock::now();
    bool ok = false, refused = false;
    try {
      const std::string resp =
          RpcClient::shared().call(host_of(cur), leader_port(port_of(cur)), L_ALIVE, "", timeout);
      Reader r(resp);
      ok = r.boolean();
    } catch (const std::exception& e) {
      // a timeout takes the whole timeout; a closed / refused connection fails at once
      refused = clock::now() - t0 < std::chrono::milliseconds(timeout / 2);
    }
    if (stop_.load()) break;
    if (ok) {
      seen_up = true;
      missed = 0;
    } else if (seen_up && leader_address() == cur) {
      ++missed;
      if (clock::now() - last_wake >= std::chrono::seconds(1)) {
        last_wake = clock::now();
        {
          std::lock_guard<std::mutex> g(wake_mu_);
          wake_ = true;
        }
        wake_cv_.notify_all();
        DMLC_LOG_INFO("leader " << cur << " missed " << missed << " heartbeat(s)" << (refused ? " (connection closed)" : "")
                                << "; checking now");
      }
    }
    const auto next = t0 + std::chrono::milliseconds(cfg_.watch_ms);
    while (!stop_.load() && clock::now() < next && leader_address() == cur)
      std::this_thread::sleep_for(std::chrono::milliseconds(20));
  }
}

}  // namespace ctl
}  // namespace dmlc
