// dmlc-node: process entry, configuration and the interactive REPL.
//
// Reference: `main` (src/main.rs:25-41) starts the membership service, the
// member server, the leader server on the three hard-coded candidate hosts,
// and `run_cli` (src/main.rs:85-338), a stdin loop with the verbs
//   list_mem|lm, list_self, join|j <host>, leave|l, put|p <local> <sdfs>,
//   get|g <sdfs> <local>, delete|d <sdfs>, ls <sdfs>, store|s,
//   get-versions|gv <sdfs> <count> <local>, train|t <sdfs> <model>,
//   predict, jobs, assign
// and the same output strings. Everything the reference hard-codes (hosts,
// ports, periods, replication factor, paths) is a flag here, so any number
// of nodes run on one machine; extra verbs: fault, info, prefetch, sleep, quit.
//
// Sub-commands: `dmlc-node selftest` (C++ unit tests) and
// `dmlc-node classify --model M --weights W.ot --labels L --image I.JPEG`
// (single-image classification from a .ot checkpoint, CPU or GPU).
#include <signal.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <csignal>
#include <set>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <iostream>
#include <map>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "../control/common.h"
#include "../control/member.h"
#include "../control/membership.h"
#include "../control/rpc.h"
#include "../control/sdfs.h"
#include "../control/table.h"
#include "../serve/executor.h"
#include "../serve/job.h"
#include "../serve/leader.h"

namespace dmlc {
namespace ctl {
int run_selftest();
}
}  // namespace dmlc

using namespace dmlc;
using namespace dmlc::ctl;

namespace {

// Grants peers access to one absolute path for the lifetime of a command.
struct PathGrant {
  PathGrant(MemberService& m, std::string p, bool write) : m_(m), p_(std::move(p)), w_(write) {
    w_ ? m_.allow_write(p_, true) : m_.allow_read(p_, true);
  }
  ~PathGrant() { w_ ? m_.allow_write(p_, false) : m_.allow_read(p_, false); }
  MemberService& m_;
  std::string p_;
  bool w_;
};

struct Args {
  std::map<std::string, std::string> kv;
  std::vector<std::string> pos;
  bool has(const std::string& k) const { return kv.count(k) > 0; }
  std::string get(const std::string& k, const std::string& d = "") const {
    auto it = kv.find(k);
    return it == kv.end() ? d : it->second;
  }
  int geti(const std::string& k, int d) const { return has(k) ? std::stoi(get(k)) : d; }
};

Args parse(int argc, char** argv, int start) {
  Args a;
  for (int i = start; i < argc; ++i) {
    std::string s = argv[i];
    if (starts_with(s, "--")) {
      s = s.substr(2);
      const auto eq = s.find('=');
      if (eq != std::string::npos) {
        a.kv[s.substr(0, eq)] = s.substr(eq + 1);
      } else if (i + 1 < argc && !starts_with(argv[i + 1], "--")) {
        a.kv[s] = argv[++i];
      } else {
        a.kv[s] = "1";
      }
    } else {
      a.pos.push_back(s);
    }
  }
  return a;
}

std::string absolutize(const std::string& p) {
  if (!p.empty() && p[0] == '/') return p;
  char buf[4096];
  if (!getcwd(buf, sizeof(buf))) return p;
  return std::string(buf) + "/" + p;
}

std::string id_rows_table(const std::vector<Id>& ids) {
  std::vector<std::vector<std::string>> rows;
  for (const auto& id : ids) rows.push_back({id.address, format_time_us(id.timestamp)});
  return make_table({"address", "timestamp"}, rows);
}

void err_line(const std::string& s) {
  std::cerr << s << std::endl;
}

struct Node {
  Args args;
  std::unique_ptr<MembershipService> ms;
  std::unique_ptr<MemberService> member;
  std::unique_ptr<LeaderService> leader;
  int base_port = 8850;

  std::string leader_host() const { return host_of(member->leader_address()); }
  int leader_rpc_port() const { return leader_port(port_of(member->leader_address())); }
  std::string call_leader(uint16_t m, const std::string& payload, int timeout_ms = 3600 * 1000) {
    return RpcClient::shared().call(leader_host(), leader_rpc_port(), m, payload, timeout_ms);
  }
};

std::unique_ptr<Node> g_node;
std::atomic<bool> g_stop{false};

void on_signal(int) { g_stop = true; }

void load_models(Executor* ex, const std::string& spec) {
  for (const auto& item : split(spec, ',')) {
    if (trim(item).empty()) continue;
    const auto eq = item.find('=');
    if (eq == std::string::npos) {
      err_line("bad --models entry (want name=path): " + item);
      continue;
    }
    const std::string name = item.substr(0, eq), path = item.substr(eq + 1);
    try {
      ex->load_model(name, path);
      DMLC_LOG_INFO("loaded " << name << " from " << path << " on " << ex->backend());
    } catch (const std::exception& e) {
      err_line("could not load model " + name + " from " + path + ": " + e.what());
    }
  }
}

void handle_line(Node& n, const std::string& line) {
  const auto t = split_ws(line);
  if (t.empty()) {
    err_line("Invalid command!");
    return;
  }
  const std::string& c = t[0];
  try {
    if (c == "list_mem" || c == "lm") {
      std::vector<std::vector<std::string>> rows;
      for (const auto& kv : n.ms->snapshot())
        if (kv.second.status == Status::Active)
          rows.push_back({kv.first.address, format_time_us(kv.first.timestamp), status_name(kv.second.status),
                          format_time_us(kv.second.last_active)});
      out_line(make_table({"address", "timestamp", "status", "last_active"}, rows));
    } else if (c == "list_self") {
      const std::string msg = "ID: " + n.ms->id().debug();
      DMLC_LOG_INFO(msg);
      out_line(msg);
    } else if (c == "join" || c == "j") {
      if (t.size() != 2) return err_line("Invalid join command!");
      std::string addr = t[1];
      if (addr.find(':') == std::string::npos) addr += ":" + std::to_string(n.base_port);
      n.ms->join(addr);
    } else if (c == "leave" || c == "l") {
      n.ms->leave();
    } else if (c == "put" || c == "p") {
      if (t.size() != 3) return err_line("Invalid put command!");
      Writer w;
      const std::string src = absolutize(t[1]);
      write_id(w, n.ms->id());
      w.str(src).str(t[2]);
      PathGrant grant(*n.member, src, /*write=*/false);  // peers may read it while the put runs
      Reader r(n.call_leader(L_PUT, w.data()));
      std::vector<Id> ids;
      const uint32_t k = r.u32();
      for (uint32_t i = 0; i < k; ++i) ids.push_back(read_id(r));
      out_line("Stored on:\n" + id_rows_table(ids));
    } else if (c == "get" || c == "g") {
      if (t.size() != 3) return err_line("Invalid get command!");
      Writer w;
      const std::string dest = absolutize(t[2]);
      w.str(t[1]);
      write_id(w, n.ms->id());
      w.str(dest);
      PathGrant grant(*n.member, dest, /*write=*/true);
      Reader r(n.call_leader(L_GET, w.data()));
      const bool found = r.boolean();
      const int v = r.i32();
      out_line(found ? "Retrieved version: " + std::to_string(v) : "File not found!");
    } else if (c == "delete" || c == "d") {
      if (t.size() != 2) return err_line("Invalid delete command!");
      Writer w;
      w.str(t[1]);
      n.call_leader(L_DELETE, w.data(), 30000);
      out_line("Deleted!");
    } else if (c == "ls") {
      if (t.size() != 2) return err_line("Invalid ls command!");
      Writer w;
      w.str(t[1]);
      Reader r(n.call_leader(L_LS, w.data(), 30000));
      const uint32_t k = r.u32();
      std::vector<std::vector<std::string>> rows;
      for (uint32_t i = 0; i < k; ++i) {
        Id id = read_id(r);
        const uint32_t nv = r.u32();
        int mx = 0;
        for (uint32_t j = 0; j < nv; ++j) mx = std::max(mx, r.i32());
        if (rows.size() < 4) rows.push_back({id.address, format_time_us(id.timestamp), std::to_string(mx)});
      }
      out_line(make_table({"address", "timestamp", "latest_version"}, rows));
    } else if (c == "store" || c == "s") {
      if (t.size() != 1) return err_line("Invalid store command!");
      std::vector<std::vector<std::string>> rows;
      for (const auto& kv : n.member->files())
        rows.push_back({kv.first, std::to_string(kv.second.empty() ? 0 : *kv.second.rbegin())});
      out_line(make_table({"filename", "latest_version"}, rows));
    } else if (c == "get-versions" || c == "gv") {
      if (t.size() != 4) return err_line("Invalid get-versions command!");
      int count;
      try {
        count = std::stoi(t[2]);
      } catch (const std::exception& e) {
        return err_line(std::string("Invalid count: ") + e.what());
      }
      const std::string dest = absolutize(t[3]);
      Writer w;
      w.str(t[1]).i32(count);
      write_id(w, n.ms->id());
      w.str(dest);
      PathGrant grant(*n.member, dest, /*write=*/true);  // and its v<N>.<name> siblings
      Reader r(n.call_leader(L_GET_VERSIONS, w.data()));
      std::set<int> vs;
      const uint32_t k = r.u32();
      for (uint32_t i = 0; i < k; ++i) vs.insert(r.i32());
      merge_versions(dest, vs);
      std::string s = "{";
      for (int v : vs) s += (s.size() > 1 ? ", " : "") + std::to_string(v);
      out_line("Retrieved versions: " + s + "}");
    } else if (c == "train" || c == "t") {
      if (t.size() != 3) return err_line("Invalid train command!");
      out_line("Starting training...");
      Writer w;
      w.str(t[1]).str(t[2]);
      Reader r(n.call_leader(L_TRAIN, w.data()));
      if (r.boolean())
        out_line("Training complete!");
      else
        err_line("Training failed: " + r.str());
    } else if (c == "predict-shard") {
      // classify an SDFS u8 shard where a replica lives (HBM-resident on GPU members)
      if (t.size() < 2 || t.size() > 3) return err_line("Invalid predict-shard command!");
      Writer w;
      w.str(t[1]).str(t.size() == 3 ? t[2] : "resnet18");
      Reader r(n.call_leader(L_PREDICT_SHARD, w.data(), 600000));
      const std::string holder = r.str();
      const int v = r.i32();
      const std::string loc = r.str();
      const int64_t us = r.i64();
      const uint32_t k = r.u32();
      std::map<int, int> hist;
      std::string head;
      for (uint32_t i = 0; i < k; ++i) {
        const int cls = r.i32();
        const double p = r.f64();
        ++hist[cls];
        if (i < 8) head += (head.empty() ? "" : " ") + std::to_string(cls) + ":" + std::to_string((int)(p * 1000) / 10.0).substr(0, 4) + "%";
      }
      char buf[256];
      snprintf(buf, sizeof(buf), "Classified %u images of %s v%d on %s [%s] in %.3f ms (%.1f images/s)", k,
               t[1].c_str(), v, holder.c_str(), loc.c_str(), us / 1000.0, us > 0 ? k * 1e6 / us : 0.0);
      out_line(buf);
      out_line("first: " + head + " | distinct classes: " + std::to_string(hist.size()));
    } else if (c == "replicas") {  // this node's staged (HBM) shard replicas
      std::string s;
      for (const auto& key : n.member->staged_replicas()) s += (s.empty() ? "" : " ") + key;
      out_line("staged: " + (s.empty() ? std::string("none") : s) + " in " +
               (n.member->executor() ? n.member->executor()->blob_location() : std::string("-")));
    } else if (c == "predict") {
      // predict                 start / resume the jobs (reference: no arguments)
      // predict <shard> ...     the jobs classify these labelled SDFS u8 shards
      //                         (resident in the replica holders' HBM) instead
      // predict dataset         back to the dataset's per-label JPEGs
      std::string resp;
      if (t.size() == 1) {
        resp = n.call_leader(L_PREDICT, "", 30000);
      } else {
        Writer w;
        const bool dataset = t.size() == 2 && t[1] == "dataset";
        w.u32(dataset ? 0u : (uint32_t)(t.size() - 1));
        if (!dataset)
          for (size_t i = 1; i < t.size(); ++i) w.str(t[i]);
        resp = n.call_leader(L_PREDICT, w.data(), 30000);
      }
      if (resp.size() >= 4) {  // notes: e.g. a running job kept its source
        Reader r(resp);
        const uint32_t k = r.u32();
        for (uint32_t i = 0; i < k && i < 64; ++i) out_line("predict: " + r.str());
      }
    } else if (c == "jobs") {
      if (t.size() != 1) return err_line("Invalid jobs command!");
      Reader r(n.call_leader(L_JOBS, "", 5000));
      const uint32_t k = r.u32();
      for (uint32_t i = 0; i < k; ++i) out_line(format_job_report((int)i + 1, read_job(r)));
    } else if (c == "jobs-dump") {
      // machine-readable job state (per-query latency and completion time)
      if (t.size() != 2) return err_line("Invalid jobs-dump command!");
      Reader r(n.call_leader(L_JOBS, "", 5000));
      const uint32_t k = r.u32();
      std::ofstream f(absolutize(t[1]));
      f << "[";
      for (uint32_t i = 0; i < k; ++i) {
        const Job j = read_job(r);
        f << (i ? "," : "") << "{\"model\":\"" << j.model_name << "\",\"finished\":" << j.finished
          << ",\"correct\":" << j.correct << ",\"started_us\":" << j.started_us
          << ",\"first_done_us\":" << j.first_done_us << ",\"assigned\":" << j.assigned.size()
          << ",\"durations_us\":[";
        for (size_t q = 0; q < j.durations_us.size(); ++q) f << (q ? "," : "") << j.durations_us[q];
        f << "],\"done_us\":[";
        for (size_t q = 0; q < j.done_us.size(); ++q) f << (q ? "," : "") << j.done_us[q];
        f << "]}";
      }
      f << "]\n";
      out_line("dumped " + std::to_string(k) + " jobs");
    } else if (c == "assign") {
      if (t.size() != 1) return err_line("Invalid assign command!");
      Reader r(n.call_leader(L_JOBS, "", 5000));
      const uint32_t k = r.u32();
      for (uint32_t i = 0; i < k; ++i) {
        const Job j = read_job(r);
        out_line("Job " + std::to_string(i + 1) + ":\n" + id_rows_table(j.assigned));
      }
    } else if (c == "fault") {
      // fault drop <p> | pause | resume | partition <addr> | heal | gpu <device>
      if (t.size() >= 3 && t[1] == "drop") n.ms->set_drop_rate(std::stod(t[2]));
      else if (t.size() == 2 && t[1] == "pause") n.ms->set_paused(true);
      else if (t.size() == 2 && t[1] == "resume") n.ms->set_paused(false);
      else if (t.size() == 3 && t[1] == "partition") n.ms->partition(t[2]);
      else if (t.size() == 2 && t[1] == "heal") n.ms->heal();
      else if (t.size() == 3 && t[1] == "gpu" && n.member->executor()) n.member->executor()->lose_device(std::stoi(t[2]));
      else return err_line("Invalid fault command!");
      out_line("ok");
    } else if (c == "info") {
      out_line("id " + n.ms->id().address + " leader " + n.member->leader_address() + " executor " +
               (n.member->executor() ? n.member->executor()->backend() : std::string("none")) + " sent " +
               std::to_string(n.ms->sent()) + " received " + std::to_string(n.ms->received()));
      if (Executor* ex = n.member->executor()) {
        out_line("placement " + ex->placement());
        const CacheStats cs = ex->cache_stats();
        out_line("cache hits " + std::to_string(cs.hits) + " misses " + std::to_string(cs.misses) + " staged " +
                 std::to_string(cs.staged) + " evictions " + std::to_string(cs.evictions) + " entries " +
                 std::to_string(cs.entries) + " bytes " + std::to_string(cs.bytes) + " capacity " +
                 std::to_string(cs.capacity) + " prefetched " + std::to_string(n.member->prefetched()));
      }
    } else if (c == "prefetch") {
      // stage the dataset's query images into the executor's (HBM) cache
      out_line(n.member->start_prefetch() ? "prefetch started" : "prefetch unavailable or running");
    } else if (c == "sleep") {
      if (t.size() == 2) std::this_thread::sleep_for(std::chrono::milliseconds(std::stoi(t[1])));
    } else if (c == "quit" || c == "exit") {
      g_stop = true;
    } else {
      DMLC_LOG_WARN("Unknown command");
      err_line("Unknown command");
    }
  } catch (const std::exception& e) {
    err_line("Error: " + std::string(e.what()));
  }
}

int run_node(const Args& a) {
  auto n = std::make_unique<Node>();
  n->args = a;
  n->base_port = a.geti("port", 8850);
  const std::string host = a.get("host", "127.0.0.1");
  const std::string self = host + ":" + std::to_string(n->base_port);
  const std::string workdir = a.get("workdir", "dmlc-" + std::to_string(n->base_port));
  ::mkdir(workdir.c_str(), 0755);
  Logger::get().open(a.get("log", workdir + "/" + host + "-" + std::to_string(n->base_port) + ".log"));

  MembershipConfig mc;
  mc.bind_host = a.get("bind", "0.0.0.0");
  mc.host = host;
  mc.port = n->base_port;
  mc.ping_ms = a.geti("ping-ms", 1000);
  mc.detect_ms = a.geti("detect-ms", 1000);
  mc.fail_ms = a.geti("fail-ms", 3000);
  mc.tombstone_ms = a.geti("tombstone-ms", 30000);
  mc.clock_skew_us = (int64_t)a.geti("clock-skew-ms", 0) * 1000;
  n->ms = std::make_unique<MembershipService>(mc);
  n->ms->start();

  std::vector<std::string> leaders;
  for (const auto& l : split(a.get("leaders", self), ','))
    if (!trim(l).empty()) leaders.push_back(trim(l));
  const Labels labels = Labels::load(a.get("labels", "synset_words.txt"));

  std::unique_ptr<Executor> ex;
  try {
    // --gpus N: this node serves on GPUs device .. device+N-1 (one engine
    // per GPU, query batches scattered over RCCL); --devices a,b,c lists them
    std::vector<int> devs;
    if (!a.get("devices", "").empty()) {
      for (const auto& d : split(a.get("devices", ""), ','))
        if (!trim(d).empty()) devs.push_back(std::stoi(trim(d)));
    } else {
      for (int i = 0; i < std::max(1, a.geti("gpus", 1)); ++i) devs.push_back(a.geti("device", 0) + i);
    }
    ex = make_executor(a.get("executor", "auto"), devs, a.geti("max-batch", 256),
                       (size_t)a.geti("hbm-cache-mb", 4096) << 20, a.geti("min-shard", 32), a.geti("lanes", 2),
                       a.geti("batch-window-us", 200));
    if (ex) {
      // the GPUs are split between the jobs in this order (first floor(n/2)
      // to the first job, src/services.rs:199-211)
      std::vector<std::string> jobs;
      for (const auto& m : split(a.get("jobs", "resnet18,alexnet"), ','))
        if (!trim(m).empty()) jobs.push_back(trim(m));
      ex->set_jobs(jobs);
      load_models(ex.get(), a.get("models", ""));
    }
  } catch (const std::exception& e) {
    err_line(std::string("executor unavailable: ") + e.what());
  }

  MemberConfig mcfg;
  mcfg.bind_host = mc.bind_host;
  mcfg.workdir = workdir;
  mcfg.dataset_dir = a.get("dataset", "test_files/imagenet_1k/train");
  mcfg.leader_candidates = leaders;
  mcfg.check_ms = a.geti("bg-ms", 3000);
  mcfg.watch_ms = a.geti("watch-ms", 250);
  mcfg.hbm_replicas = !a.has("no-hbm-replicas");
  n->member = std::make_unique<MemberService>(mcfg, n->ms.get(), std::move(ex), labels);
  n->member->start(n->base_port);
  if (a.has("prefetch")) n->member->start_prefetch();

  bool candidate = false;
  for (const auto& l : leaders) candidate |= (l == self);
  if (candidate) {
    LeaderConfig lc;
    lc.bind_host = mc.bind_host;
    lc.replication = a.geti("rf", 4);
    lc.bg_ms = a.geti("bg-ms", 3000);
    lc.standby_copy_ms = a.geti("standby-copy-ms", 250);
    lc.query_interval_ms = a.geti("query-interval-ms", 500);
    lc.query_batch = a.geti("query-batch", 1);
    lc.max_inflight = a.geti("max-inflight", 32);
    lc.adaptive_window = a.geti("adaptive-window", 0);
    lc.job_limit = a.geti("job-limit", 0);
    lc.print_predictions = !a.has("quiet-predictions");
    lc.new_conn_per_query = a.has("new-conn-per-query");
    lc.max_attempts = a.geti("max-attempts", 3);
    lc.query_timeout_ms = a.geti("query-timeout-ms", 120000);
    lc.query_timeout_min_ms = a.geti("query-timeout-min-ms", 1000);
    lc.job_models.clear();
    for (const auto& m : split(a.get("jobs", "resnet18,alexnet"), ','))
      if (!trim(m).empty()) lc.job_models.push_back(trim(m));
    n->leader = std::make_unique<LeaderService>(lc, n->ms.get(), n->member.get(), labels);
    n->leader->start(n->base_port);
  }
  if (a.has("join")) n->ms->join(a.get("join"));

  signal(SIGTERM, on_signal);
  signal(SIGINT, on_signal);
  signal(SIGPIPE, SIG_IGN);
  g_node = std::move(n);
  Node& node = *g_node;
  if (a.has("daemon")) {
    while (!g_stop.load()) std::this_thread::sleep_for(std::chrono::milliseconds(100));
  } else {
    std::string line;
    const bool ack = a.has("ack");  // scripted drivers: mark the end of each command's output
    while (!g_stop.load() && std::getline(std::cin, line)) {
      handle_line(node, line);
      if (ack) out_line("<<done>>");
    }
    if (a.has("stay")) while (!g_stop.load()) std::this_thread::sleep_for(std::chrono::milliseconds(100));
  }
  // orderly shutdown
  if (node.leader) node.leader->stop();
  node.member->stop();
  node.ms->stop();
  RpcClient::shared().clear();
  Logger::get().close();
  std::fflush(stdout);
  _exit(0);  // detached worker threads may still hold RPC sockets
}

int run_classify(const Args& a) {
  const std::string model = a.get("model", "alexnet");
  std::vector<Image> imgs;
  for (const auto& p : split(a.get("image"), ',')) imgs.push_back(decode_jpeg_file(p));
  // all images in one batch (one forward on the GPU executor)
  auto ex = make_executor(a.get("executor", "cpu"), a.geti("device", 0), std::max<int>(1, (int)imgs.size()));
  if (!ex) throw std::runtime_error("no inference executor in this build");
  ex->load_model(model, a.get("weights"));
  const Labels labels = Labels::load(a.get("labels", "synset_words.txt"));
  const int64_t t0 = steady_us();
  const auto preds = ex->predict(model, imgs);
  const int64_t dt = steady_us() - t0;
  for (size_t i = 0; i < preds.size(); ++i) {
    char buf[64];
    snprintf(buf, sizeof(buf), "%.2f%%", preds[i].prob * 100.0);
    std::cout << model << " [" << ex->backend() << "] " << labels.text(preds[i].class_idx) << " (" << buf
              << ") class=" << preds[i].class_idx << std::endl;
  }
  std::cout << "latency_ms " << dt / 1000.0 << std::endl;
  return 0;
}

}  // namespace

int main(int argc, char** argv) {
  if (argc >= 2 && std::string(argv[1]) == "selftest") return run_selftest();
  if (argc >= 2 && std::string(argv[1]) == "classify") return run_classify(parse(argc, argv, 2));
  if (argc >= 2 && (std::string(argv[1]) == "--help" || std::string(argv[1]) == "-h")) {
    std::cout << "usage: dmlc-node [--host H] [--port P] [--leaders h:p,...] [--workdir D] [--dataset D]\n"
                 "                 [--labels F] [--models name=path,...] [--executor auto|gpu|cpu] [--device N]\n"
                 "                 [--gpus N | --devices a,b,...] [--min-shard 32] [--lanes 2]\n"
                 "                 [--rf 4] [--ping-ms 1000] [--fail-ms 3000] [--bg-ms 3000] [--standby-copy-ms 250]\n"
                 "                 [--query-interval-ms 500] [--adaptive-window 0] [--query-batch 1] [--jobs resnet18,alexnet]\n"
                 "                 [--join h:p] [--daemon] [--stay] [--quiet-predictions] [--new-conn-per-query]\n"
                 "                 [--max-attempts 3] [--watch-ms 250] [--query-timeout-ms 120000]\n"
                 "                 [--query-timeout-min-ms 1000]\n"
                 "                 [--max-batch 256] [--batch-window-us 200] [--hbm-cache-mb 4096] [--prefetch]\n"
                 "       dmlc-node selftest\n"
                 "       dmlc-node classify --model M --weights W.ot --labels L --image I.JPEG [--executor cpu|gpu]\n";
    return 0;
  }
  return run_node(parse(argc, argv, 1));
}
