// Leader service: SDFS metadata + replication, inference job coordinator,
// fair-share scheduler, fail-over with job resume.
//
// Reference: tarpc `Leader` (get, get_versions, put, delete, ls, train,
// predict, jobs, alive; src/services.rs:38-160), LeaderState::new background
// loops (re-replication, job assignment, succession/job-state copy;
// src/services.rs:163-242), put_version/get_version (:283-405) and run_job
// (:407-433).
// Differences: bytes move member-to-member over RPC instead
// of scp; standbys copy the SDFS directory along with the jobs (#5); delete
// removes replica files (#6); train hot-swaps weights on every member (#7);
// a job with no assigned member borrows all active members instead of
// silently skipping queries; queries can be batched (query_batch) and the
// tick is configurable (reference: 1 query / 0.5 s / job).
// Adaptive rate (the report claims the leader adjusts the
// query rate, the code has a fixed tick): with adaptive_window > 0 a job has
// no tick; it keeps adaptive_window queries in flight per assigned member and
// sends each to the member with the fewest of them outstanding, so its rate
// follows what its members can serve (rate = window / latency) and a slow or
// overloaded member gets fewer queries.
#pragma once
#include <atomic>
#include <condition_variable>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <optional>
#include <random>
#include <set>
#include <string>
#include <thread>
#include <vector>

#include "../control/member.h"
#include "../control/membership.h"
#include "../control/rpc.h"
#include "../control/sdfs.h"
#include "job.h"

namespace dmlc {
namespace ctl {

struct LeaderConfig {
  std::string bind_host = "0.0.0.0";
  int replication = 4;
  int bg_ms = 3000;
  // A standby copies the leader's job progress this often (incremental: the
  // queries completed since its last copy). The reference copies at its
  // background period; answers completed after the last copy are redone by a
  // successor, and show up as part of the fail-over gap.
  int standby_copy_ms = 250;
  int query_interval_ms = 500;
  int query_batch = 1;
  int max_inflight = 32;
  int adaptive_window = 0;  // >0: closed-loop rate, queries in flight per member
  int job_limit = 0;  // queries per job (0 = every label, as the reference)
  bool print_predictions = true;
  bool new_conn_per_query = false;  // the reference's per-query TCP connect (src/services.rs:420)
  int max_attempts = 3;  // sends of one query (across members and requeues) before it is dropped
  // A query's RPC deadline: 10 x the job's recent p99 query time, within
  // [query_timeout_min_ms, query_timeout_ms] (query_timeout_ms until 20
  // queries have completed). A hung member (its socket open, nothing
  // answering) then costs a query about that long before it is sent
  // elsewhere, not the fixed ceiling.
  int query_timeout_ms = 120000;
  int query_timeout_min_ms = 1000;
  std::vector<std::string> job_models = {"resnet18", "alexnet"};
};

class LeaderService {
 public:
  LeaderService(LeaderConfig cfg, MembershipService* ms, MemberService* member, Labels labels);
  ~LeaderService();
  void start(int base_port);
  void stop();

  bool is_leader() const;
  // RPC bodies (also used locally)
  std::set<Id> put(const Id& src, const std::string& src_path, const std::string& filename);
  int get(const std::string& filename, const Id& dest, const std::string& dest_path);
  std::set<int> get_versions(const std::string& filename, int count, const Id& dest, const std::string& dest_path);
  void del(const std::string& filename);
  std::vector<std::pair<Id, std::vector<int>>> ls(const std::string& filename);
  void train(const std::string& filename, const std::string& model_name);
  // Start the jobs that are not running. shards == nullptr: each job keeps
  // its source (resume); otherwise the jobs take their queries from these
  // SDFS shards (empty: the dataset's labels), starting over if that changes.
  // Returns notes for the caller: a job still running keeps its source
  // (a different one is not applied until it is idle).
  std::vector<std::string> predict(const std::vector<std::string>* shards = nullptr);
  std::vector<Job> jobs() const;

 private:
  void register_handlers();
  int latest_version(const std::string& f) const;
  std::set<Id> put_version(const Id* src_id, const std::string* src_spec, const std::string& filename, int version);
  bool copy_to(const Id& src, const std::string& src_spec, const Id& dest, const std::string& dest_spec);
  std::optional<Id> get_version(const std::string& filename, int version, const Id& dest, const std::string& dest_spec);
  // One query's images: [first, first + n) of the job's index space, sent
  // `attempts` times so far.
  struct Range {
    size_t first = 0, n = 0;
    int attempts = 0;
  };
  // A labelled shard of a job's source: global indices [start, start + n).
  struct Seg {
    std::string file;
    size_t start = 0, n = 0;
    uint32_t label0 = 0;
  };
  void run_job(size_t j);
  bool load_segments(size_t j, const std::vector<std::string>& source);
  std::vector<Id> shard_holders(const std::string& file);
  void rereplicate_loop();
  void assign_loop();
  void succession_loop();
  void standby_copy_loop();
  int query_timeout(size_t j) const;  // under mu_
  void sleep_bg();

  LeaderConfig cfg_;
  MembershipService* ms_;
  MemberService* member_;
  Labels labels_;
  std::unique_ptr<RpcServer> server_;
  std::string self_;  // base address
  mutable std::mutex mu_;
  Directory dir_;
  std::vector<Job> jobs_;
  std::vector<bool> running_;
  std::atomic<bool> stop_{false};
  bool leading_ = false;  // took over as leader (the standby copy stops applying), under mu_
  std::vector<std::thread> loops_;
  std::mutex runners_mu_;
  std::vector<std::thread> runners_;
  std::atomic<int> inflight_{0};
  std::unique_ptr<std::atomic<int>[]> job_inflight_;  // per job (adaptive window)
  std::map<std::string, int> member_inflight_;         // per member address, under rng_mu_
  Id pick_target(const std::vector<Id>& pool);
  bool benched(const std::string& addr);  // under rng_mu_
  std::optional<Id> retry_target(size_t j, const std::set<std::string>& tried, const std::vector<Id>* only);
  void query(size_t j, const std::string& model, Id target, Range range, int64_t run0, int64_t elapsed0);
  void submit(std::function<void()> task);
  std::map<std::string, int64_t> bench_until_;          // member -> steady us, under rng_mu_
  std::vector<std::deque<Range>> retry_;  // per job: queries handed back, under mu_
  std::vector<std::vector<Seg>> segs_;    // per job: shard segments of its source, under mu_
  std::mutex pool_mu_;
  std::condition_variable pool_cv_;
  std::deque<std::function<void()>> tasks_;
  std::vector<std::thread> workers_;
  bool pool_stop_ = false;
  std::mutex rng_mu_;
  std::mt19937_64 rng_{std::random_device{}()};
};

}  // namespace ctl
}  // namespace dmlc
