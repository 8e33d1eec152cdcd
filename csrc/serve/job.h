// Inference job bookkeeping and latency statistics.
//
// Reference: `Job{model_name, finished_prediction_count,
// correct_prediction_count, query_durations, assigned_member_ids}` and
// `add_query_result` (src/services.rs:54-81); the `jobs` report computes
// accuracy and mean/std/median/p90/p95/p99 with the `histogram` crate at
// millisecond resolution (src/main.rs:271-314). Here durations are kept in
// microseconds and percentiles are exact (sorted), reported in ms with
// sub-millisecond resolution.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "../control/membership.h"
#include "../control/wire.h"

namespace dmlc {
namespace ctl {

struct Job {
  std::string model_name;
  int32_t finished = 0;
  int32_t correct = 0;
  std::vector<int64_t> durations_us;
  std::vector<int64_t> done_us;  // wall-clock completion time of each query
  std::vector<Id> assigned;
  int64_t started_us = 0;   // wall clock when the job first issued a query
  int64_t first_done_us = 0;
  // Time the job has been running, summed over the leaders that ran it,
  // each measured on its own steady clock (the Throughput line; wall clocks
  // of different leaders are never subtracted from each other).
  int64_t elapsed_us = 0;
  // Where the queries come from: empty = the dataset's label list (the
  // reference, src/services.rs:410-411); else SDFS shard names, in order
  // (labelled u8 shards, csrc/serve/shard.h: BASELINE config 3).
  std::vector<std::string> source;
  int32_t failed = 0;  // images of queries no member answered after every retry (dropped)

  void add_result(bool ok, int64_t dur_us, int64_t done_wall_us = 0) {
    ++finished;
    if (ok) ++correct;
    durations_us.push_back(dur_us);
    done_us.push_back(done_wall_us);
  }
};

void write_job(Writer& w, const Job& j);
Job read_job(Reader& r);
// Incremental form for the standby copy: per-query vectors from index
// `from` on (the standby already holds the first `from`).
void write_job_delta(Writer& w, const Job& j, uint32_t from);
// Applies a delta onto `j` (which holds `from` entries); false if `j` does
// not line up (the standby then asks for everything again).
bool read_job_delta(Reader& r, Job& j);
// A standby that takes over resumes the jobs when its copy shows them
// running: any job that issued a query or has a completed one.
bool jobs_running(const std::vector<Job>& jobs);

struct LatencyStats {
  size_t count = 0;
  double mean = 0, stddev = 0, p50 = 0, p90 = 0, p95 = 0, p99 = 0, max = 0;  // ms
};
LatencyStats latency_stats(const std::vector<int64_t>& durations_us);
double percentile_sorted(const std::vector<double>& sorted, double q);

// The `jobs` report block (same fields and layout as src/main.rs:291-309).
std::string format_job_report(int n, const Job& j);

}  // namespace ctl
}  // namespace dmlc
