#include "job.h"

#include <algorithm>
#include <cmath>
#include <cstdio>

namespace dmlc {
namespace ctl {

namespace {
// A count read off the wire may not promise more elements than the bytes
// that are left (a forged count would otherwise allocate gigabytes).
uint32_t bounded(Reader& r, size_t elem_bytes) {
  const uint32_t n = r.u32();
  if ((uint64_t)n * elem_bytes > r.left()) throw WireError("count exceeds message");
  return n;
}
void write_tail(Writer& w, const Job& j) {
  w.u32((uint32_t)j.source.size());
  for (const auto& s : j.source) w.str(s);
  w.i32(j.failed);
}
void read_tail(Reader& r, Job& j) {
  const uint32_t n = bounded(r, 4);
  j.source.clear();
  for (uint32_t i = 0; i < n; ++i) j.source.push_back(r.str());
  j.failed = r.i32();
}
}  // namespace

void write_job(Writer& w, const Job& j) {
  w.str(j.model_name);
  w.i32(j.finished);
  w.i32(j.correct);
  w.u32((uint32_t)j.durations_us.size());
  for (int64_t d : j.durations_us) w.i64(d);
  w.u32((uint32_t)j.done_us.size());
  for (int64_t d : j.done_us) w.i64(d);
  w.u32((uint32_t)j.assigned.size());
  for (const auto& id : j.assigned) write_id(w, id);
  w.i64(j.started_us);
  w.i64(j.first_done_us);
  w.i64(j.elapsed_us);
  write_tail(w, j);
}

void write_job_delta(Writer& w, const Job& j, uint32_t from) {
  if (from > j.durations_us.size() || from > j.done_us.size()) from = 0;
  w.u32(from);
  w.str(j.model_name);
  w.i32(j.finished);
  w.i32(j.correct);
  w.u32((uint32_t)(j.durations_us.size() - from));
  for (size_t i = from; i < j.durations_us.size(); ++i) w.i64(j.durations_us[i]);
  w.u32((uint32_t)(j.done_us.size() - from));
  for (size_t i = from; i < j.done_us.size(); ++i) w.i64(j.done_us[i]);
  w.u32((uint32_t)j.assigned.size());
  for (const auto& id : j.assigned) write_id(w, id);
  w.i64(j.started_us);
  w.i64(j.first_done_us);
  w.i64(j.elapsed_us);
  write_tail(w, j);
}

bool read_job_delta(Reader& r, Job& j) {
  const uint32_t from = r.u32();
  Job d;
  d.model_name = r.str();
  d.finished = r.i32();
  d.correct = r.i32();
  uint32_t n = bounded(r, 8);
  std::vector<int64_t> dur(n), done;
  for (uint32_t i = 0; i < n; ++i) dur[i] = r.i64();
  n = bounded(r, 8);
  done.resize(n);
  for (uint32_t i = 0; i < n; ++i) done[i] = r.i64();
  n = r.u32();
  for (uint32_t i = 0; i < n; ++i) d.assigned.push_back(read_id(r));
  d.started_us = r.i64();
  d.first_done_us = r.i64();
  d.elapsed_us = r.i64();
  read_tail(r, d);
  if (from > 0 && (j.durations_us.size() != from || j.done_us.size() != from || j.model_name != d.model_name ||
                   j.source != d.source))
    return false;
  d.durations_us = from ? j.durations_us : std::vector<int64_t>();
  d.done_us = from ? j.done_us : std::vector<int64_t>();
  d.durations_us.insert(d.durations_us.end(), dur.begin(), dur.end());
  d.done_us.insert(d.done_us.end(), done.begin(), done.end());
  j = std::move(d);
  return true;
}

bool jobs_running(const std::vector<Job>& jobs) {
  for (const auto& j : jobs)
    if (j.started_us != 0 || !j.durations_us.empty()) return true;
  return false;
}

Job read_job(Reader& r) {
  Job j;
  j.model_name = r.str();
  j.finished = r.i32();
  j.correct = r.i32();
  uint32_t n = bounded(r, 8);
  j.durations_us.resize(n);
  for (uint32_t i = 0; i < n; ++i) j.durations_us[i] = r.i64();
  n = bounded(r, 8);
  j.done_us.resize(n);
  for (uint32_t i = 0; i < n; ++i) j.done_us[i] = r.i64();
  n = r.u32();
  for (uint32_t i = 0; i < n; ++i) j.assigned.push_back(read_id(r));
  j.started_us = r.i64();
  j.first_done_us = r.i64();
  j.elapsed_us = r.i64();
  read_tail(r, j);
  return j;
}

double percentile_sorted(const std::vector<double>& s, double q) {
  if (s.empty()) return 0;
  const double k = (s.size() - 1) * q / 100.0;
  const size_t lo = (size_t)k, hi = std::min(lo + 1, s.size() - 1);
  return s[lo] + (s[hi] - s[lo]) * (k - lo);
}

LatencyStats latency_stats(const std::vector<int64_t>& d) {
  LatencyStats st;
  st.count = d.size();
  if (d.empty()) return st;
  std::vector<double> ms(d.size());
  for (size_t i = 0; i < d.size(); ++i) ms[i] = d[i] / 1000.0;
  double sum = 0;
  for (double v : ms) sum += v;
  st.mean = sum / ms.size();
  double var = 0;
  for (double v : ms) var += (v - st.mean) * (v - st.mean);
  st.stddev = std::sqrt(var / ms.size());
  std::sort(ms.begin(), ms.end());
  st.p50 = percentile_sorted(ms, 50);
  st.p90 = percentile_sorted(ms, 90);
  st.p95 = percentile_sorted(ms, 95);
  st.p99 = percentile_sorted(ms, 99);
  st.max = ms.back();
  return st;
}

std::string format_job_report(int n, const Job& j) {
  const LatencyStats s = latency_stats(j.durations_us);
  const double acc = j.finished > 0 ? 100.0 * j.correct / j.finished : 0.0;
  char buf[1024];
  snprintf(buf, sizeof(buf),
           "Job %d:\n"
           "\tModel: %s\n"
           "\tAccuracy: %d/%d = %.2f%%\n"
           "\tQueries: %zu total, %.3f ms avg, %.3f ms std, %.3f ms median,\n"
           "\t\t%.3f ms p90, %.3f ms p95, %.3f ms p99",
           n, j.model_name.c_str(), j.correct, j.finished, acc, s.count, s.mean, s.stddev, s.p50, s.p90, s.p95,
           s.p99);
  std::string out = buf;
  if (!j.source.empty()) {
    std::string src;
    for (const auto& x : j.source) src += (src.empty() ? "" : ", ") + x;
    out += "\n\tData: SDFS shards " + src;
  }
  if (j.failed > 0) out += "\n\tUnanswered: " + std::to_string(j.failed) + " images (dropped after retries)";
  if (j.finished > 0 && j.elapsed_us > 0) {
    const double secs = j.elapsed_us * 1e-6;
    snprintf(buf, sizeof(buf), "\n\tThroughput: %.2f queries/s", j.finished / secs);
    out += buf;
  }
  return out;
}

}  // namespace ctl
}  // namespace dmlc
