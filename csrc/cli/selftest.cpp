// `dmlc-node selftest`: C++ unit tests of the control-plane pure logic.
// Includes the reference's three ring-neighbour tests (src/utils.rs:29-92)
// as the spec for symmetric_ring_neighbors.
#include <cstdio>
#include <functional>
#include <string>
#include <vector>

#include "../control/common.h"
#include "../control/membership.h"
#include "../control/ring.h"
#include "../control/sdfs.h"
#include "../control/table.h"
#include "../serve/job.h"

namespace dmlc {
namespace ctl {

namespace {
int g_fail = 0, g_pass = 0;
#define CHECK(cond)                                                         \
  do {                                                                      \
    if (!(cond)) {                                                          \
      std::fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #cond);  \
      ++g_fail;                                                             \
    } else {                                                                \
      ++g_pass;                                                             \
    }                                                                       \
  } while (0)

std::map<int, std::string> letters(int n) {
  std::map<int, std::string> m;
  for (int i = 1; i <= n; ++i) m[i] = std::string(1, (char)('a' + i - 1));
  return m;
}
auto all = [](const std::pair<const int, std::string>&) { return true; };

void test_ring() {
  CHECK((symmetric_ring_neighbors(letters(26), 13, 3, all) == std::vector<int>{12, 14, 11, 15, 10, 16}));
  CHECK((symmetric_ring_neighbors(letters(8), 8, 3, all) == std::vector<int>{7, 1, 6, 2, 5, 3}));
  CHECK((symmetric_ring_neighbors(letters(3), 2, 3, all) == std::vector<int>{1, 3}));
  // predicate filtering + k=2 as used by the pinger
  auto odd = [](const std::pair<const int, std::string>& e) { return e.first % 2 == 1; };
  CHECK((symmetric_ring_neighbors(letters(10), 5, 2, odd) == std::vector<int>{3, 7, 1, 9}));
  CHECK((symmetric_ring_neighbors(letters(1), 1, 2, all).empty()));
}

Id mk(const std::string& a, int64_t t) { return Id{a, t}; }

void test_merge() {
  MembershipList local, remote;
  CHECK(!merge_membership(local, remote));  // empty local: not in a group
  local[mk("a:1", 1)] = {Status::Active, 100};
  remote[mk("a:1", 1)] = {Status::Active, 90};
  CHECK(!merge_membership(local, remote));  // older info ignored
  remote[mk("a:1", 1)] = {Status::Failed, 100};
  std::vector<std::string> ch;
  CHECK(merge_membership(local, remote, {}, &ch));  // tie: Failed wins
  CHECK(local[mk("a:1", 1)].status == Status::Failed);
  CHECK(ch.size() == 1);
  remote[mk("a:1", 1)] = {Status::Active, 100};
  CHECK(!merge_membership(local, remote));  // tie does not resurrect
  remote[mk("a:1", 1)] = {Status::Active, 101};
  CHECK(merge_membership(local, remote));  // newer heartbeat wins
  CHECK(local[mk("a:1", 1)].status == Status::Active);
  remote.clear();
  remote[mk("b:1", 5)] = {Status::Active, 5};
  std::set<Id> dead = {mk("c:1", 7)};
  remote[mk("c:1", 7)] = {Status::Active, 9};
  CHECK(merge_membership(local, remote, dead));
  CHECK(local.count(mk("b:1", 5)) == 1 && local.count(mk("c:1", 7)) == 0);
}

void test_codec() {
  Message m;
  m.type = MsgType::Ping;
  m.sender = mk("127.0.0.1:9000", 123456789);
  m.list[mk("x:1", 1)] = {Status::Active, 11};
  m.list[mk("y:2", 2)] = {Status::Failed, 22};
  const std::string enc = encode_message(m);
  Message d = decode_message(enc.data(), enc.size());
  CHECK(d.type == MsgType::Ping && d.sender == m.sender && d.list == m.list);
  Message a;
  a.type = MsgType::Ack;
  a.sender = m.sender;
  a.last_active = 77;
  const std::string e2 = encode_message(a);
  Message d2 = decode_message(e2.data(), e2.size());
  CHECK(d2.type == MsgType::Ack && d2.last_active == 77);
  bool threw = false;
  try {
    decode_message(e2.data(), e2.size() - 3);
  } catch (const WireError&) {
    threw = true;
  }
  CHECK(threw);
}

void test_sdfs_naming() {
  CHECK(storage_filename("a.txt", 3) == "v3.a.txt");
  CHECK(storage_filename("dir/x:y", 1) == "v1.dirxy");
  CHECK(version_delimiter(1) == "============== Version 1 ===============");
  CHECK(version_delimiter(12).size() == 40);
  CHECK(versioned_sibling("/tmp/out.txt", 4) == "/tmp/v4.out.txt");
  std::vector<Id> c = {mk("a:1", 1), mk("b:1", 1), mk("c:1", 1), mk("d:1", 1), mk("e:1", 1)};
  auto r1 = choose_replicas("file", c, 4), r2 = choose_replicas("file", c, 4);
  CHECK(r1 == r2 && r1.size() == 4);
  CHECK(choose_replicas("file", std::vector<Id>(c.begin(), c.begin() + 2), 4).size() == 2);
  Directory d;
  d["f"][mk("a:1", 1)] = {1, 2};
  d["g"][mk("b:1", 2)] = {7};
  Writer w;
  write_directory(w, d);
  Reader rd(w.data());
  CHECK(read_directory(rd) == d);
}

void test_stats() {
  std::vector<int64_t> us;
  for (int i = 1; i <= 100; ++i) us.push_back(i * 1000);
  const LatencyStats s = latency_stats(us);
  CHECK(s.count == 100);
  CHECK(std::abs(s.mean - 50.5) < 1e-9);
  CHECK(std::abs(s.p50 - 50.5) < 1e-9);
  CHECK(std::abs(s.p99 - 99.01) < 1e-9);
  Job j;
  j.model_name = "resnet18";
  j.add_result(true, 1500);
  j.add_result(false, 2500);
  j.assigned.push_back(mk("a:1", 3));
  Writer w;
  write_job(w, j);
  Reader r(w.data());
  Job k = read_job(r);
  CHECK(k.model_name == "resnet18" && k.finished == 2 && k.correct == 1 && k.durations_us == j.durations_us &&
        k.assigned.size() == 1);
  const std::string rep = format_job_report(1, j);
  CHECK(rep.find("Accuracy: 1/2 = 50.00%") != std::string::npos);
  CHECK(rep.find("2 total, 2.000 ms avg") != std::string::npos);
}

// The take-over's resume decision on a standby's copy (LeaderService::
// succession_loop): job 0 issued queries but had no answer yet when the copy
// was taken, job 1 had answers; the started stamp travels in the delta copy.
void test_resume_decision() {
  Job a, b;
  a.model_name = "resnet18";
  b.model_name = "alexnet";
  CHECK(!jobs_running({a, b}));
  a.started_us = 123;
  b.add_result(true, 1000);
  CHECK(jobs_running({a, Job{}}));
  CHECK(jobs_running({Job{}, b}));
  Writer w;
  write_job_delta(w, a, 0);
  Reader r(w.data());
  Job copy;
  CHECK(read_job_delta(r, copy));
  CHECK(copy.started_us == 123 && copy.durations_us.empty() && jobs_running({copy, Job{}}));
}

void test_table() {
  const std::string t = make_table({"a", "bb"}, {{"xyz", "1"}});
  CHECK(t == "+-----+----+\n| a   | bb |\n+-----+----+\n| xyz | 1  |\n+-----+----+");
}

}  // namespace

int run_selftest() {
  test_ring();
  test_merge();
  test_codec();
  test_sdfs_naming();
  test_stats();
  test_resume_decision();
  test_table();
  std::printf("selftest: %d passed, %d failed\n", g_pass, g_fail);
  return g_fail == 0 ? 0 : 1;
}

}  // namespace ctl
}  // namespace dmlc
