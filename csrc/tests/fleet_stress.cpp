// Sanitizer stress of the serving fleet's coalesced direct path
// (csrc/comm/fleet.cpp Fleet::direct) on host workers and the host
// communicator: many threads send small queries to one model; some queries
// fail inside their stage function (a bad image, as the GPU executor's JPEG
// stage throws); a GPU is lost halfway through. Built twice by tools/build.py,
// with -fsanitize=thread and with -fsanitize=address,undefined
// (build/bin/dmlc-fleet-stress-{tsan,asan}); tests/test_fleet_cpu.py runs both.
//
// Exit status 0 iff every good query got exactly its expected answers and
// every bad query got its own error and no other query did.
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <random>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "../comm/dp.h"
#include "../comm/fleet.h"

using namespace dmlc;

namespace {
constexpr int H = 4, W = 4;
constexpr size_t IB = (size_t)H * W * 3;

// The host worker's class for an image: (sum of its bytes + seed) % classes
// (csrc/comm/dp.cpp make_host_worker).
int32_t expect_idx(const uint8_t* img, uint32_t seed) {
  int64_t s = 0;
  for (size_t i = 0; i < IB; ++i) s += img[i];
  return (int32_t)((s + seed) % 1000);
}
}  // namespace

int main(int argc, char** argv) {
  const int queries = argc > 1 ? std::atoi(argv[1]) : 400;
  const int threads = argc > 2 ? std::atoi(argv[2]) : 24;
  const uint32_t seed = 11;
  std::vector<uint8_t> images(512 * IB);
  std::mt19937 rng(5);
  for (auto& b : images) b = (uint8_t)(rng() & 255);

  dp::FleetOptions o;
  o.max_per_rank = 16;
  o.image_bytes = IB;
  o.min_shard = 1000;  // direct path only
  o.batch_window_us = 300;
  o.timeout_ms = 5000;
  auto wf = [&](const std::string&, int d, dp::Worker* rep) {
    return dp::make_host_worker(d, H, W, 1000, 2, rep ? 0u : seed, 300);
  };
  auto cf = [](const std::vector<int>& devs) { return comm::host_world((int)devs.size(), 5000); };
  dp::Fleet fleet({0, 1, 2}, wf, cf, o);
  fleet.set_jobs({"resnet18"});
  fleet.load("resnet18");

  struct Q {
    int64_t first;
    int n;
    bool bad;
    std::vector<int32_t> idx;
    std::vector<float> prob;
    std::string err;
  };
  std::vector<Q> qs(queries);
  for (int i = 0; i < queries; ++i) {
    qs[i].n = 1 + (int)(rng() % 5);
    qs[i].first = (int64_t)(rng() % (512 - qs[i].n));
    qs[i].bad = i % 6 == 3;
    qs[i].idx.assign(qs[i].n, -1);
    qs[i].prob.assign(qs[i].n, 0.f);
  }
  std::atomic<int> next{0};
  std::vector<std::thread> ts;
  for (int t = 0; t < threads; ++t)
    ts.emplace_back([&] {
      for (int i = next++; i < queries; i = next++) {
        Q& q = qs[i];
        if (i == queries / 2) {  // an abrupt GPU loss under load
          dp::Worker* w = fleet.worker("resnet18", 1);
          if (w) dp::host_worker_set_healthy(*w, false);
        }
        auto stage = [&](const dp::StageCtx& c, int64_t off, int64_t n) -> const uint8_t* {
          if (q.bad) throw std::runtime_error("bad image size");
          std::memcpy(c.batch, images.data() + (size_t)(q.first + off) * IB, (size_t)n * IB);
          return (const uint8_t*)c.batch;
        };
        try {
          fleet.classify("resnet18", q.n, stage, q.idx.data(), q.prob.data());
        } catch (const std::exception& e) {
          q.err = e.what();
        }
      }
    });
  for (auto& t : ts) t.join();

  int bad_ok = 0, good_ok = 0, wrong = 0;
  for (int i = 0; i < queries; ++i) {
    const Q& q = qs[i];
    if (q.bad) {
      if (q.err.find("bad image size") != std::string::npos) ++bad_ok;
      else ++wrong, std::fprintf(stderr, "query %d: bad query got '%s'\n", i, q.err.c_str());
      continue;
    }
    bool ok = q.err.empty();
    for (int k = 0; ok && k < q.n; ++k) ok = q.idx[k] == expect_idx(images.data() + (size_t)(q.first + k) * IB, seed);
    if (ok) ++good_ok;
    else ++wrong, std::fprintf(stderr, "query %d: err '%s' or wrong answers\n", i, q.err.c_str());
  }
  int64_t fw = 0;
  for (const auto& kv : fleet.forwards("resnet18")) fw += kv.second;
  std::printf("fleet_stress: %d good ok, %d bad ok, %d wrong, %lld forwards, %d rebalances\n", good_ok, bad_ok,
              wrong, (long long)fw, fleet.rebalances());
  return wrong == 0 ? 0 : 1;
}
