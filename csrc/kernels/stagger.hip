// Per-kernel-family workgroup start stagger (kernels.h kernel_stagger,
// common.h start_stagger): the defaults, the A/B hook and the single-lane
// setting. Measured (profiles/r6_stagger.txt): one forward at a time
// (tools/engine_ab.py, ResNet18 b256) runs 926 -> 911 us with the stream
// convs staggered by 4 (bench --lanes 1: +1.0%), and no other family gains
// (ResNet50's stream8 / conv1x1 lose); with two compute lanes the other
// lane's kernels already fill the phases the stagger would de-synchronise,
// and the sleeping workgroups hold their CUs from it (bench --lanes 2: -0.5%),
// so the defaults are 0 and kernel_stagger_for_lanes(1) turns it on.
#include <atomic>
#include <stdexcept>

#include "kernels.h"

namespace dmlc {

namespace {
constexpr int kDefaultStagger[kStagCount] = {0, 0, 0, 0, 0, 0, 0, 0};
std::atomic<int> g_stagger[kStagCount] = {-1, -1, -1, -1, -1, -1, -1, -1};
}  // namespace

int kernel_stagger(int k) {
  const int v = g_stagger[k].load(std::memory_order_relaxed);
  return v < 0 ? kDefaultStagger[k] : v;
}

void kernel_stagger_set(int k, int n) {
  if (k < 0 || k >= kStagCount || n > 32) throw std::invalid_argument("kernel_stagger_set: bad kernel / count");
  g_stagger[k] = n;
}

void kernel_stagger_for_lanes(int lanes) { kernel_stagger_set(kStagStream, lanes == 1 ? 4 : -1); }

}  // namespace dmlc
