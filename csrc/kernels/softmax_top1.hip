// Fused softmax + top-1 over the classifier logits.
//
// Reference: `forward_t(..).softmax(-1)` then `imagenet::top(output, 1)` per
// query (src/services.rs:493-494). One wave per row: a single pass computes
// the running max/argmax, a second the exp-sum; the top-1 probability is
// 1 / sum(exp(x - max)). Ties resolve to the lowest class index.
#include "common.h"
#include "kernels.h"

#include <algorithm>

namespace dmlc {

namespace {

__global__ __launch_bounds__(256) void softmax_top1_kernel(const float* __restrict__ logits, int B,
                                                           int N, int ld, int32_t* __restrict__ idx,
                                                           float* __restrict__ prob) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= B) return;
  const float* p = logits + (long)row * ld;
  float best = -INFINITY;
  int bi = 0x7fffffff;
  for (int i = lane; i < N; i += 64) {
    const float v = p[i];
    if (v > best) {  // i increases per lane, so the first max wins within a lane
      best = v;
      bi = i;
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(best, o, 64);
    const int oi = __shfl_xor(bi, o, 64);
    if (ov > best || (ov == best && oi < bi)) {
      best = ov;
      bi = oi;
    }
  }
  float s = 0.f;
  for (int i = lane; i < N; i += 64) s += __expf(p[i] - best);
  s = wave_sum(s);
  if (lane == 0) {
    idx[row] = bi;
    prob[row] = 1.f / s;
  }
}

}  // namespace

void softmax_top1(const float* logits, int B, int N, int ld, int32_t* idx, float* prob,
                  hipStream_t s) {
  if (B <= 0) return;
  if (N <= 0 || ld < N) throw std::invalid_argument("softmax_top1: bad N/ld");
  hipLaunchKernelGGL(softmax_top1_kernel, dim3((B + 3) / 4), dim3(256), 0, s, logits, B, N, ld, idx,
                     prob);
  DMLC_HIP_CHECK(hipGetLastError());
}

}  // namespace dmlc
