// Fully-connected layers at small batch (B <= 16): weight-streaming GEMV on
// MFMA. AlexNet's classifier (9216x4096, 4096x4096, 4096x1000 = 117 MB of
// bf16 weights) is pure weight bandwidth at query batch sizes: every weight
// is used B times. As an implicit-GEMM conv (conv_igemm.hip) the 128-row
// tiles leave 3/4 of the M dimension empty and ~16 workgroups stream the
// whole matrix; here the weight rows are the MFMA A operand (16 rows x 32 k
// per 16-B lane load, the [N][K] row-major layout as stored) and the batch is
// the B operand (images in the 16 columns, zero columns beyond B), so:
//
//  * one wave owns 16 output rows for a K range and streams their weights
//    with UNROLL k-steps of 16-B loads in flight (1 KB per wave instruction);
//    the activations ([B, K], a few hundred KB) stay L2-resident;
//  * a tile's 8 waves split K (128 KB of weight loads in flight per tile)
//    and meet in LDS; one pass adds the bias, applies ReLU and writes the
//    bf16 / fp32 output in a fixed summation order (no global hand-off, no
//    workspace).
//
// Reference equivalent: `classifier.{1,4,6}` (+ReLU) of tch::vision::alexnet
// run per single-image query by `forward_t` (src/services.rs:519-524, 493).
#include "common.h"
#include "kernels.h"

#include <algorithm>

namespace dmlc {

namespace {

constexpr int kUnroll = 16;  // k-steps (32 k each) with their weight loads in flight per wave (16 KB)
constexpr int kWaves = 8;    // waves per workgroup = K split of one 16-row tile

struct FcSmallArgs {
  const bf16* x;      // [B, K] (row stride ldx)
  const bf16* w;      // [Npad, ldw]
  const float* bias;  // [Npad]
  void* y;            // [B, ldo] bf16 or fp32
  int B, K, N, ldx, ldw, ldo;
  int relu, out_f32;
};

// One workgroup per 16 output rows; its 8 waves split K and meet in LDS
// (fixed summation order: deterministic, no global hand-off).
__global__ __launch_bounds__(64 * kWaves) void fc_small_kernel(FcSmallArgs a) {
  __shared__ float part[kWaves][256];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int n0 = blockIdx.x * 16;
  const int row = lane & 15, kq = lane >> 4;  // A: weight row n0+row, k chunk kq; B: image col = row
  const int col = lane & 15;
  const int ksteps = a.K / 32, per = (ksteps + kWaves - 1) / kWaves;
  const int ks0 = wave * per, ks1 = min(ks0 + per, ksteps);
  const bf16* wrow = a.w + (long)(n0 + row) * a.ldw + kq * 8;
  const bool live = col < a.B;
  const bf16* xrow = a.x + (long)(live ? col : 0) * a.ldx + kq * 8;
  floatx4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int ks = ks0; ks < ks1; ks += kUnroll) {
    bf16x8 wv[kUnroll], xv[kUnroll];
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      const int k = (ks + u) * 32;
      const bool in = ks + u < ks1;
      wv[u] = in ? *(const bf16x8*)(wrow + k) : bf16x8{};
      xv[u] = (in && live) ? *(const bf16x8*)(xrow + k) : bf16x8{};
    }
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wv[u], xv[u], acc, 0, 0, 0);
  }
  // lane holds D[rows 4kq..4kq+3][col]: element (r, c) at 16r + c
#pragma unroll
  for (int r = 0; r < 4; ++r) part[wave][(4 * kq + r) * 16 + col] = acc[r];
  __syncthreads();
  if (tid >= 256) return;
  const int r = tid >> 4, c = tid & 15, n = n0 + r;
  if (c >= a.B || n >= a.N) return;
  float t = 0.f;
#pragma unroll
  for (int w = 0; w < kWaves; ++w) t += part[w][tid];
  t += a.bias[n];
  if (a.relu) t = fmaxf(t, 0.f);
  if (a.out_f32) ((float*)a.y)[(long)c * a.ldo + n] = t;
  else ((bf16*)a.y)[(long)c * a.ldo + n] = f2bf(t);
}

}  // namespace

bool fc_small_supported(int B, int K, int ldx, int ldw) {
  return B >= 1 && B <= 16 && K % 32 == 0 && ldx % 8 == 0 && ldw % 8 == 0 && ldw >= K && ldx >= K;
}

void fc_small(const void* x, int ldx, const void* w, int ldw, const float* bias, void* y, int ldo, bool out_f32,
              int B, int K, int N, int Npad, bool relu, hipStream_t s) {
  if (B <= 0) return;
  if (!fc_small_supported(B, K, ldx, ldw) || Npad < ((N + 15) / 16) * 16)
    throw std::invalid_argument("fc_small: unsupported shape");
  if (!x || !w || !bias || !y || (((uintptr_t)x | (uintptr_t)w) & 15))
    throw std::invalid_argument("fc_small: null / misaligned operand");
  FcSmallArgs a;
  a.x = (const bf16*)x;
  a.w = (const bf16*)w;
  a.bias = bias;
  a.y = y;
  a.B = B;
  a.K = K;
  a.N = N;
  a.ldx = ldx;
  a.ldw = ldw;
  a.ldo = ldo;
  a.relu = relu;
  a.out_f32 = out_f32;
  hipLaunchKernelGGL(fc_small_kernel, dim3((N + 15) / 16), dim3(64 * kWaves), 0, s, a);
  DMLC_HIP_CHECK(hipGetLastError());
}

}  // namespace dmlc
