// One-wave probe of the block-scaled fp8 MFMA (v_mfma_scale_f32_16x16x128_f8f6f4)
// with raw per-lane operand registers, so a test can pin the lane -> (row, k)
// operand map with exact integer data before a kernel relies on it
// (cdna_hip_programming.md: "check the map with exact integer data").
#include "common.h"
#include "kernels.h"

namespace dmlc {

namespace {

typedef int v8i __attribute__((ext_vector_type(8)));

__global__ __launch_bounds__(64) void mfma_fp8_probe_kernel(const int* a, const int* b, float* d) {
  const int l = threadIdx.x;
  v8i A, B;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    A[i] = a[l * 8 + i];
    B[i] = b[l * 8 + i];
  }
  floatx4 c = {0.f, 0.f, 0.f, 0.f};
  // A/B format 0 = fp8 e4m3 (OCP); scales 127 = 2^0 (E8M0)
  c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(A, B, c, 0, 0, 0, 127, 0, 127);
#pragma unroll
  for (int r = 0; r < 4; ++r) d[l * 4 + r] = c[r];
}

}  // namespace

void mfma_fp8_probe(const void* a, const void* b, float* d, hipStream_t s) {
  if (!a || !b || !d) throw std::invalid_argument("mfma_fp8_probe: null operand");
  hipLaunchKernelGGL(mfma_fp8_probe_kernel, dim3(1), dim3(64), 0, s, (const int*)a, (const int*)b, d);
  DMLC_HIP_CHECK(hipGetLastError());
}

}  // namespace dmlc
