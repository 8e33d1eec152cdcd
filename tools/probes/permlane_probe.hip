// Semantics probe for gfx950 v_permlane16_swap / v_permlane32_swap (which
// lanes of each operand end up where). Prints, per lane, the four results
// for a = lane, b = 100 + lane.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(unsigned* out) {
  const unsigned l = threadIdx.x;
  auto r32 = __builtin_amdgcn_permlane32_swap(l, 100u + l, false, false);
  auto r16 = __builtin_amdgcn_permlane16_swap(l, 100u + l, false, false);
  out[l] = r32[0];
  out[64 + l] = r32[1];
  out[128 + l] = r16[0];
  out[192 + l] = r16[1];
}
int main() {
  unsigned* d;
  unsigned h[256];
  if (hipMalloc(&d, sizeof(h)) != hipSuccess) return 1;
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 2;
  const char* names[4] = {"p32[0]", "p32[1]", "p16[0]", "p16[1]"};
  for (int i = 0; i < 4; ++i) {
    printf("%s:", names[i]);
    for (int l = 0; l < 64; l += 8) printf(" l%d=%u", l, h[i * 64 + l]);
    printf("\n");
  }
  return 0;
}
