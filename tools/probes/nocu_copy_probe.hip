// Does hipMemcpyDeviceToDeviceNoCU (copy engine, no blit kernel) accept a
// pinned host destination, and is the result exact? Compare with the default
// D2H path under rocprofv3 --kernel-trace (a blit kernel shows up as
// __amd_rocclr_copyBuffer*).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
int main(int argc, char** argv) {
  const bool nocu = argc > 1 && argv[1][0] == '1';
  const size_t n = 4096;
  unsigned char *d, *h;
  hipStream_t s;
  if (hipMalloc(&d, n) != hipSuccess || hipHostMalloc(&h, n, hipHostMallocDefault) != hipSuccess ||
      hipStreamCreate(&s) != hipSuccess)
    return 1;
  unsigned char ref[4096];
  for (size_t i = 0; i < n; ++i) ref[i] = (unsigned char)(i * 7 + 3);
  if (hipMemcpy(d, ref, n, hipMemcpyHostToDevice) != hipSuccess) return 2;
  int bad = 0;
  for (int it = 0; it < 50; ++it) {
    memset(h, 0, n);
    hipError_t e = hipMemcpyAsync(h, d, n, nocu ? hipMemcpyDeviceToDeviceNoCU : hipMemcpyDeviceToHost, s);
    if (e != hipSuccess) {
      printf("memcpy error: %s\n", hipGetErrorString(e));
      return 3;
    }
    if (hipStreamSynchronize(s) != hipSuccess) return 4;
    bad += memcmp(h, ref, n) != 0;
  }
  printf("%s: %d/50 mismatched\n", nocu ? "NoCU" : "D2H", bad);
  return bad ? 5 : 0;
}
