// Fully connected layers at throughput batches (AlexNet's classifier,
// M = B <= 256 images): y[M][N] = x[M][K] . W[N][K]^T (+ bias, ReLU).
//
// Reference equivalent: tch::vision::alexnet's classifier Linear layers, run
// per query by `forward_t` (src/services.rs:493). On the implicit GEMM
// (conv_igemm.hip, 128x128 tiles, 8 K slices) the three FCs took ~40 + ~20 +
// ~8 us plus three split-K reductions at B = 256, bound by the per-CU
// LDS-DMA ingest of the re-staged tiles (~30 GB/s per CU; profiles/
// r5_fc_splitk.txt). Here:
//
//  * a workgroup owns all M (<= 256) rows x 128 output columns x one K slice,
//    so every weight byte is read from HBM exactly once and the activations
//    (<= 4.7 MB, L2 / MALL resident) once per 128 columns;
//  * tiles reach a 3-slot LDS ring by LDS-DMA, two K blocks (64) in flight
//    while one is computed (with one in flight, register-staged, the stages
//    were load-latency bound at ~25 GB/s per CU), 16-B chunks XOR-swizzled
//    by row through the source addresses (conflict-free fragment reads);
//  * 8 waves = 2 row halves x 4 column quarters: 8 x 2 fragments of
//    v_mfma_f32_16x16x32_bf16 per K step, fp32 partials per K slice into the
//    split-K workspace, reduced (+ bias, ReLU, bf16 / fp32 out) by
//    conv_igemm.hip's splitk_reduce.
#include "common.h"
#include "kernels.h"

#include <algorithm>
#include <stdexcept>

namespace dmlc {

namespace {

constexpr int kBM = 256;   // rows (images) per workgroup: all of them
constexpr int kBN = 128;   // output columns per workgroup
constexpr int kKB = 64;    // K block per stage
constexpr int kAB = kBM * kKB * 2;  // 32 KB A stage
constexpr int kBB = kBN * kKB * 2;  // 16 KB B stage
constexpr int kStage = kAB + kBB;
static_assert(kAB / 1024 == 32 && kBB / 1024 == 16, "6 DMA instructions per wave per stage");

template <int N>
__device__ __forceinline__ void vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}

// 16-B chunk c (0..7) of a 128-B LDS row r
__device__ __forceinline__ int fc_off(int r, int c) { return r * 128 + ((c ^ (r & 7)) << 4); }

__global__ __launch_bounds__(512, 1) void fc_gemm_kernel(const bf16* __restrict__ x, const bf16* __restrict__ w,
                                                         float* __restrict__ ws, int M, int K, int Npad, int kslice,
                                                         int nslices, const bf16* __restrict__ zero) {
  extern __shared__ __attribute__((aligned(16))) uint4 smem[];
  char* lds = (char*)smem;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave & 1, wn = wave >> 1;
  const int fr = lane & 15, fq = lane >> 4;
  // workgroup -> (column block nb, K slice ks). Workgroups are dealt to the 8
  // XCDs round-robin: with a multiple of 8 slices, XCD x takes slices x, x+8,
  // ... for every column block, so each XCD's L2 holds only its own slices'
  // activations (read once from HBM chip-wide) instead of all of them
  const int cols = Npad / kBN, L = blockIdx.x;
  int nb, ks;
  if (nslices % 8 == 0) {
    const int i = L >> 3;
    nb = i % cols;
    ks = (L & 7) + 8 * (i / cols);
  } else {
    nb = L % cols;
    ks = L / cols;
  }
  const int n0 = nb * kBN;
  const int k0 = ks * kslice;
  const int nstages = kslice / kKB;

  // Staging: a 3-slot LDS ring filled by LDS-DMA (global_load_lds_dwordx4,
  // 1 KB per wave instruction: lane l's 16 B land at slot offset 1024 i +
  // 16 l), two K blocks in flight while one is computed. A stage is 32 A
  // instructions (256 rows x 128 B) + 16 B instructions (128 rows), 6 per
  // wave; LDS position p = 64 i + l holds row p >> 3, physical chunk p & 7 =
  // logical chunk (p & 7) ^ (row & 7), so the source address carries the
  // swizzle. Rows >= M read the zero page.
  floatx4 acc[8][2];
#pragma unroll
  for (int mf = 0; mf < 8; ++mf)
#pragma unroll
    for (int nf = 0; nf < 2; ++nf) acc[mf][nf] = floatx4{0.f, 0.f, 0.f, 0.f};
  const bf16* asrc[4];
  const bf16* bsrc[2];
  int aoff[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int p = (4 * wave + j) * 64 + lane, r = p >> 3, lc = (p & 7) ^ (r & 7);
    asrc[j] = r < M ? x + (long)r * K + k0 + 8 * lc : zero;
    aoff[j] = r < M ? 1 : 0;  // (the zero page does not advance with K)
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int p = (2 * wave + j) * 64 + lane, r = p >> 3, lc = (p & 7) ^ (r & 7);
    bsrc[j] = w + (long)(n0 + r) * K + k0 + 8 * lc;
  }
  auto dma_stage = [&](int st, int slot) __attribute__((always_inline)) {
    char* base = lds + slot * kStage;
    const int ko = st * kKB;
#pragma unroll
    for (int j = 0; j < 4; ++j) dma16(asrc[j] + ko * aoff[j], base + (4 * wave + j) * 1024);
#pragma unroll
    for (int j = 0; j < 2; ++j) dma16(bsrc[j] + ko, base + kAB + (2 * wave + j) * 1024);
  };
  dma_stage(0, 0);
  if (nstages > 1) dma_stage(1, 1);
  for (int s = 0; s < nstages; ++s) {
    // this wave's DMA of stage s has landed (stage s+1's may stay in flight),
    // and after the barrier everyone's has, and every wave is done with stage
    // s-1, whose slot stage s+2 reuses
    if (s + 1 < nstages) vm_wait<6>();
    else vm_wait<0>();
    __builtin_amdgcn_s_barrier();
    if (s + 2 < nstages) dma_stage(s + 2, (s + 2) % 3);
    const char* base = lds + (s % 3) * kStage;
#pragma unroll
    for (int kk = 0; kk < kKB / 32; ++kk) {
      bf16x8 af[8], bf[2];
#pragma unroll
      for (int mf = 0; mf < 8; ++mf) af[mf] = *(const bf16x8*)(base + fc_off(128 * wm + 16 * mf + fr, 4 * kk + fq));
#pragma unroll
      for (int nf = 0; nf < 2; ++nf) bf[nf] = *(const bf16x8*)(base + kAB + fc_off(32 * wn + 16 * nf + fr, 4 * kk + fq));
#pragma unroll
      for (int mf = 0; mf < 8; ++mf)
#pragma unroll
        for (int nf = 0; nf < 2; ++nf)
          acc[mf][nf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[mf], bf[nf], acc[mf][nf], 0, 0, 0);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // (this wave's reads of the slot are done)
  }
  // D lane (fr, fq): row 4 fq + r of the fragment, column fr
  float* wsp = ws + (long)ks * M * Npad;
#pragma unroll
  for (int mf = 0; mf < 8; ++mf)
#pragma unroll
    for (int nf = 0; nf < 2; ++nf) {
      const int n = n0 + 32 * wn + 16 * nf + fr;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = 128 * wm + 16 * mf + 4 * fq + r;
        if (m < M) wsp[(long)m * Npad + n] = acc[mf][nf][r];
      }
    }
}

}  // namespace

int fc_gemm_splits(const ConvArgs& a, int num_cus) {
  if (a.Kpad <= 0 || a.Npad % kBN) return 0;
  const int kb = a.Kpad / kKB;
  const int cols = a.Npad / kBN;
  // about one workgroup per CU, each at least 4 K blocks
  int s = std::max(1, std::min(kb / 4, (num_cus + cols - 1) / cols));
  while (s > 1 && kb % s) --s;  // whole K blocks per slice
  return s;
}

bool fc_gemm_supported(const ConvArgs& a) {
  return a.H == 1 && a.W == 1 && a.KH == 1 && a.KW == 1 && a.Ho == 1 && a.Wo == 1 && !a.stem && !a.in_fp8 &&
         !a.out_fp8 && !a.res && a.B >= 1 && a.B <= kBM && a.Cin == a.Kpad && a.Kpad % kKB == 0 &&
         a.Npad % kBN == 0 && a.N <= a.Npad;
}

void fc_gemm(const ConvArgs& a, int splits, hipStream_t s) {
  if (!fc_gemm_supported(a)) throw std::invalid_argument("fc_gemm: unsupported layer");
  if (splits < 1 || (a.Kpad / kKB) % splits) throw std::invalid_argument("fc_gemm: K blocks must split evenly");
  if (!a.x || !a.w || !a.y || !a.zero || !a.ws || (((uintptr_t)a.x | (uintptr_t)a.w | (uintptr_t)a.zero) & 15))
    throw std::invalid_argument("fc_gemm: null / misaligned operand (the workspace is required)");
  const int M = a.B;
  const int kslice = a.Kpad / splits;
  hipLaunchKernelGGL(fc_gemm_kernel, dim3(a.Npad / kBN * splits), dim3(512), (size_t)3 * kStage, s,
                     (const bf16*)a.x, (const bf16*)a.w, a.ws, M, a.Kpad, a.Npad, kslice, splits,
                     (const bf16*)a.zero);
  DMLC_HIP_CHECK(hipGetLastError());
  ConvArgs b = a;
  b.split_k = splits;
  splitk_reduce(b, M, splits, s);
}

}  // namespace dmlc
