// Stride-2 3x3 conv 56x56x64 -> 28x28x128 (BN folded, ReLU) together with the
// block's 1x1/s2 downsample (BN folded, no ReLU), row-streamed: ResNet18
// layer2.0.conv1 + layer2.0.downsample.
//
// Reference equivalent: layer2.0.{conv1,bn1,relu} and layer2.0.downsample of
// tch::vision::resnet18, run per query by `forward_t` (src/services.rs:493).
// As a stream conv (conv3x3_stream.hip: 7-output-row strips with their 15
// input rows resident in LDS, 1024 workgroups at one per CU) the input
// staging of every round is exposed: 4 rounds of HBM-bound prologue around
// ~2 us of MFMAs each, 72 us for 33 GFLOP (profiles/r2_final_resnet18_kernels.txt).
// Here one workgroup walks one image top to bottom (one round at B = 256),
// 4 output rows per step, the 8 input rows of the next step arriving by
// LDS-DMA while the current step computes:
//
//  * weight-stationary: 4 waves (one per SIMD), wave w owns output channels
//    32w .. 32w + 31 and keeps all 20 of their K-step fragments (18 for the
//    3x3 taps, 2 for the downsample) in registers, so the only global traffic
//    in the loop is the row DMA (whose vmcnt, being asm, the compiler cannot
//    see or wait on) and the output stores;
//  * staged input row: two K-half planes of 57 pixel slots x 64 B (slot 0 =
//    column -1, zero; 1..28 = odd columns; 29..56 = even columns), so output
//    pixels c, c+1 read adjacent slots at every tap (kw 0: slot c, kw 1: 29 + c
//    as an immediate, kw 2: c + 1); rows padded to 7424 B (a bank-row
//    multiple) in a ring of 17 + 2 guard slots (copies of slots 0, 1) so the
//    3 kernel rows of a fragment are immediate offsets of one address;
//  * 16-B chunk c of a K-half of stored pixel (y, x) sits at physical chunk
//    c ^ ((K >> 1) & 3), K = ((y + 1) >> 1) * 28 + ((x + 1) >> 1): along a
//    fragment K is the output pixel index plus a tap constant, also where a
//    fragment wraps an output row, and every ds_read_b128 is conflict free
//    (tests/test_layouts_cpu.py).
#include "common.h"
#include "kernels.h"

namespace dmlc {

namespace {

template <int N>
__device__ __forceinline__ void vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}

struct S2Args {
  const bf16* x;      // [B, 56, 56, 64]
  const bf16* wf;     // 3x3 weights, fragment order [4][18][2][64][8] (stream_frag_index, K = 576)
  const bf16* wdf;    // 1x1 weights, fragment order [4][2][2][64][8] (K = 64)
  const float* bias;  // [128]
  const float* bd;    // [128]
  bf16* y;            // [B, 28, 28, 128]
  bf16* yd;           // [B, 28, 28, 128]
  const bf16* zero;
  int relu;
  int stagger;  // start_stagger (common.h)
};

constexpr int kHI = 56, kWI = 56, kCI = 64, kH = 28, kW = 28, kCO = 128;
constexpr int kR = 4;                 // output rows per step
constexpr int kSteps = kH / kR;       // 7
constexpr int kE0 = 29;               // first even-column slot
constexpr int kHalf = 3712;           // bytes per K-half plane (58 slots x 64 B)
constexpr int kRB = 2 * kHalf;        // 7424 B per staged row
constexpr int kRing = 17;             // rows 2 r0 - 1 .. 2 r0 + 7 in use + 8 in flight
constexpr int kSlotsAlloc = kRing + 2;
constexpr int kRun = 4 * 2 * kW;      // 224 DMA chunks per K-half plane (slots 1..56)
constexpr int kMF = kR * kW / 16;     // 7 pixel fragments per step
constexpr int kKT = 18, kCT = 2;      // 3x3 / downsample K steps
constexpr int kOffKw1 = kE0 * 64;     // kw = 1 reads slot 29 + c

__device__ __forceinline__ int swz_of(int y, int x) { return ((((y + 1) >> 1) * kW + ((x + 1) >> 1)) >> 1) & 3; }

// DS: also the block's 1x1/s2 downsample (K = 64 more, the yd output). Off
// (ds_into_conv2): the downsample is a K-extension of the block's conv2
// (conv3x3_rows28_kernel DSX), so yd is neither written here nor read back
// there: 51 of the 205 MB this kernel moved at B = 256, and 2 of its 20 K steps.
template <bool DS>
__global__ __launch_bounds__(256, 1) void conv3x3_s2rows_kernel(S2Args a) {
  constexpr int kKS = kKT + (DS ? kCT : 0);
  extern __shared__ __attribute__((aligned(16))) uint4 smem[];
  char* ring = (char*)smem;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  start_stagger(a.stagger);
  const int fr = lane & 15, g = lane >> 4;
  const int b = blockIdx.x;
  const bf16* img = a.x + (long)b * kHI * kWI * kCI;

  // Every slot's pad column (slot 0 of each K-half plane), its spare slot
  // and the zero row y = -1 are zeroed once here and never DMA'd over (a
  // shared zero page read by every workgroup's pad lanes is one hot L2
  // channel per XCD).
  for (int o = tid * 16; o < kSlotsAlloc * kRB; o += 256 * 16) *(uint4*)(ring + o) = make_uint4(0, 0, 0, 0);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  // input row yy >= 0 -> ring slot (yy + 1) % 17, and guard slot 17 / 18 too
  // for slots 0 / 1: per K-half plane the 224 chunks of slots 1..56 are one
  // contiguous run; wave w DMAs chunks 64 w .. 64 w + 63 of both runs
  auto load_row = [&](int yy) __attribute__((always_inline)) {
    const int slot = (yy + 1) % kRing;
    const int k = wave * 64 + lane;
    const int pos = 1 + (k >> 2), c = k & 3;
    const int x = pos < kE0 ? 2 * pos - 1 : 2 * (pos - kE0);
    const int sw = swz_of(yy, x);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const bf16* src = img + ((long)yy * kWI + x) * kCI + 8 * (4 * h + (c ^ sw));
      char* dst = ring + h * kHalf + 64 + wave * 1024;
      if (k < kRun) {
        dma16(src, dst + slot * kRB);
        if (slot < 2) dma16(src, dst + (slot + kRing) * kRB);
      }
    }
  };
  // this lane's 8 output channels ch0 + 8g .. +7 (weight rows permuted,
  // perm32); loaded before the row DMAs so the prologue wait below can leave
  // exactly the weight loads in flight
  const int ch0 = wave * 32;
  float bs[8], bsd[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    bs[e] = a.bias[ch0 + 8 * g + e];
    bsd[e] = DS ? a.bd[ch0 + 8 * g + e] : 0.f;
  }
  for (int yy = 0; yy <= 7; ++yy) load_row(yy);

  // ---- per-lane constants. Fragment f covers tile pixels p = 16 f + fr (row
  // p / 28 of the step, column c = p % 28). col[f][v]: the in-row byte offset
  // of K-half 0 for variant v = (kw == 2) + 2 (kh == 2)
  int prow2[kMF], col[kMF][4];
#pragma unroll
  for (int f = 0; f < kMF; ++f) {
    const int p = 16 * f + fr;
    prow2[f] = 2 * (p / kW);
    const int c = p % kW;
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int kw2 = v & 1, kh2 = v >> 1;
      const int s = ((p + kw2 + kW * kh2) >> 1) & 3;  // K of r0 = 0 (r0 is a multiple of 4)
      col[f][v] = (c + kw2) * 64 + ((g ^ s) << 4);
    }
  }
  bf16x8 w[kKS][2];
#pragma unroll
  for (int t = 0; t < kKS; ++t)
#pragma unroll
    for (int nf = 0; nf < 2; ++nf) {
      const bf16* src = t < kKT ? a.wf + ((((long)wave * kKT + t) * 2 + nf) * 64 + lane) * 8
                                : a.wdf + ((((long)wave * kCT + (t - kKT)) * 2 + nf) * 64 + lane) * 8;
      w[t][nf] = *(const bf16x8*)src;
    }
  // the prologue rows (DMA'd before the weights) have landed; the weights may
  // still be in flight: the first step's MFMAs wait for each K step's own
  // fragments (the compiler's counted waits), so the 160 KB weight load from
  // L2 overlaps the first step instead of preceding it
  vm_wait<2 * kKS>();
  __builtin_amdgcn_s_barrier();

  // step 0 is peeled (a separate copy of the body): at a loop header the
  // compiler waits for every outstanding load (vmcnt(0)), which would put the
  // whole weight load back in front of the first MFMA
  auto step_body = [&](const int step) __attribute__((always_inline)) {
    const int r0 = step * kR;  // first output row; input rows 2 r0 - 1 .. 2 r0 + 7
    if (step + 1 < kSteps)
      for (int yy = 2 * r0 + 8; yy <= 2 * r0 + 15; ++yy) load_row(yy);
    // ring slot of kernel row 0 of every fragment (+ kh rows: immediate, guard slots)
    const int sb = (2 * r0) % kRing;
    int rowoff[kMF];
#pragma unroll
    for (int f = 0; f < kMF; ++f) {
      int sl = sb + prow2[f];
      sl = sl >= kRing ? sl - kRing : sl;
      rowoff[f] = sl * kRB;
    }
    floatx4 acc[kMF][2], accd[kMF][2];
#pragma unroll
    for (int f = 0; f < kMF; ++f)
#pragma unroll
      for (int nf = 0; nf < 2; ++nf) {  // the biases are the accumulators' starting values
        acc[f][nf] = floatx4{bs[4 * nf], bs[4 * nf + 1], bs[4 * nf + 2], bs[4 * nf + 3]};
        if constexpr (DS) accd[f][nf] = floatx4{bsd[4 * nf], bsd[4 * nf + 1], bsd[4 * nf + 2], bsd[4 * nf + 3]};
      }
    // K step t: tap = t >> 1 (downsample steps: tap 4 = (1, 1)), K-half h = t & 1
    auto xread = [&](int t, int f) __attribute__((always_inline)) {
      const int tap = t < kKT ? t >> 1 : 4, h = t & 1;
      const int kh = tap / 3, kw = tap % 3;
      const int v = (kw == 2) + 2 * (kh == 2);
      const int imm = kh * kRB + (kw == 1 ? kOffKw1 : 0) + h * kHalf;
      return *(const bf16x8*)(ring + (rowoff[f] + col[f][v]) + imm);
    };
    bf16x8 xc[kMF];
#pragma unroll
    for (int f = 0; f < kMF; ++f) xc[f] = xread(0, f);
#pragma unroll
    for (int t = 0; t < kKS; ++t) {
#pragma unroll
      for (int f = 0; f < kMF; ++f) {
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int nf = 0; nf < 2; ++nf) {
          if (t < kKT)
            acc[f][nf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[t][nf], xc[f], acc[f][nf], 0, 0, 0);
          else
            accd[f][nf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[t][nf], xc[f], accd[f][nf], 0, 0, 0);
        }
        if (t + 1 < kKS) xc[f] = xread(t + 1, f);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    // ---- epilogue: lane holds channels ch0 + 8g .. +7 of tile pixel 16 f + fr
#pragma unroll
    for (int f = 0; f < kMF; ++f) {
      const long o = (((long)b * kH + r0) * kW + 16 * f + fr) * kCO + ch0 + 8 * g;
      float v[8], vd[8];
#pragma unroll
      for (int nf = 0; nf < 2; ++nf)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          v[4 * nf + i] = acc[f][nf][i];
          vd[4 * nf + i] = DS ? accd[f][nf][i] : 0.f;
        }
      *(uint4*)(a.y + o) = pack8_relu(v, a.relu);
      if constexpr (DS) *(uint4*)(a.yd + o) = pack8(vd);
    }
    // the next step's rows have landed (the (2) kMF stores just issued may
    // still be in flight: vmcnt retires in order) and every wave is done
    // reading the rows they replace
    vm_wait<(DS ? 2 : 1) * kMF>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  };
  step_body(0);
  for (int step = 1; step < kSteps; ++step) step_body(step);
}

}  // namespace

bool conv3x3_s2rows_supported(int Hin, int Win, int Cin, int Cout) {
  return Hin == kHI && Win == kWI && Cin == kCI && Cout == kCO;
}

void conv3x3_s2rows(const void* x, const void* wf, const float* bias, const void* wdf, const float* bd, void* y,
                    void* yd, const void* zero, int B, bool relu, hipStream_t s) {
  if (B <= 0) return;
  if ((wdf == nullptr) != (bd == nullptr) || (wdf == nullptr) != (yd == nullptr))
    throw std::invalid_argument("conv3x3_s2rows: the downsample needs wdf, bd and yd together");
  if (!x || !wf || !bias || !y || !zero ||
      (((uintptr_t)x | (uintptr_t)wf | (uintptr_t)wdf | (uintptr_t)y | (uintptr_t)yd | (uintptr_t)zero) & 15))
    throw std::invalid_argument("conv3x3_s2rows: null / misaligned operand");
  S2Args a;
  a.stagger = kernel_stagger(kStagS2rows);
  a.x = (const bf16*)x;
  a.wf = (const bf16*)wf;
  a.wdf = (const bf16*)wdf;
  a.bias = bias;
  a.bd = bd;
  a.y = (bf16*)y;
  a.yd = (bf16*)yd;
  a.zero = (const bf16*)zero;
  a.relu = relu;
  if (wdf)
    hipLaunchKernelGGL(conv3x3_s2rows_kernel<true>, dim3(B), dim3(256), (size_t)kSlotsAlloc * kRB, s, a);
  else
    hipLaunchKernelGGL(conv3x3_s2rows_kernel<false>, dim3(B), dim3(256), (size_t)kSlotsAlloc * kRB, s, a);
  DMLC_HIP_CHECK(hipGetLastError());
}

}  // namespace dmlc
