// Stride-2 3x3 conv 56x56x128 -> 28x28x128 (BN folded, ReLU), row-streamed:
// ResNet50 layer2.0.conv2 (the first layer2 bottleneck's strided 3x3).
//
// Reference equivalent: layer2.0.{conv2,bn2,relu} of tch::vision::resnet50
// (src/services.rs:513-524 loads it; `forward_t` runs it per query). As a
// stream conv (conv3x3_stream.hip: 4-output-row strips, their 9 input rows
// resident in LDS) each of the 7 rounds of workgroups waits for its 129 KB
// of input before its MFMAs start: 102 us at B = 256
// (profiles/r4_r50_3x3_e4m3_out.txt). Here, as conv3x3_s2rows.hip does for
// ResNet18's 56x56x64 stride-2 conv, one workgroup walks one image top to
// bottom (one round at B = 256), the input rows of the next step arriving by
// LDS-DMA while the current step computes:
//
//  * weight-stationary: 4 waves (one per SIMD), wave w owns output channels
//    32w .. 32w + 31 and keeps all 36 of their K-step fragments (9 taps x 4
//    channel quarters) in registers (288 VGPRs: the 512-register budget of a
//    single wave per SIMD), so the loop's only global traffic is the row DMA
//    and the output stores;
//  * 2 output rows per step (56 pixels = 3.5 fragments: the 4th fragment's
//    last 8 lanes re-read pixel 55 and store nothing): 4 output rows would
//    need a 17-row ring of 14.6 KB rows;
//  * staged input row: four channel-quarter planes of 57 pixel slots x 64 B
//    (slot 0 = column -1, zero; 1..28 = odd columns; 29..56 = even columns),
//    rows of 14592 B (57 bank rows) in a ring of 9 + 2 guard slots (copies of
//    slots 0, 1) so a fragment's 3 kernel rows are immediate offsets of one
//    address: 160,512 B of LDS;
//  * 16-B chunk c of a quarter of stored pixel (y, x) sits at physical chunk
//    c ^ ((K >> 1) & 3), K = ((y + 1) >> 1) * 28 + ((x + 1) >> 1), the
//    conv3x3_s2rows swizzle: conflict-free fragment reads
//    (tests/test_layouts_cpu.py);
//  * the output is bf16, or e4m3 (relu(v) * out_inv_scale, saturated) for
//    ResNet50's e4m3 expand conv (EngineOptions::fp8_3x3_out).
#include "common.h"
#include "kernels.h"

namespace dmlc {

namespace {

template <int N>
__device__ __forceinline__ void vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}

struct S2R128Args {
  const bf16* x;    // [B, 56, 56, 128]
  const bf16* wf;   // weights, fragment order [4][36][2][64][8] (stream_frag_index, K = 1152)
  const float* bias;  // [128]
  void* y;          // [B, 28, 28, 128], bf16 or (out_inv_scale > 0) e4m3
  int relu;
  float out_inv_scale;
};

constexpr int kHI = 56, kWI = 56, kCI = 128, kH = 28, kW = 28, kCO = 128;
constexpr int kR = 2;                 // output rows per step
constexpr int kSteps = kH / kR;       // 14
constexpr int kE0 = 29;               // first even-column slot
constexpr int kPlane = 57 * 64;       // one channel quarter of a staged row: 3648 B
constexpr int kRB = 4 * kPlane;       // 14592 B per staged row (57 x 256)
constexpr int kRing = 9;              // rows 2 r0 - 1 .. 2 r0 + 3 in use + 4 in flight
constexpr int kSlotsAlloc = kRing + 2;
constexpr int kRun = 4 * 2 * kW;      // 224 DMA chunks per quarter plane (slots 1..56)
constexpr int kNPix = kR * kW;        // 56 output pixels per step
constexpr int kMF = (kNPix + 15) / 16;  // 4 pixel fragments per step
constexpr int kKS = 36;               // K steps: 9 taps x 4 quarters
constexpr int kOffKw1 = kE0 * 64;     // kw = 1 reads slot 29 + c
static_assert((size_t)kSlotsAlloc * kRB <= 160 * 1024, "LDS budget");

__device__ __forceinline__ int swz_of(int y, int x) { return ((((y + 1) >> 1) * kW + ((x + 1) >> 1)) >> 1) & 3; }

// 4 floats (within +-448) -> 4 e4m3 bytes
__device__ __forceinline__ uint32_t s2r_e4m3x4(float a, float b, float c, float d) {
  int v = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
  v = __builtin_amdgcn_cvt_pk_fp8_f32(c, d, v, true);
  return (uint32_t)v;
}

template <bool OUT8>
__global__ __launch_bounds__(256, 1) void conv3x3_s2rows128_kernel(S2R128Args a) {
  extern __shared__ __attribute__((aligned(16))) uint4 smem[];
  char* ring = (char*)smem;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, g = lane >> 4;
  const int b = blockIdx.x;
  const bf16* img = a.x + (long)b * kHI * kWI * kCI;

  // pad slots, the spare guard copies and the zero row y = -1 (slot 0): zero once
  for (int o = tid * 16; o < kSlotsAlloc * kRB; o += 256 * 16) *(uint4*)(ring + o) = make_uint4(0, 0, 0, 0);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  // input row yy >= 0 -> ring slot (yy + 1) % 9 (and guard slot 9 / 10 for
  // slots 0 / 1): per quarter plane the 224 chunks of slots 1..56 are one
  // contiguous run; wave w DMAs chunks 64 w .. 64 w + 63 of all four runs
  auto load_row = [&](int yy) __attribute__((always_inline)) {
    const int slot = (yy + 1) % kRing;
    const int k = wave * 64 + lane;
    const int pos = 1 + (k >> 2), c = k & 3;
    const int x = pos < kE0 ? 2 * pos - 1 : 2 * (pos - kE0);
    const int sw = swz_of(yy, x);
    if (k < kRun) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const bf16* src = img + ((long)yy * kWI + x) * kCI + 32 * q + 8 * (c ^ sw);
        char* dst = ring + q * kPlane + 64 + wave * 1024;
        dma16(src, dst + slot * kRB);
        if (slot < 2) dma16(src, dst + (slot + kRing) * kRB);
      }
    }
  };
  // this lane's 8 output channels ch0 + 8g .. +7 (weight rows permuted, perm32)
  const int ch0 = wave * 32;
  float bs[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) bs[e] = a.bias[ch0 + 8 * g + e];
  for (int yy = 0; yy <= 3; ++yy) load_row(yy);  // step 0 reads rows -1 .. 3

  // ---- per-lane constants. Fragment f covers step pixels p = 16 f + fr (the
  // 4th fragment's lanes past pixel 55 re-read pixel 55): row p / 28 of the
  // step, column c = p % 28. col[f][v]: the in-row byte offset of quarter 0
  // for variant v = (kw == 2) + 2 (kh == 2)
  int prow2[kMF], col[kMF][4];
#pragma unroll
  for (int f = 0; f < kMF; ++f) {
    const int p = min(16 * f + fr, kNPix - 1);
    prow2[f] = 2 * (p / kW);
    const int c = p % kW;
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int kw2 = v & 1, kh2 = v >> 1;
      const int s = ((p + kw2 + kW * kh2) >> 1) & 3;  // K of r0 = 0 (28 r0 = 56 step: a multiple of 8)
      col[f][v] = (c + kw2) * 64 + ((g ^ s) << 4);
    }
  }
  bf16x8 w[kKS][2];
#pragma unroll
  for (int t = 0; t < kKS; ++t)
#pragma unroll
    for (int nf = 0; nf < 2; ++nf) w[t][nf] = *(const bf16x8*)(a.wf + ((((long)wave * kKS + t) * 2 + nf) * 64 + lane) * 8);
  // the prologue rows (DMA'd before the weights) have landed; the weights may
  // still be in flight (the first step's MFMAs wait for their own fragments;
  // vmcnt tops out at 63 of the 72 weight loads)
  vm_wait<63>();
  __builtin_amdgcn_s_barrier();

  // step 0 is peeled (at a loop header the compiler waits for every
  // outstanding load, which would put the whole weight load back in front
  // of the first MFMA)
  auto step_body = [&](const int step) __attribute__((always_inline)) {
    const int r0 = step * kR;  // output rows r0, r0 + 1; input rows 2 r0 - 1 .. 2 r0 + 3
    if (step + 1 < kSteps)
      for (int yy = 2 * r0 + 4; yy <= 2 * r0 + 7; ++yy) load_row(yy);
    // ring slot of kernel row 0 of every fragment (+ kh rows: immediate, guard slots)
    const int sb = (2 * r0) % kRing;
    int rowoff[kMF];
#pragma unroll
    for (int f = 0; f < kMF; ++f) {
      int sl = sb + prow2[f];
      sl = sl >= kRing ? sl - kRing : sl;
      rowoff[f] = sl * kRB;
    }
    floatx4 acc[kMF][2];
#pragma unroll
    for (int f = 0; f < kMF; ++f)
#pragma unroll
      for (int nf = 0; nf < 2; ++nf) acc[f][nf] = floatx4{0.f, 0.f, 0.f, 0.f};
    // K step t: tap = t >> 2, channel quarter q = t & 3
    auto xread = [&](int t, int f) __attribute__((always_inline)) {
      const int tap = t >> 2, q = t & 3;
      const int kh = tap / 3, kw = tap % 3;
      const int v = (kw == 2) + 2 * (kh == 2);
      const int imm = kh * kRB + (kw == 1 ? kOffKw1 : 0) + q * kPlane;
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
        for (int nf = 0; nf < 2; ++nf)
          acc[f][nf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[t][nf], xc[f], acc[f][nf], 0, 0, 0);
        if (t + 1 < kKS) xc[f] = xread(t + 1, f);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    // ---- epilogue: lane holds channels ch0 + 8g .. +7 of step pixel 16 f + fr
#pragma unroll
    for (int f = 0; f < kMF; ++f) {
      const int p = 16 * f + fr;
      float v[8];
#pragma unroll
      for (int nf = 0; nf < 2; ++nf)
#pragma unroll
        for (int i = 0; i < 4; ++i) v[4 * nf + i] = acc[f][nf][i] + bs[4 * nf + i];
      const long o = (((long)b * kH + r0) * kW + p) * kCO + ch0 + 8 * g;  // element offset
      if constexpr (OUT8) {
        float qv[8];
#pragma unroll
        for (int e = 0; e < 8; ++e)
          qv[e] = fminf(fmaxf((a.relu ? fmaxf(v[e], 0.f) : v[e]) * a.out_inv_scale, -448.f), 448.f);
        const uint2 pk = make_uint2(s2r_e4m3x4(qv[0], qv[1], qv[2], qv[3]), s2r_e4m3x4(qv[4], qv[5], qv[6], qv[7]));
        if (p < kNPix) *(uint2*)((uint8_t*)a.y + o) = pk;
      } else {
        const uint4 pk = pack8_relu(v, a.relu);
        if (p < kNPix) *(uint4*)((bf16*)a.y + o) = pk;
      }
    }
    // the next step's rows have landed (this step's kMF stores may still be
    // in flight: vmcnt retires in order) and every wave is done reading the
    // rows they replace
    vm_wait<kMF>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  };
  step_body(0);
  for (int step = 1; step < kSteps; ++step) step_body(step);
}

}  // namespace

bool conv3x3_s2rows128_supported(int Hin, int Win, int Cin, int Cout) {
  return Hin == kHI && Win == kWI && Cin == kCI && Cout == kCO;
}

void conv3x3_s2rows128(const void* x, const void* wf, const float* bias, void* y, int B, bool relu,
                       float out_inv_scale, hipStream_t s) {
  if (B <= 0) return;
  if (!x || !wf || !bias || !y || (((uintptr_t)x | (uintptr_t)wf | (uintptr_t)y) & 15))
    throw std::invalid_argument("conv3x3_s2rows128: null / misaligned operand");
  if (x == y) throw std::invalid_argument("conv3x3_s2rows128: in-place not supported");
  if ((long)B * kHI * kWI * kCI >= (1L << 31)) throw std::invalid_argument("conv3x3_s2rows128: batch too large");
  S2R128Args a;
  a.x = (const bf16*)x;
  a.wf = (const bf16*)wf;
  a.bias = bias;
  a.y = y;
  a.relu = relu;
  a.out_inv_scale = out_inv_scale;
  const size_t lds = (size_t)kSlotsAlloc * kRB;
  if (out_inv_scale > 0.f)
    hipLaunchKernelGGL(conv3x3_s2rows128_kernel<true>, dim3(B), dim3(256), lds, s, a);
  else
    hipLaunchKernelGGL(conv3x3_s2rows128_kernel<false>, dim3(B), dim3(256), lds, s, a);
  DMLC_HIP_CHECK(hipGetLastError());
}

}  // namespace dmlc
