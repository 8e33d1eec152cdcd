// Weight-stationary row-streaming 3x3/s1/p1 conv for 28x28x128 -> 128 (BN
// folded, optional residual, ReLU): ResNet18 layer2's stride-1 convs
// (layer2.0.conv2, layer2.1.conv1, layer2.1.conv2).
//
// Reference equivalent: those convs + bn (+ residual) + relu of
// tch::vision::resnet18, run per query by `forward_t` (src/services.rs:493).
// As a stream conv (conv3x3_stream.hip) these run 2 rounds of half-image
// workgroups whose 15-row input prologue is exposed each round, with the
// weights streamed from L2 through a register ring (64-70 us at B=256,
// profiles/r2_final_resnet18_kernels.txt). The 32 x 1152 bf16 weights of
// one wave's 32 output channels are 288 VGPRs: with one wave per SIMD the
// whole 128 x 1152 weight matrix fits in one workgroup's registers, so here
// a workgroup walks one image (one round at B = 256) with no weight traffic
// in its loop, the same scheme as conv3x3_s2rows.hip:
//
//  * 4 waves; wave w owns output channels 32w .. 32w + 31 (2 N fragments)
//    for all 112 pixels (7 fragments) of a 4-output-row step; 36 K steps
//    (9 taps x 4 channel quarters) x 14 MFMAs per step;
//  * staged input row: 4 channel-quarter planes of 30 pixel slots x 64 B
//    (slot 0 / 29 = columns -1 / 28, zero; slot x + 1 = column x), rows
//    7680 B (a bank-row multiple) in a ring of 10 + 2 guard slots (copies of
//    slots 0, 1) so a fragment's 3 kernel rows and 4 quarters are immediate
//    offsets of one address per (fragment, kw);
//  * 16-B chunk c of a quarter of stored pixel (y, x) sits at physical chunk
//    c ^ ((K >> 1) & 3), K = 28 y + x: along a fragment K is the output pixel
//    index plus a tap constant, also across a row wrap, and every
//    ds_read_b128 is conflict free (tests/test_layouts_cpu.py); kernel rows
//    0 and 2 differ from row 1 by 28 in K, an XOR of 2 on the chunk;
//  * the pad slots are zeroed once (no zero-page DMA: one hot L2 channel
//    per XCD); the 4 rows of the next step arrive by LDS-DMA (wave w: its
//    own quarter plane) while the current step computes.
#include "common.h"
#include "kernels.h"

#include <cstdlib>
#include <type_traits>

namespace dmlc {

namespace {

template <int N>
__device__ __forceinline__ void vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}

struct R28Args {
  const bf16* x;      // [B, 28, 28, 128]
  const bf16* wf;     // weights, fragment order [4][36][2][64][8] (stream_frag_index, K = 1152)
  const float* bias;  // [128]
  const bf16* res;    // [B, 28, 28, 128] or null
  bf16* y;            // [B, 28, 28, 128] (OUT8: e4m3 bytes)
  int relu;
  float out_inv_scale;  // OUT8: y = e4m3(relu(v) * out_inv_scale)
  // DSX (ResNet18 layer2.0.conv2, ds_into_conv2): the block's 1x1/s2
  // downsample of its input xds [B, 56, 56, 64] as 2 more K steps of this
  // conv (K = 1152 + 64), weights wds in fragment order [4][2][2][64][8],
  // bias bds added to bias: y = relu(conv3x3(x) + b + wds * xds[2y, 2x] + bds),
  // exactly the residual block's output without the yd round trip
  const bf16* xds;
  const bf16* wds;
  const float* bds;
  int stagger;  // start_stagger (common.h)
};

// 4 floats (within +-448) -> 4 e4m3 bytes
__device__ __forceinline__ uint32_t r28_e4m3x4(float a, float b, float c, float d) {
  int v = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
  v = __builtin_amdgcn_cvt_pk_fp8_f32(c, d, v, true);
  return (uint32_t)v;
}

constexpr int kH = 28, kW = 28, kC = 128;
constexpr int kR = 4;                 // output rows per step
constexpr int kSteps = kH / kR;       // 7
constexpr int kPlane = 30 * 64;       // one channel quarter of a staged row: 1920 B
constexpr int kRB = 4 * kPlane;       // 7680 B per staged row
// Input rows are DMA'd one step ahead: rows r0 - 1 .. r0 + 4 in use + 4 in
// flight (10-row ring; two steps ahead, a 14-row ring, measured slower: 48.2-48.9
// vs 51.5-52.0 us at B = 256 with warm clocks, profiles/r3_rows28_ahead.txt).
constexpr int kRing = 10;
constexpr int kSlotsAlloc = kRing + 2;  // + guard copies of slots 0, 1
constexpr int kRun = 4 * kW;          // 112 DMA chunks per quarter plane (slots 1..28)
constexpr int kMF = kR * kW / 16;     // 7 pixel fragments per step
constexpr int kKS = 9 * kC / 32;      // 36 K steps
constexpr int kResCh = kMF * 16 * 16;  // residual chunks per step (112 pixels x 16)

__device__ __forceinline__ int swz_of(int y, int x) { return ((kW * y + x) >> 1) & 3; }

// 4 waves (one per SIMD) x 32 output channels, 288 weight registers per wave
// (their AGPR / VGPR split costs ~0.6 register moves per MFMA; 8 waves x 16
// channels measured slower, profiles/r3_rows28_ahead.txt).
// OUT8: e4m3 output (ResNet50's layer2 3x3 -> its e4m3 expand conv; no residual)
// DSX: see R28Args::xds (no residual operand: the downsample is the residual)
// RES: the residual is DMA'd one step ahead into two LDS buffers, so the
// epilogue reads it with no wait and no workgroup barrier of its own (the
// previous step's end-of-step wait covered it)
template <bool RES, bool OUT8 = false, bool DSX = false>
__global__ __launch_bounds__(256, 1) void conv3x3_rows28_kernel(R28Args a) {
  static_assert(!OUT8 || !RES, "e4m3 output: no residual");
  static_assert(!DSX || (!RES && !OUT8), "downsample K steps: the bf16 form");
  constexpr int kDS = DSX ? 2 : 0;  // downsample K steps (64 input channels)
  constexpr int kRB2 = kResCh * 16;  // 28672 B per residual buffer
  constexpr int NF = 2;  // N fragments (16 channels) per wave
  constexpr int NT = 256;
  extern __shared__ __attribute__((aligned(16))) uint4 smem[];
  char* ring = (char*)smem;
  char* resbuf = ring + kSlotsAlloc * kRB;  // RES: [112 pixels][16 chunks]
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  start_stagger(a.stagger);
  const int fr = lane & 15, g = lane >> 4;
  const int b = blockIdx.x;
  const bf16* img = a.x + (long)b * kH * kW * kC;

  for (int o = tid * 16; o < kSlotsAlloc * kRB; o += NT * 16) *(uint4*)(ring + o) = make_uint4(0, 0, 0, 0);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  // input row yy -> ring slot (yy + 1) % kRing (+ guard slot kRing / kRing+1
  // for slots 0 / 1); wave w stages quarter plane w & 3: chunks 0..63 and
  // 64..111 of its run. Row 28 (below the image) reuses a slot: its run is
  // written as zeros.
  const int qp = wave & 3;  // the quarter plane this wave stages
  auto load_row = [&](int yy) __attribute__((always_inline)) {
    const int slot = (yy + 1) % kRing;
    char* dst = ring + qp * kPlane + 64;
#pragma unroll
    for (int i0 = 0; i0 < kRun; i0 += 64) {
      const int k = i0 + lane;
      const int x = k >> 2, c = k & 3;
      if (k < kRun) {
        if (yy < kH) {
          const bf16* src = img + ((long)yy * kW + x) * kC + 32 * qp + 8 * (c ^ swz_of(yy, x));
          dma16(src, dst + slot * kRB + i0 * 16);
          if (slot < 2) dma16(src, dst + (slot + kRing) * kRB + i0 * 16);
        } else {
          *(uint4*)(dst + slot * kRB + k * 16) = make_uint4(0, 0, 0, 0);
          if (slot < 2) *(uint4*)(dst + (slot + kRing) * kRB + k * 16) = make_uint4(0, 0, 0, 0);
        }
      }
    }
  };
  // this lane's 8 output channels ch0 + 8g .. +7 (weight rows permuted,
  // perm32); loaded before the row DMAs so the prologue wait below can leave
  // exactly the weight loads in flight
  const int cg = wave;
  const int ch0 = cg * 32;
  constexpr int CPL = 4 * NF;  // output channels per lane
  float bs[CPL];
#pragma unroll
  for (int e = 0; e < CPL; ++e) bs[e] = a.bias[ch0 + 8 * g + e];
  if constexpr (DSX)
#pragma unroll
    for (int e = 0; e < CPL; ++e) bs[e] += a.bds[ch0 + 8 * g + e];
  // DSX: the downsample's input pixels x[2 (r0 + p / 28), 2 (p % 28)] of
  // step s (128 B each) -> LDS buffer s & 1 [112 pixels][8 chunks], chunk c
  // at physical c ^ (p & 7): the B-fragment reads of the 2 downsample K steps
  // are conflict free (tests/test_layouts_cpu.py). DMA'd one step ahead, so
  // the downsample K steps open a step's K loop with no wait of their own
  constexpr int kDSB = kMF * 16 * 8 * 16;  // 14336 B per buffer
  auto ds_dma = [&](int st) __attribute__((always_inline)) {
    const bf16* ximg = a.xds + (long)b * (2 * kH) * (2 * kW) * 64;
    const int r0s = st * kR;
    char* dst = resbuf + (st & 1) * kDSB;
    // (an opaque lane id: hoisted out of the step loop, the per-lane part of
    // these addresses stayed live across the K loop and spilled)
    int ln = lane;
    asm volatile("" : "+v"(ln));
#pragma unroll
    for (int j = 0; j < (kMF * 16 * 8 + NT - 1) / NT; ++j) {
      const int i0 = j * NT + wave * 64;
      if (i0 < kMF * 16 * 8) {
        const int i = i0 + ln;
        const int p = i >> 3, c = (i & 7) ^ (p & 7);
        const int yy = 2 * (r0s + p / kW), xx = 2 * (p % kW);
        dma16(ximg + ((long)yy * (2 * kW) + xx) * 64 + 8 * c, dst + i0 * 16);
      }
    }
  };
  auto res_dma = [&](int st, char* dst) __attribute__((always_inline)) {
    const bf16* rimg = a.res + ((long)b * kH + st * kR) * kW * kC;
    int ln = lane;  // (opaque: see ds_dma)
    asm volatile("" : "+v"(ln));
#pragma unroll
    for (int j = 0; j < (kResCh + NT - 1) / NT; ++j) {
      const int i0 = j * NT + wave * 64;
      if (i0 < kResCh) {  // (wave-uniform: kResCh is a multiple of 64)
        const int i = i0 + ln;
        const int p = i >> 4, c = i & 15;
        dma16(rimg + (long)p * kC + 8 * (c ^ (p & 15)), dst + i0 * 16);
      }
    }
  };
  if constexpr (DSX) ds_dma(0);  // (older than the rows: the prologue's wait covers it)
  if constexpr (RES) res_dma(0, resbuf);
  for (int yy = 0; yy <= 4; ++yy) load_row(yy);
  __builtin_amdgcn_sched_barrier(0);  // (the staging arithmetic is dead before the 304 weight registers load)

  // ---- per-lane constants: fragment f = tile pixels p = 16 f + fr (row
  // p / 28 of the step, column p % 28). col[f][kw]: in-row byte offset of
  // quarter 0 for kernel row 1; rows 0 / 2 flip chunk bit 1 (XOR 32).
  int prow[kMF], col[kMF][3];
#pragma unroll
  for (int f = 0; f < kMF; ++f) {
    const int p = 16 * f + fr;
    prow[f] = p / kW;
    const int c = p % kW;
#pragma unroll
    for (int kw = 0; kw < 3; ++kw) {
      const int s = ((p + kw - 1) >> 1) & 3;  // K & ... of (r0 + prow, c + kw - 1), r0 % 4 == 0
      col[f][kw] = (c + kw) * 64 + ((g ^ s) << 4);
    }
  }
  bf16x8 w[kKS + kDS][NF];
#pragma unroll
  for (int t = 0; t < kKS; ++t)
#pragma unroll
    for (int nf = 0; nf < NF; ++nf)
      w[t][nf] = *(const bf16x8*)(a.wf + ((((long)cg * kKS + t) * 2 + nf) * 64 + lane) * 8);
#pragma unroll
  for (int t = 0; t < kDS; ++t)
#pragma unroll
    for (int nf = 0; nf < NF; ++nf)
      w[kKS + t][nf] = *(const bf16x8*)(a.wds + ((((long)cg * kDS + t) * 2 + nf) * 64 + lane) * 8);
  // the prologue rows (DMA'd before the weights) have landed; the weights
  // (72 loads, 288 KB per workgroup from L2) may still be in flight: the
  // first step's MFMAs wait for each K step's own fragments (the compiler's
  // counted waits), so the load overlaps the first step instead of preceding it
  vm_wait<63>();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();

  // step 0 is peeled (a separate copy of the body): at a loop header the
  // compiler waits for every outstanding load (vmcnt(0)), which would put the
  // whole weight load back in front of the first MFMA
  auto step_body = [&](const int step) __attribute__((always_inline)) {
    const int r0 = step * kR;  // output rows r0 .. r0 + 3; input rows r0 - 1 .. r0 + 4
    // residual of this step's 112 output pixels -> LDS (lands during the K
    // loop; registers are full of weights): 16-B chunk c of pixel p at
    // physical chunk c ^ (p & 15), so the epilogue's reads are conflict free.
    // Issued before this step's row DMAs: its wait leaves those in flight.
    const long obase = ((long)b * kH + r0) * kW * kC + ch0 + 8 * g;
    if constexpr (DSX)  // the next step's downsample input (this step's landed during the last one)
      if (step + 1 < kSteps) ds_dma(step + 1);
    if constexpr (RES)  // the next step's residual
      if (step + 1 < kSteps) res_dma(step + 1, resbuf + ((step + 1) & 1) * kRB2);
    // the rows of the next step
    if (step + 1 < kSteps)
      for (int yy = 4 * step + 5; yy <= 4 * step + 8; ++yy) load_row(yy);
    // ring slot of kernel row 0 of each fragment (+ kh rows: immediate, guard slots)
    int rowoff[kMF];
#pragma unroll
    for (int f = 0; f < kMF; ++f) {
      int sl = r0 % kRing + prow[f];  // slot of input row r0 + prow - 1
      sl = sl >= kRing ? sl - kRing : sl;
      rowoff[f] = sl * kRB;
    }
    // K step t: tap = t >> 2 (kh = tap / 3, kw = tap % 3), quarter q = t & 3
    // tb[f]: fragment f's address for the current tap (quarter 0, kernel row
    // 0's slot; kh and the quarter are immediates). Computed by volatile asm
    // at its point of use, so the compiler neither hoists nor keeps the 63
    // per-(fragment, tap) sums live (the weights hold 288 registers).
    int tb[kMF];
    auto tap_addr = [&](int tap, int f) __attribute__((always_inline)) {
      const int kh = tap / 3, kw = tap % 3;
      if (kh == 1)
        asm volatile("v_add_u32 %0, %1, %2" : "=v"(tb[f]) : "v"(rowoff[f]), "v"(col[f][kw]));
      else
        asm volatile("v_xor_b32 %0, 32, %1\n\tv_add_u32 %0, %2, %0" : "=&v"(tb[f]) : "v"(col[f][kw]), "v"(rowoff[f]));
    };
    auto xread = [&](int t, int f) __attribute__((always_inline)) {
      const int tap = t >> 2, q = t & 3;
      if (q == 0) tap_addr(tap, f);
      return *(const bf16x8*)(ring + tb[f] + (tap / 3) * kRB + q * kPlane);
    };
    // the step's fragments: the K loop, then their epilogue
    {
      constexpr int FB = 0, PF = kMF;
      // the bias is the first MFMA's accumulator input (no zeroing, no bias
      // adds in the epilogue, which with one wave per SIMD runs with the
      // matrix core idle)
      floatx4 acc[PF][NF], bv[NF];
#pragma unroll
      for (int nf = 0; nf < NF; ++nf) bv[nf] = floatx4{bs[4 * nf], bs[4 * nf + 1], bs[4 * nf + 2], bs[4 * nf + 3]};
      bf16x8 xc[PF];
#pragma unroll
      for (int f = 0; f < PF; ++f) xc[f] = xread(0, FB + f);
#pragma unroll
      for (int t = 0; t < kKS; ++t) {
#pragma unroll
        for (int f = 0; f < PF; ++f) {
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int nf = 0; nf < NF; ++nf)
            acc[f][nf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[t][nf], xc[f], t == 0 ? bv[nf] : acc[f][nf], 0, 0, 0);
          if (t + 1 < kKS) xc[f] = xread(t + 1, FB + f);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (DSX) {
        // the 2 downsample K steps on this step's x[2y, 2x], DMA'd during the
        // previous step (its end-of-step wait and barrier covered it: no wait
        // and no workgroup barrier here)
        const char* dsb = resbuf + (step & 1) * kDSB;
#pragma unroll
        for (int u = 0; u < kDS; ++u) {
#pragma unroll
          for (int f = 0; f < PF; ++f) {
            const int p = 16 * (FB + f) + fr;
            xc[f] = *(const bf16x8*)(dsb + p * 128 + (((4 * u + g) ^ (p & 7)) << 4));
          }
#pragma unroll
          for (int f = 0; f < PF; ++f)
#pragma unroll
            for (int nf = 0; nf < NF; ++nf)
              acc[f][nf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[kKS + u][nf], xc[f], acc[f][nf], 0, 0, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      // ---- epilogue: lane holds channels ch0 + 8g .. +7 of tile pixel 16 f + fr
#pragma unroll
      for (int f = 0; f < PF; ++f) {
        const int ff = FB + f;
        float v[8];
#pragma unroll
        for (int nf = 0; nf < NF; ++nf)
#pragma unroll
          for (int i = 0; i < 4; ++i) v[4 * nf + i] = acc[f][nf][i];
        const char* rp = resbuf + (RES ? (step & 1) * kRB2 : 0) + (16 * ff + fr) * 256 + (((4 * cg + g) ^ fr) << 4);
        {
          if constexpr (RES) {
            // residual bf16 pairs added by v_dot2c_f32_bf16 (pair . (1, 0) /
            // (0, 1): exact), one VALU per channel instead of an unpack and
            // an add; the selectors live in registers (as an inline constant
            // the pair (1, 0) became f32 1.0 = (0, 1): conv3x3_block.hip)
            typedef __bf16 bf16x2v __attribute__((ext_vector_type(2)));
            uint32_t slo = 0x00003f80u, shi = 0x3f800000u;
            asm volatile("" : "+v"(slo), "+v"(shi));
            const uint4 rr = *(const uint4*)rp;
            const uint32_t rw4[4] = {rr.x, rr.y, rr.z, rr.w};
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const bf16x2v pr = __builtin_bit_cast(bf16x2v, rw4[i]);
              v[2 * i] = __builtin_amdgcn_fdot2_f32_bf16(pr, __builtin_bit_cast(bf16x2v, slo), v[2 * i], false);
              v[2 * i + 1] = __builtin_amdgcn_fdot2_f32_bf16(pr, __builtin_bit_cast(bf16x2v, shi), v[2 * i + 1], false);
            }
          }
          if constexpr (OUT8) {
            float q[8];
#pragma unroll
            for (int e = 0; e < 8; ++e)
              q[e] = fminf(fmaxf((a.relu ? fmaxf(v[e], 0.f) : v[e]) * a.out_inv_scale, -448.f), 448.f);
            *(uint2*)((uint8_t*)a.y + obase + (long)(16 * ff + fr) * kC) =
                make_uint2(r28_e4m3x4(q[0], q[1], q[2], q[3]), r28_e4m3x4(q[4], q[5], q[6], q[7]));
          } else {
            *(uint4*)(a.y + obase + (long)(16 * ff + fr) * kC) = pack8_relu(v, a.relu);
          }
        }
      }
    }
    // the next step's rows have landed and every wave is done with the rows
    // they replace. vmcnt retires in order; younger than those rows: this
    // step's kMF stores (step 0: its K loop already drained every load, the
    // compiler's waits on the weights)
    vm_wait<kMF>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  };
  step_body(0);
  for (int step = 1; step < kSteps; ++step) step_body(step);
}

}  // namespace

bool conv3x3_rows28_supported(int H, int W, int Cin, int Cout) {
  return H == kH && W == kW && Cin == kC && Cout == kC;
}

void conv3x3_rows28(const void* x, const void* wf, const float* bias, const void* res, void* y, int B, bool relu,
                    hipStream_t s, float out_inv_scale, const void* xds, const void* wds, const float* bds) {
  if (B <= 0) return;
  if (xds || wds || bds) {  // the block's downsample as 2 more K steps (ds_into_conv2)
    if (!xds || !wds || !bds || res || out_inv_scale > 0.f || !x || !wf || !bias || !y ||
        (((uintptr_t)x | (uintptr_t)wf | (uintptr_t)xds | (uintptr_t)wds | (uintptr_t)y) & 15))
      throw std::invalid_argument("conv3x3_rows28: downsample K steps need xds, wds, bds (no residual, bf16 out)");
    if (x == y || xds == y) throw std::invalid_argument("conv3x3_rows28: in-place not supported");
    R28Args a{};
    a.x = (const bf16*)x;
    a.wf = (const bf16*)wf;
    a.bias = bias;
    a.y = (bf16*)y;
    a.relu = relu;
    a.xds = (const bf16*)xds;
    a.wds = (const bf16*)wds;
    a.bds = bds;
    a.stagger = kernel_stagger(kStagRows28);
    const size_t lds = (size_t)kSlotsAlloc * kRB + 2 * (size_t)kMF * 16 * 128;  // two downsample-input buffers
    hipLaunchKernelGGL((conv3x3_rows28_kernel<false, false, true>), dim3(B), dim3(256), lds, s, a);
    DMLC_HIP_CHECK(hipGetLastError());
    return;
  }
  if (out_inv_scale > 0.f && res) throw std::invalid_argument("conv3x3_rows28: e4m3 output without residual only");
  if (!x || !wf || !bias || !y ||
      (((uintptr_t)x | (uintptr_t)wf | (uintptr_t)res | (uintptr_t)y) & 15))
    throw std::invalid_argument("conv3x3_rows28: null / misaligned operand");
  if (x == y || (res && res == y)) throw std::invalid_argument("conv3x3_rows28: in-place not supported");
  R28Args a{};
  a.x = (const bf16*)x;
  a.wf = (const bf16*)wf;
  a.bias = bias;
  a.res = (const bf16*)res;
  a.y = (bf16*)y;
  a.relu = relu;
  a.out_inv_scale = out_inv_scale;
  a.stagger = kernel_stagger(kStagRows28);
  if (out_inv_scale > 0.f) {
    hipLaunchKernelGGL((conv3x3_rows28_kernel<false, true>), dim3(B), dim3(256),
                       (size_t)kSlotsAlloc * kRB, s, a);
    DMLC_HIP_CHECK(hipGetLastError());
    return;
  }
  // (the residual is double-buffered one step ahead)
  const size_t lds = (size_t)kSlotsAlloc * kRB + (res ? (size_t)2 * kResCh * 16 : 0);  // 90 / 151 KB
  static_assert(kSlotsAlloc * kRB + 2 * kResCh * 16 <= 160 * 1024, "LDS budget");
  if (res)
    hipLaunchKernelGGL(conv3x3_rows28_kernel<true>, dim3(B), dim3(256), lds, s, a);
  else
    hipLaunchKernelGGL(conv3x3_rows28_kernel<false>, dim3(B), dim3(256), lds, s, a);
  DMLC_HIP_CHECK(hipGetLastError());
}

}  // namespace dmlc
