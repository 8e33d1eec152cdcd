// Fused ResNet basic block for narrow layers (ResNet18 layer1: 56x56x64):
//   y = relu(bn2(conv2(relu(bn1(conv1(x))))) + x)
// in ONE kernel, the intermediate activation never leaving LDS.
//
// Reference equivalent: layer1.{0,1} (BasicBlock: conv1/bn1/relu, conv2/bn2,
// += identity, relu) of tch::vision::resnet18, run per query by `forward_t`
// (src/services.rs:493). As two conv3x3_rows launches each block writes its
// 103 MB intermediate at B=256, reads it back, and reads the block input a
// second time for the residual; here only x in and y out touch memory.
//
// One workgroup = one whole image (56 rows), 8 waves:
//  * waves 0-3 PRODUCE the intermediate t = relu(conv1(x) + b1): 4 rows per
//    step from a 10-row LDS-DMA ring of x (the conv3x3_rows layout: 58 staged
//    columns with zero pads, 16-B chunks XOR-swizzled by column), written as
//    bf16 into a 10-row LDS ring of t with the same layout;
//  * waves 4-7 CONSUME it: conv2 over t rows + b2 + residual (x rows re-read
//    from L2/MALL: they were DMA'd a few steps earlier) + ReLU -> y.
//  Producer wave w and consumer wave w+4 share SIMD w: matrix work of both
//  roles interleaves on every SIMD. Each role's 4 waves = 2 pixel halves (2
//  rows x 56 = 7 fragments of 16 pixels) x 2 channel halves (2 N fragments),
//  weights streamed per wave from L2 in fragment order through a register
//  ring (the WR scheme of conv3x3_rows / conv3x3_stream).
//
// Pipeline (o = image row, P_k = t rows 4k+1..4k+4, P_-1 = t rows -1, 0;
// C_k = y rows 4k..4k+3, which needs t rows 4k-1..4k+4):
//   step 0: producers P_-1 (pixel half 1 only: tile base row -3)
//   step s >= 1: producers P_{s-1} (s <= 14), consumers C_{s-2} (s >= 2)
// one workgroup barrier per step. t rows -1 and 56 are the conv2 padding and
// are written as zeros. Ring slots: t row r -> (r + 10) % 10 (rows read and
// written in one step span 10 rows), x row r -> (r + 10) % 10 likewise.
#include "common.h"
#include "kernels.h"

#include <type_traits>

namespace dmlc {

namespace {

template <int N>
__device__ __forceinline__ void vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}

struct BlockArgs {
  const bf16* x;       // [B, 56, 56, 64]
  const bf16* wf1;     // conv1 weights, fragment order [2][KS][2][64][8] (stream_frag_index, K = 576)
  const bf16* wf2;     // conv2 weights, same order
  const float* bias1;  // [64]
  const float* bias2;  // [64]
  bf16* y;             // [B, 56, 56, 64]
  const bf16* zero;    // >= 16 zero bytes
  int stagger;         // start_stagger (common.h)
};

constexpr int kH = 56, kW = 56, kC = 64;
constexpr int kR = 4;                  // rows per step
constexpr int kMF = kR * kW / 32;      // 7 pixel fragments per wave (2 pixel halves)
constexpr int kKS = 9 * kC / 32;       // 18 K steps
constexpr int kQ = kW + 2;             // staged columns
constexpr int kHalf = kQ * 64;         // one K half (32 channels) of a staged row: 3712 B
constexpr int kSlot = 2 * kHalf;       // 7424 B per staged row
constexpr int kRing = 10;
constexpr int kRun = 4 * kW;           // 224 DMA chunks per K half of a row (q = 1..56)
constexpr int kSteps = kH / kR + 2;    // 16

// One role's whole pipeline (PROD: conv1 producer, else conv2 consumer).
// Both roles pass the same kSteps + 1 workgroup barriers.
// PD: weight register ring depth (divides kKS; PD - 1 K steps of lookahead).
// DMA_KS: K step at which producers issue the next step's x-row DMA (vmcnt
// retires in order: a weight load issued after the DMA cannot be waited on
// without waiting for the DMA too).
template <bool PROD, int PD, int DMA_KS>
__device__ __forceinline__ void block_role(const BlockArgs& a, char* xring, char* tring, int rw, int lane) {
  const int wm = rw & 1, wn = rw >> 1;
  const int fr = lane & 15, g = lane >> 4;
  const int b = blockIdx.x;
  const bf16* img = a.x + (long)b * kH * kW * kC;

  // ---- x row r (-1 / 56: zero row) -> x ring. Staged layout (x and t
  // rings): [row slot][K half h][column q][4 chunks of 16 B], chunk c of
  // (h, q) holding channels 8*(4h + (c ^ ((q >> 1) & 3))); zeros at q = 0,
  // 57. The h = 1 fragment of a tap is the h = 0 one + kHalf (an immediate
  // ds_read offset), and every 16-lane group of a ds_read_b128 / ds_write_b128
  // hits 16 distinct bank groups (tests/test_layouts_cpu.py). Producers only.
  // The pad columns q = 0, 57 and the zero row -1 are zeroed once (kernel
  // start) and never DMA'd: a zero page read by every workgroup's pad lanes
  // is one hot L2 channel per XCD (conv3x3_s2rows.hip measured 7 us of it).
  // Row 56 reuses a ring slot, so its data chunks are written as zeros.
  // Per K half the chunks of q = 1..56 are one contiguous run of 224;
  // wave rw DMAs chunks 64 rw .. 64 rw + 63 of both runs.
  auto load_row = [&](int r) __attribute__((always_inline)) {
    char* dst = xring + ((r + kRing) % kRing) * kSlot + 64 + rw * 1024;
    const int k = rw * 64 + lane;
    const int q = 1 + (k >> 2), c = k & 3;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      if (k < kRun) {
        if (r < kH)
          dma16(img + ((long)r * kW + (q - 1)) * kC + 8 * (4 * h + (c ^ ((q >> 1) & 3))), dst + h * kHalf);
        else
          *(uint4*)(dst + h * kHalf + lane * 16) = make_uint4(0, 0, 0, 0);
      }
    }
  };
  // x rows -1 .. 5: P_-1 needs x rows -2..1 (row -2 only feeds t row -1,
  // which is written as zeros), P_0 needs rows 0..5
  if constexpr (PROD)
    for (int r = 0; r <= 5; ++r) load_row(r);

  // ---- per-lane constants (4-row tile, 2 pixel halves)
  // fragment f, lane fr: pixel p = wm*112 + 16f + fr of the tile, in tile row
  // 2wm + bit f of hi1. Its input for tap (kh, kw), K half h sits at ring row
  // base + 2wm + hi + kh - 1 (a wave-uniform slot offset picked per lane) and
  // staged column q = col + kw, chunk g ^ ((q >> 1) & 3) of K half h.
  int hi1 = 0, colq[kMF][3];
#pragma unroll
  for (int f = 0; f < kMF; ++f) {
    const int p = wm * (kR * kW / 2) + 16 * f + fr;
    hi1 |= (p / kW - 2 * wm) << f;
    const int col = p % kW;
#pragma unroll
    for (int kw = 0; kw < 3; ++kw) {
      const int q = col + kw;
      colq[f][kw] = q * 64 + ((g ^ ((q >> 1) & 3)) << 4);
    }
  }
  const __amdgpu_buffer_rsrc_t wrs =
      wave_rsrc((PROD ? a.wf1 : a.wf2) + (long)wn * kKS * 2 * 64 * 8, kKS * 2 * 1024);
  auto wload = [&](int kf) __attribute__((always_inline)) {
    return __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(wrs, lane * 16, kf * 1024, 0));
  };
  static_assert(kKS % PD == 0, "ring period");
  bf16x8 wq[PD][2];
#pragma unroll
  for (int ks = 0; ks < PD - 1; ++ks)
#pragma unroll
    for (int nf = 0; nf < 2; ++nf) wq[ks][nf] = wload(ks * 2 + nf);
  // this lane's 8 output channels: wn*32 + 8g .. +7 (weight rows permuted, perm32)
  const float* bias = PROD ? a.bias1 : a.bias2;
  float bs[2][4];
#pragma unroll
  for (int nf = 0; nf < 2; ++nf)
#pragma unroll
    for (int i = 0; i < 4; ++i) bs[nf][i] = bias[wn * 32 + 8 * g + 4 * nf + i];

  vm_wait<0>();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();

  const char* src_ring = PROD ? xring : tring;
  for (int step = 0; step < kSteps; ++step) {
    // producer: t rows base..base+3 = P_{step-1} (step 0: base -3, only rows
    // -1, 0 = pixel half 1); consumer: y rows base..base+3 = C_{step-2}
    const bool work = PROD ? (step <= kH / kR && (step > 0 || wm == 1)) : step >= 2;
    const int base = PROD ? (step == 0 ? -3 : 4 * (step - 1) + 1) : 4 * (step - 2);
    // producers: DMA the new x rows of the next producer step (its t rows
    // nb..nb+3 need x rows nb-1..nb+4; up to nb are here already)
    auto issue_dma = [&]() __attribute__((always_inline)) {
      if (PROD && step + 1 <= kH / kR) {
        const int nb = step == 0 ? 1 : base + 4;
        for (int r = nb + 1; r <= nb + 4; ++r)
          if (r >= 6) load_row(r);
      }
    };
    if (DMA_KS == 0 || !work) issue_dma();
    if (work) {
      // ring offsets of tile rows 2wm - 1 .. 2wm + 2 (wave-uniform; named
      // scalars, not an array: a select between array elements becomes a
      // dynamically indexed private array)
      const int rb = base + 2 * wm - 1 + 2 * kRing;
      const int rs0 = (rb % kRing) * kSlot, rs1 = ((rb + 1) % kRing) * kSlot;
      const int rs2 = ((rb + 2) % kRing) * kSlot, rs3 = ((rb + 3) % kRing) * kSlot;
      auto rsl = [&](int j) __attribute__((always_inline)) { return j == 0 ? rs0 : j == 1 ? rs1 : j == 2 ? rs2 : rs3; };
      // consumer: residual rows (x), loaded now so they land during the MFMAs
      const long obase = ((long)b * kH + base) * kW * kC;
      uint4 rres[PROD ? 1 : kMF];
      if constexpr (!PROD) {
#pragma unroll
        for (int f = 0; f < kMF; ++f) {
          const int p = wm * (kR * kW / 2) + 16 * f + fr;
          rres[f] = *(const uint4*)(a.x + obase + (long)p * kC + wn * 32 + 8 * g);
        }
      }
      floatx4 acc[kMF][2];
      // the bias is the first MFMA's accumulator input (no zeroing, no bias
      // adds in the epilogue)
      const floatx4 bv[2] = {floatx4{bs[0][0], bs[0][1], bs[0][2], bs[0][3]},
                             floatx4{bs[1][0], bs[1][1], bs[1][2], bs[1][3]}};
      bf16x8 xc[kMF], xn[kMF];
      auto load_k = [&](int ks, bf16x8* xd) __attribute__((always_inline)) {
        const int tap = ks >> 1, h = ks & 1;
        const int kh = tap / 3, kw = tap % 3;
#pragma unroll
        for (int f = 0; f < kMF; ++f)
          xd[f] = *(const bf16x8*)(src_ring + (((hi1 >> f) & 1) ? rsl(kh + 1) : rsl(kh)) + colq[f][kw] + h * kHalf);
      };
      load_k(0, xc);
#pragma unroll
      for (int ks = 0; ks < kKS; ++ks) {
        if (ks + 1 < kKS) load_k(ks + 1, xn);
        if (DMA_KS > 0 && ks == DMA_KS) issue_dma();
        {  // K step ks + PD - 1 (wrapping into the next step's first ones)
          const int kl = (ks + PD - 1) % kKS;
#pragma unroll
          for (int nf = 0; nf < 2; ++nf) wq[(ks + PD - 1) % PD][nf] = wload(kl * 2 + nf);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int f = 0; f < kMF; ++f)
#pragma unroll
          for (int nf = 0; nf < 2; ++nf)
            acc[f][nf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wq[ks % PD][nf], xc[f],
                                                                 ks == 0 ? bv[nf] : acc[f][nf], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
        if (ks + 1 < kKS) {
#pragma unroll
          for (int f = 0; f < kMF; ++f) xc[f] = xn[f];
        }
      }
      // ---- epilogue: lane holds channels wn*32 + 8g .. +7 of pixel (row, col)
      // ~17 VALU per fragment instead of ~41 (the epilogues of both roles
      // meet at the step barrier with the matrix cores idle, and an MFMA
      // leaves its SIMD 8 of its 16 cycles for other vector instructions):
      // bias already in the accumulators, the residual added from its bf16
      // pairs by v_dot2c_f32_bf16 (x.lo * 1 + x.hi * 0: exact), ReLU and the
      // padding rows' zeros on the packed bf16 words
      {
        typedef __bf16 bf16x2v __attribute__((ext_vector_type(2)));
        // (bf16 1.0 = 0x3f80 in the low / high half, kept in registers: the
        // compiler turned the constant pair into the inline constant 1.0,
        // which the hardware reads as the f32 bits 0x3f800000 = (0, 1))
        uint32_t slo = 0x00003f80u, shi = 0x3f800000u;
        asm volatile("" : "+v"(slo), "+v"(shi));
        const bf16x2v sel_lo = __builtin_bit_cast(bf16x2v, slo), sel_hi = __builtin_bit_cast(bf16x2v, shi);
#pragma unroll
        for (int f = 0; f < kMF; ++f) {
          const int p = wm * (kR * kW / 2) + 16 * f + fr;
          float v[8];
#pragma unroll
          for (int nf = 0; nf < 2; ++nf)
#pragma unroll
            for (int i = 0; i < 4; ++i) v[4 * nf + i] = acc[f][nf][i];
          if constexpr (PROD) {
            const int row = base + p / kW, col = p % kW;
            const bool outside = (unsigned)row >= (unsigned)kH;
            const int q = col + 1;
            const uint4 pk = relu_bf16x8(pack8(v));
            *(uint4*)(tring + ((row + kRing) % kRing) * kSlot + wn * kHalf + q * 64 + ((g ^ ((q >> 1) & 3)) << 4)) =
                outside ? make_uint4(0, 0, 0, 0) : pk;
          } else {
            const uint32_t rw4[4] = {rres[f].x, rres[f].y, rres[f].z, rres[f].w};
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const bf16x2v rp = __builtin_bit_cast(bf16x2v, rw4[i]);
              v[2 * i] = __builtin_amdgcn_fdot2_f32_bf16(rp, sel_lo, v[2 * i], false);
              v[2 * i + 1] = __builtin_amdgcn_fdot2_f32_bf16(rp, sel_hi, v[2 * i + 1], false);
            }
            const uint4 pk = relu_bf16x8(pack8(v));
            *(uint4*)(a.y + obase + (long)p * kC + wn * 32 + 8 * g) = pk;
          }
        }
      }
    }
    // (an idle role's weight ring needs nothing: it is periodic over K steps)
    // t rows written and the next step's x rows landed, for every wave
    if constexpr (PROD) vm_wait<0>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  }
}

template <int PD, int DMA_KS>
__global__ __launch_bounds__(512, 1) void conv3x3_block_kernel(BlockArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint4 smem[];
  char* xring = (char*)smem;
  char* tring = xring + kRing * kSlot;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  start_stagger(a.stagger);
  // zero both rings (pad columns stay zero; x row -1 is the zeroed slot 9;
  // t halo rows are written as zeros), before any x-row DMA lands
  for (int i = tid; i < 2 * kRing * kSlot / 16; i += 512) ((uint4*)xring)[i] = make_uint4(0, 0, 0, 0);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  if (wave < 4)
    block_role<true, PD, DMA_KS>(a, xring, tring, wave & 3, lane);
  else
    block_role<false, PD, DMA_KS>(a, xring, tring, wave & 3, lane);
}

}  // namespace

bool conv3x3_block_supported(int H, int W, int C) { return H == kH && W == kW && C == kC; }

void conv3x3_block(const void* x, const void* wf1, const float* bias1, const void* wf2, const float* bias2, void* y,
                   const void* zero, int B, hipStream_t s) {
  if (B <= 0) return;
  if (!x || !wf1 || !wf2 || !bias1 || !bias2 || !y || !zero ||
      (((uintptr_t)x | (uintptr_t)wf1 | (uintptr_t)wf2 | (uintptr_t)y | (uintptr_t)zero) & 15))
    throw std::invalid_argument("conv3x3_block: null / misaligned operand");
  if (x == y) throw std::invalid_argument("conv3x3_block: in-place not supported (the residual is re-read)");
  BlockArgs a;
  a.x = (const bf16*)x;
  a.wf1 = (const bf16*)wf1;
  a.wf2 = (const bf16*)wf2;
  a.bias1 = bias1;
  a.bias2 = bias2;
  a.y = (bf16*)y;
  a.zero = (const bf16*)zero;
  a.stagger = kernel_stagger(kStagBlock);
  const size_t lds = (size_t)2 * kRing * kSlot;  // 148.5 KB
  // PD 6: 5 K steps of weight lookahead (PD 3 and a mid-step DMA measured
  // the same, 116-120 us at B=256); tools/block_bench.py
  hipLaunchKernelGGL((conv3x3_block_kernel<6, 0>), dim3(B), dim3(512), lds, s, a);
  DMLC_HIP_CHECK(hipGetLastError());
}

}  // namespace dmlc
