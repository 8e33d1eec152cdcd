// Direct 3x3 / stride 1 / pad 1 convolution on 13x13 images with the whole
// input image resident in LDS (AlexNet features.6 / .8 / .10: 13x13x192 ->
// 384, 384 -> 256, 256 -> 256), bias (+ ReLU), bf16 NHWC in and out.
//
// Reference equivalent: those Conv2d + ReLU modules of tch::vision::alexnet,
// run per query by `forward_t` (src/services.rs:493). As implicit-GEMM tiles
// (conv_igemm.hip, 128x128) every tile re-gathers its 3x3 windows through L2
// and the three convs ran at 680-870 TFLOP/s (66 / 105 / 75 us at B=256,
// profiles/r3_alexnet_ops_blaslt.txt). Here one workgroup = one image:
//
//  * the image (169 pixels, 75-130 KB) goes HBM -> LDS once by LDS-DMA, its
//    16-B chunks XOR-swizzled per pixel (the conv3x3_stream.hip scheme: every
//    16-lane group of a fragment read hits 16 distinct bank slots); pixels are
//    padded to a multiple of 256 B; taps outside the image read one zero pixel;
//  * 4 waves, one per SIMD with up to 512 registers each: a wave owns Cout/4
//    output channels (2 N fragments per 32-channel group, perm32 row order: a
//    lane ends with 8 consecutive channels of one pixel) for all 11 pixel
//    fragments, so each weight fragment feeds 11 MFMAs and each X fragment
//    4-6; the weights stream from L2 in fragment order (stream_frag_index)
//    through a PD-deep register ring, no LDS stage and no barrier in the K
//    loop. (8 waves of 256 registers
//    spilled the ring: the compiler double-buffers the X fragments.)
#include "common.h"
#include "kernels.h"

namespace dmlc {

namespace {

template <int N>
__device__ __forceinline__ void vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}
struct D13Args {
  const bf16* x;      // [B, 13, 13, CI]
  const bf16* wf;     // [CO/32][KT][2][64][8] fragment order (stream_frag_index, K = 9 CI)
  const float* bias;  // [CO]
  bf16* y;            // [B, 13, 13, CO]
  const bf16* zero;   // >= 16 zero bytes
  int relu;
  // fused 3x3/s2 max-pool (AlexNet features.12 after features.10): [B, 6, 6, CO]
  // written instead of y (one pass per wave, ReLU on)
  bf16* ypool;
};

constexpr int kH = 13, kW = 13, kNPix = kH * kW;  // 169
constexpr int kMF = (kNPix + 15) / 16;             // 11 pixel fragments

// chunk swizzle of a staged pixel with key K (its pixel index): >= 256-B
// pixels, as conv3x3_stream.hip's xswz for CPX >= 16
__device__ __forceinline__ int swz13(int K) { return (K & 7) << 1; }

template <int CI>
struct D13Geom {
  static constexpr int CPX = CI / 8;                    // 16-B chunks per pixel
  static constexpr int PXC = (CPX + 15) / 16 * 16;      // padded chunks per staged pixel
  static constexpr int PXB = PXC * 16;                  // bytes per staged pixel
  static constexpr int ZB = kNPix * PXB;                // zero pixel
  static constexpr size_t LDS = (size_t)ZB + PXB;
};

template <int CI, int CO, int PD, int GPP>
__global__ __launch_bounds__(256, 1) void conv3x3_13_kernel(D13Args a) {
  using G = D13Geom<CI>;
  constexpr int CPX = G::CPX, PXC = G::PXC, PXB = G::PXB, ZB = G::ZB;
  constexpr int CT = CI / 32;       // K steps per tap
  constexpr int KT = 9 * CT;        // K steps
  constexpr int NGW = CO / 32 / 4;  // 32-channel groups per wave (4 waves, one per SIMD)
  constexpr int NF = 2 * GPP;       // N fragments per pass (GPP groups: the accumulators of one pass)
  static_assert(NGW % GPP == 0, "passes");
  static_assert(CT % PD == 0, "the weight ring's slot must be a compile-time function of the K step in a tap");
  static_assert(CO % 128 == 0, "channel groups over 4 waves");
  extern __shared__ __attribute__((aligned(16))) uint4 smem[];
  char* xs = (char*)smem;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, g = lane >> 4;
  const int b = blockIdx.x;
  const bf16* img = a.x + (long)b * kNPix * CI;

  // ---- stage the image: physical slot ps = K * PXC + pc holds logical chunk
  // pc ^ swz(K) of pixel K (slots whose logical chunk is past CPX: padding,
  // loaded from the zero page); one LDS-DMA instruction = 64 slots
  constexpr int NSLOT = kNPix * PXC;
  for (int i = wave; i * 64 < NSLOT; i += 4) {
    const int ps = i * 64 + lane;
    if (ps < NSLOT) {
      const int K = ps / PXC, pc = ps - K * PXC;
      const int lc = pc ^ swz13(K);
      dma16(lc < CPX ? (const void*)(img + (long)K * CI + lc * 8) : (const void*)a.zero, xs + i * 1024);
    }
  }
  for (int i = tid; i < PXB / 16; i += 256) ((uint4*)(xs + ZB))[i] = make_uint4(0, 0, 0, 0);

  // ---- per-lane pixel geometry, recomputed per tap (held across the K loop
  // it cost 11 VGPRs the loop needs): p = 16 f + fr (clamped for the padding
  // lanes of the last fragment: they compute a duplicate, never stored)
  int xa[kMF], tsw = 0;
  auto set_tap = [&](int tap) __attribute__((always_inline)) {
    const int kh = tap / 3, kw = tap - kh * 3;
    const int ktap = (kh - 1) * kW + kw - 1;
#pragma unroll
    for (int f = 0; f < kMF; ++f) {
      const int p = min(16 * f + fr, kNPix - 1);
      const int r = (p * 79) >> 10, c = p - r * kW;  // p / 13 for p < 169
      const bool out = (kh == 0 && r == 0) || (kh == 2 && r == kH - 1) || (kw == 0 && c == 0) ||
                       (kw == 2 && c == kW - 1);
      xa[f] = out ? ZB : (p + ktap) * PXB;
    }
    // K = p + ktap with p & 15 == fr for every real pixel: one swizzle per tap
    tsw = (g << 4) ^ (swz13(fr + ktap) << 4);
  };
  auto xread = [&](int f, int cc) __attribute__((always_inline)) {
    return *(const bf16x8*)(xs + xa[f] + (tsw ^ (cc * 64)));
  };

  vm_wait<0>();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();

#pragma nounroll
  for (int pass = 0; pass < NGW / GPP; ++pass) {
    const int grp0 = wave * NGW + pass * GPP;  // first 32-channel group of this pass
    // this pass's groups grp0 .. grp0 + GPP - 1 are consecutive in the
    // fragment-order array: fragment nf (group nf / 2) of K step t at
    // base + ((nf / 2) KT + t) 2 KB + (nf % 2) KB, lane l's 16 B at 16 l;
    // steps past the end re-load step 0 (uniform load counts for the waits)
    // (compiler-visible buffer loads: untracked asm loads into a register
    // ring raced the register allocator at 254 VGPRs -- an in-flight load
    // landed in a reused register and faulted a later address)
    const __amdgpu_buffer_rsrc_t wrs = wave_rsrc(a.wf + (long)grp0 * KT * 2 * 512, GPP * KT * 2 * 1024);
    auto wfetch = [&](int t, bf16x8* dst) __attribute__((always_inline)) {
      const int tt = t < KT ? t : 0;
#pragma unroll
      for (int nf = 0; nf < NF; ++nf)
        dst[nf] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(
                                                 wrs, lane * 16, (nf >> 1) * KT * 2048 + tt * 2048 + (nf & 1) * 1024, 0));
    };
    bf16x8 wq[PD][NF];
#pragma unroll
    for (int t = 0; t < PD - 1; ++t) wfetch(t, wq[t]);
    floatx4 acc[kMF][NF];
#pragma unroll
    for (int f = 0; f < kMF; ++f)
#pragma unroll
      for (int nf = 0; nf < NF; ++nf) acc[f][nf] = floatx4{0.f, 0.f, 0.f, 0.f};
    set_tap(0);
    bf16x8 xf[kMF];
#pragma unroll
    for (int f = 0; f < kMF; ++f) xf[f] = xread(f, 0);
#pragma nounroll
    for (int tap = 0; tap < 9; ++tap) {
#pragma unroll
      for (int cc = 0; cc < CT; ++cc) {
        const int t = tap * CT + cc;
        wfetch(t + PD - 1, wq[(cc + PD - 1) % PD]);
        // next K step's X: same tap at cc + 1, or the next tap's first (the
        // final step re-reads a valid tile, unused)
        if (cc + 1 == CT && tap + 1 < 9) set_tap(tap + 1);
        const int cn = cc + 1 == CT ? 0 : cc + 1;
        // the X fragments (read during the previous step) landed: one wait
        // instead of the compiler's one per fragment
        __builtin_amdgcn_s_waitcnt(0xC07F);
#pragma unroll
        for (int f = 0; f < kMF; ++f) {
#pragma unroll
          for (int nf = 0; nf < NF; ++nf)
            acc[f][nf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wq[cc % PD][nf], xf[f], acc[f][nf], 0, 0, 0);
          xf[f] = xread(f, cn);
        }
#pragma unroll
        for (int f = 0; f < kMF; ++f) {
          __builtin_amdgcn_sched_group_barrier(0x008, NF, 0);
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        }
      }
    }
    // ---- epilogue: lane holds channels 32 grp + 8 g .. +7 of pixel 16 f + fr
    if constexpr (NGW == GPP) {
      if (a.ypool) {
        // fused max-pool: every wave is done with the staged image, so this
        // wave's 169 x 32 GPP-channel output tile goes into its own quarter of
        // that LDS (chunks XOR-swizzled by pixel), then the wave pools its own
        // channels: nothing crosses waves after the barrier
        __syncthreads();
        constexpr int TB = GPP * 64;  // bytes per pixel of a wave's tile
        char* tile = xs + wave * (kNPix * TB);
#pragma unroll
        for (int j = 0; j < GPP; ++j) {
          const int ch = 32 * (grp0 + j) + 8 * g;
          float bs[8];
          {
            const float4 lo = *(const float4*)(a.bias + ch), hi = *(const float4*)(a.bias + ch + 4);
            bs[0] = lo.x, bs[1] = lo.y, bs[2] = lo.z, bs[3] = lo.w, bs[4] = hi.x, bs[5] = hi.y, bs[6] = hi.z,
            bs[7] = hi.w;
          }
#pragma unroll
          for (int f = 0; f < kMF; ++f) {
            const int p = 16 * f + fr;
            if (p < kNPix) {
              float v[8];
#pragma unroll
              for (int e = 0; e < 8; ++e) v[e] = acc[f][2 * j + (e >> 2)][e & 3] + bs[e];
              *(uint4*)(tile + p * TB + (((4 * j + g) ^ (p & (4 * GPP - 1))) << 4)) = relu_bf16x8(pack8(v));
            }
          }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        // 6 x 6 pooled pixels x 4 GPP chunks of 8 channels; post-ReLU bf16 >= 0,
        // so the max is an unsigned 16-bit max
        typedef unsigned short ushort8 __attribute__((ext_vector_type(8)));
        constexpr int NC = 4 * GPP;
        for (int it = lane; it < 36 * NC; it += 64) {
          const int pp = it / NC, c = it - pp * NC;
          const int ph = pp / 6, pw = pp - ph * 6;
          ushort8 m = ushort8{0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
          for (int dy = 0; dy < 3; ++dy)
#pragma unroll
            for (int dx = 0; dx < 3; ++dx) {
              const int q = (2 * ph + dy) * kW + 2 * pw + dx;
              m = __builtin_elementwise_max(m, *(const ushort8*)(tile + q * TB + ((c ^ (q & (NC - 1))) << 4)));
            }
          *(ushort8*)(a.ypool + ((long)b * 36 + pp) * CO + 32 * grp0 + 8 * c) = m;
        }
        continue;
      }
    }
    bf16* yim = a.y + (long)b * kNPix * CO;
#pragma unroll
    for (int j = 0; j < GPP; ++j) {
      const int ch = 32 * (grp0 + j) + 8 * g;
      float bs[8];
      {
        const float4 lo = *(const float4*)(a.bias + ch), hi = *(const float4*)(a.bias + ch + 4);
        bs[0] = lo.x, bs[1] = lo.y, bs[2] = lo.z, bs[3] = lo.w, bs[4] = hi.x, bs[5] = hi.y, bs[6] = hi.z, bs[7] = hi.w;
      }
#pragma unroll
      for (int f = 0; f < kMF; ++f) {
        const int p = 16 * f + fr;
        if (p < kNPix) {
          float v[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            v[e] = acc[f][2 * j + (e >> 2)][e & 3] + bs[e];
          }
          *(uint4*)(yim + (long)p * CO + ch) = pack8_relu(v, a.relu);
        }
      }
    }
  }
}

template <int CI, int CO, int PD, int GPP>
void launch13(const D13Args& a, int B, hipStream_t s) {
  hipLaunchKernelGGL((conv3x3_13_kernel<CI, CO, PD, GPP>), dim3(B), dim3(256), D13Geom<CI>::LDS, s, a);
}

}  // namespace

// the fused max-pool needs one pass per wave (the 256 -> 256 variant)
bool conv3x3_13_pool_supported(int Cin, int Cout) { return Cin == 256 && Cout == 256; }

bool conv3x3_13_supported(int H, int W, int Cin, int Cout) {
  return H == kH && W == kW &&
         ((Cin == 192 && Cout == 384) || (Cin == 384 && Cout == 256) || (Cin == 256 && Cout == 256));
}

void conv3x3_13(const void* x, const void* wf, const float* bias, void* y, const void* zero, int B, int Cin, int Cout,
                bool relu, hipStream_t s, void* ypool) {
  if (B <= 0) return;
  if (!conv3x3_13_supported(kH, kW, Cin, Cout)) throw std::invalid_argument("conv3x3_13: unsupported channels");
  if (!x || !wf || !bias || !y || !zero || (((uintptr_t)x | (uintptr_t)wf | (uintptr_t)y | (uintptr_t)zero) & 15))
    throw std::invalid_argument("conv3x3_13: null / misaligned operand");
  D13Args a;
  a.x = (const bf16*)x;
  a.wf = (const bf16*)wf;
  a.bias = bias;
  a.y = (bf16*)y;
  a.zero = (const bf16*)zero;
  a.relu = relu ? 1 : 0;
  a.ypool = (bf16*)ypool;
  if (ypool && (!relu || !conv3x3_13_pool_supported(Cin, Cout) || ((uintptr_t)ypool & 15)))
    throw std::invalid_argument("conv3x3_13: fused pool needs ReLU, Cin = Cout = 256, aligned output");
  // (ring depth / groups per pass: the largest without spills)
  if (Cin == 192) launch13<192, 384, 3, 1>(a, B, s);
  else if (Cin == 384) launch13<384, 256, 3, 2>(a, B, s);
  else launch13<256, 256, 2, 2>(a, B, s);
  DMLC_HIP_CHECK(hipGetLastError());
}

}  // namespace dmlc
