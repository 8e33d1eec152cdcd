// Direct 5x5 / stride 1 / pad 2 convolution on 27x27x64 images with the
// whole input image resident in LDS (AlexNet features.3: 64 -> 192), bias +
// ReLU, bf16 NHWC in and out.
//
// Reference equivalent: features.3 (Conv2d(64, 192, 5, padding=2)) + ReLU of
// tch::vision::alexnet, run per query by `forward_t` (src/services.rs:493).
// As 256x64 implicit-GEMM tiles it was AlexNet's largest kernel: 146-161 us
// at B=256 (~750 TFLOP/s, profiles/r3_alexnet_direct13.txt), every tile
// re-gathering its 25-tap windows through L2. Here one workgroup = one image,
// the conv3x3_13.hip design with the other split:
//
//  * the image (729 pixels x 128 B = 93 KB) goes HBM -> LDS once by LDS-DMA,
//    16-B chunks swizzled within each pixel (128-B pixels: conv3x3_stream.hip's
//    CPX = 8 scheme, consecutive pixels alternate bank-window halves), taps
//    outside the image read one zero pixel;
//  * 8 waves (2 per SIMD): wave w owns pixel fragments 6w .. 6w+5 (46 real;
//    the last wave's 2 extra duplicate pixel 728 and are never stored) for all
//    192 channels, in 3 passes of 64 channels (4 N fragments: each X fragment
//    read feeds 4 MFMAs, each weight fragment 6; the 8 waves fetch the same
//    weight fragments, mostly L1 hits). (4 waves of 12 fragments at 512
//    registers: accumulators bounced between VGPRs and AGPRs every K step.)
//    weights stream from L2 in fragment order (stream_frag_index, K = 1600)
//    through a 2-deep register ring; no barrier in the K loop.
#include "common.h"
#include "kernels.h"

namespace dmlc {

namespace {

template <int N>
__device__ __forceinline__ void vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}

struct D27Args {
  const bf16* x;      // [B, 27, 27, 64]
  const bf16* wf;     // [6][50][2][64][8] fragment order (stream_frag_index, K = 1600)
  const float* bias;  // [192]
  bf16* y;            // [B, 27, 27, 192]
  const bf16* zero;   // >= 16 zero bytes
  // fused 3x3/s2 max-pool (features.5): [B, 13, 13, 192] written instead of y
  bf16* ypool;
};

constexpr int kH = 27, kW = 27, kNPix = kH * kW;  // 729
constexpr int kCI = 64, kCO = 192, kKS = 5, kPad = 2;
constexpr int kPXB = kCI * 2;                      // 128 B per staged pixel
constexpr int kZB = kNPix * kPXB;                  // zero pixel
constexpr int kTile = kNPix * 64;                  // fused pool: one 32-channel group's output [729][32]
constexpr size_t kLds = (size_t)kZB + kPXB;
constexpr size_t kLdsPool = kLds + kTile;
constexpr int kWaves = 8;                          // 2 per SIMD
constexpr int kFPW = 6;                            // pixel fragments per wave (46 real over 8 waves)
constexpr int kCT = kCI / 32;                      // 2 K steps per tap
constexpr int kKT = kKS * kKS * kCT;               // 50 K steps
constexpr int kGPP = 2;                            // 32-channel groups per pass
constexpr int kNF = 2 * kGPP;                      // N fragments per pass
constexpr int kPD = 2;                             // weight ring depth (divides kCT)

// 128-B pixels: chunk c of pixel K at physical c ^ (((K >> 1) & 3) << 1)
__device__ __forceinline__ int swz27(int K) { return ((K >> 1) & 3) << 1; }

__global__ __launch_bounds__(512, 1) void conv5x5_27_kernel(D27Args a) {
  extern __shared__ __attribute__((aligned(16))) uint4 smem[];
  char* xs = (char*)smem;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, g = lane >> 4;
  const int b = blockIdx.x;
  const bf16* img = a.x + (long)b * kNPix * kCI;

  // ---- stage the image: slot ps = K * 8 + pc holds logical chunk pc ^ swz(K)
  constexpr int NSLOT = kNPix * 8;
  for (int i = wave; i * 64 < NSLOT; i += kWaves) {
    const int ps = i * 64 + lane;
    if (ps < NSLOT) {
      const int K = ps >> 3, pc = ps & 7;
      dma16(img + (long)K * kCI + (pc ^ swz27(K)) * 8, xs + i * 1024);
    }
  }
  if (tid < kPXB / 16) ((uint4*)(xs + kZB))[tid] = make_uint4(0, 0, 0, 0);

  // ---- per-lane fragment constants: p = 16 (FPW w + f) + fr, clamped to the
  // last pixel for padding lanes / fragments (a duplicate, never stored);
  // pix[f] = its staged offset, inm[f] bit tap = the tap's input pixel lies in
  // the image. A tap then costs 3 VALU per fragment (the 5x5 conv changes tap
  // every 2 K steps: recomputing row / column per tap was ~100 unhidden VALU
  // per 48 MFMAs at one wave per SIMD).
  const int f0 = wave * kFPW;
  int pix[kFPW], inm[kFPW];
#pragma unroll
  for (int f = 0; f < kFPW; ++f) {
    const int p = min(16 * (f0 + f) + fr, kNPix - 1);
    const int r = (p * 2428) >> 16, c = p - r * kW;  // p / 27 for p < 768
    int m = 0;
#pragma unroll
    for (int tap = 0; tap < kKS * kKS; ++tap) {
      const int kh = tap / kKS, kw = tap % kKS;
      if ((unsigned)(r + kh - kPad) < (unsigned)kH && (unsigned)(c + kw - kPad) < (unsigned)kW) m |= 1 << tap;
    }
    pix[f] = p * kPXB;
    inm[f] = m;
  }
  int xa[kFPW], tsw = 0;
  auto set_tap = [&](int tap) __attribute__((always_inline)) {
    const int kh = tap / kKS, kw = tap - kh * kKS;
    const int toff = ((kh - kPad) * kW + kw - kPad) * kPXB;
#pragma unroll
    for (int f = 0; f < kFPW; ++f) xa[f] = ((inm[f] >> tap) & 1) ? pix[f] + toff : kZB;
    // K = p + ktap with p & 15 == fr for every real pixel: one swizzle per tap
    tsw = (g << 4) ^ (swz27(fr + (kh - kPad) * kW + kw - kPad) << 4);
  };
  auto xread = [&](int f, int cc) __attribute__((always_inline)) {
    return *(const bf16x8*)(xs + xa[f] + (tsw ^ (cc * 64)));
  };

  vm_wait<0>();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();

#pragma nounroll
  for (int pass = 0; pass < kCO / 32 / kGPP; ++pass) {
    const int grp0 = pass * kGPP;
    const __amdgpu_buffer_rsrc_t wrs = wave_rsrc(a.wf + (long)grp0 * kKT * 2 * 512, kGPP * kKT * 2 * 1024);
    auto wfetch = [&](int t, bf16x8* dst) __attribute__((always_inline)) {
      const int tt = t < kKT ? t : 0;
#pragma unroll
      for (int nf = 0; nf < kNF; ++nf)
        dst[nf] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(
                                                 wrs, lane * 16, (nf >> 1) * kKT * 2048 + tt * 2048 + (nf & 1) * 1024,
                                                 0));
    };
    bf16x8 wq[kPD][kNF];
#pragma unroll
    for (int t = 0; t < kPD - 1; ++t) wfetch(t, wq[t]);
    floatx4 acc[kFPW][kNF];
#pragma unroll
    for (int f = 0; f < kFPW; ++f)
#pragma unroll
      for (int nf = 0; nf < kNF; ++nf) acc[f][nf] = floatx4{0.f, 0.f, 0.f, 0.f};
    set_tap(0);
    bf16x8 xf[kFPW];
#pragma unroll
    for (int f = 0; f < kFPW; ++f) xf[f] = xread(f, 0);
#pragma nounroll
    for (int tap = 0; tap < kKS * kKS; ++tap) {
#pragma unroll
      for (int cc = 0; cc < kCT; ++cc) {
        const int t = tap * kCT + cc;
        wfetch(t + kPD - 1, wq[(cc + kPD - 1) % kPD]);
        if (cc + 1 == kCT && tap + 1 < kKS * kKS) set_tap(tap + 1);
        const int cn = cc + 1 == kCT ? 0 : cc + 1;
        // the X fragments (read during the previous step) landed: one wait
        // instead of the compiler's one per fragment
        __builtin_amdgcn_s_waitcnt(0xC07F);
#pragma unroll
        for (int f = 0; f < kFPW; ++f) {
#pragma unroll
          for (int nf = 0; nf < kNF; ++nf)
            acc[f][nf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wq[cc % kPD][nf], xf[f], acc[f][nf], 0, 0, 0);
          xf[f] = xread(f, cn);
        }
#pragma unroll
        for (int f = 0; f < kFPW; ++f) {
          __builtin_amdgcn_sched_group_barrier(0x008, kNF, 0);
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        }
      }
    }
    // ---- epilogue: lane holds channels 32 grp + 8 g .. +7 of pixel 16 (f0 + f) + fr
    if (a.ypool) {
      // fused max-pool, one 32-channel group at a time through an LDS tile
      // after the staged image ([729][32] bf16, 16-B chunks XOR-swizzled by
      // pixel): every wave writes its pixels, then all 512 threads pool
      typedef unsigned short ushort8 __attribute__((ext_vector_type(8)));
      char* tile = xs + kLds;
#pragma unroll
      for (int j = 0; j < kGPP; ++j) {
        const int ch = 32 * (grp0 + j) + 8 * g;
        float bs[8];
        {
          const float4 lo = *(const float4*)(a.bias + ch), hi = *(const float4*)(a.bias + ch + 4);
          bs[0] = lo.x, bs[1] = lo.y, bs[2] = lo.z, bs[3] = lo.w, bs[4] = hi.x, bs[5] = hi.y, bs[6] = hi.z,
          bs[7] = hi.w;
        }
        __syncthreads();  // the previous group's pooling reads are done
#pragma unroll
        for (int f = 0; f < kFPW; ++f) {
          const int p = 16 * (f0 + f) + fr;
          if (p < kNPix) {
            float v[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] = acc[f][2 * j + (e >> 2)][e & 3] + bs[e];
            *(uint4*)(tile + p * 64 + ((g ^ (p & 3)) << 4)) = relu_bf16x8(pack8(v));
          }
        }
        __syncthreads();
        // 13 x 13 pooled pixels x 4 chunks; post-ReLU bf16 >= 0: unsigned max
        for (int it = threadIdx.x; it < 169 * 4; it += 64 * kWaves) {
          const int pp = it >> 2, c = it & 3;
          const int ph = (pp * 79) >> 10, pw = pp - ph * 13;  // pp / 13 for pp < 169
          ushort8 m = ushort8{0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
          for (int dy = 0; dy < 3; ++dy)
#pragma unroll
            for (int dx = 0; dx < 3; ++dx) {
              const int q = (2 * ph + dy) * kW + 2 * pw + dx;
              m = __builtin_elementwise_max(m, *(const ushort8*)(tile + q * 64 + ((c ^ (q & 3)) << 4)));
            }
          *(ushort8*)(a.ypool + ((long)b * 169 + pp) * kCO + 32 * (grp0 + j) + 8 * c) = m;
        }
      }
      continue;
    }
    bf16* yim = a.y + (long)b * kNPix * kCO;
#pragma unroll
    for (int j = 0; j < kGPP; ++j) {
      const int ch = 32 * (grp0 + j) + 8 * g;
      float bs[8];
      {
        const float4 lo = *(const float4*)(a.bias + ch), hi = *(const float4*)(a.bias + ch + 4);
        bs[0] = lo.x, bs[1] = lo.y, bs[2] = lo.z, bs[3] = lo.w, bs[4] = hi.x, bs[5] = hi.y, bs[6] = hi.z, bs[7] = hi.w;
      }
#pragma unroll
      for (int f = 0; f < kFPW; ++f) {
        const int p = 16 * (f0 + f) + fr;
        if (p < kNPix) {
          float v[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = acc[f][2 * j + (e >> 2)][e & 3] + bs[e];
          *(uint4*)(yim + (long)p * kCO + ch) = relu_bf16x8(pack8(v));
        }
      }
    }
  }
}

}  // namespace

bool conv5x5_27_supported(int H, int W, int Cin, int Cout, int pad) {
  return H == kH && W == kW && Cin == kCI && Cout == kCO && pad == kPad;
}

void conv5x5_27(const void* x, const void* wf, const float* bias, void* y, const void* zero, int B, hipStream_t s,
                void* ypool) {
  if (B <= 0) return;
  if (!x || !wf || !bias || !y || !zero || (((uintptr_t)x | (uintptr_t)wf | (uintptr_t)y | (uintptr_t)zero) & 15))
    throw std::invalid_argument("conv5x5_27: null / misaligned operand");
  D27Args a;
  a.x = (const bf16*)x;
  a.wf = (const bf16*)wf;
  a.bias = bias;
  a.y = (bf16*)y;
  a.zero = (const bf16*)zero;
  a.ypool = (bf16*)ypool;
  if ((uintptr_t)ypool & 15) throw std::invalid_argument("conv5x5_27: misaligned pooled output");
  hipLaunchKernelGGL(conv5x5_27_kernel, dim3(B), dim3(64 * kWaves), ypool ? kLdsPool : kLds, s, a);
  DMLC_HIP_CHECK(hipGetLastError());
}

}  // namespace dmlc
