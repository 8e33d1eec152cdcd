// Fused ResNet50 identity bottleneck for layer1 (resnet50_fp8: layer1.1 and
// layer1.2), 56x56x256 e4m3 in and out:
//   t1 = relu(bn1(conv1x1 256->64 (x)))          e4m3 MFMA, t1 bf16 in LDS
//   t2 = relu(bn2(conv3x3 64->64 (t1)))          bf16 MFMA, t2 bf16 in LDS
//   y  = relu(bn3(conv1x1 64->256 (t2)) + x)     bf16 MFMA, y e4m3
// in ONE kernel: x is read once (conv1 operand, then the residual as an L2
// hit), y written once, and the two 64-channel intermediates never leave LDS.
//
// Reference equivalent: torchvision Bottleneck.forward (conv1/bn1/relu,
// conv2/bn2/relu, conv3/bn3, += identity, relu) of tch::vision::resnet50, run
// per query by `forward_t` (src/services.rs:493; BASELINE config 5). As three
// conv1x1 / conv3x3 launches one layer1 block moved ~1.6 GB at B=256 (the
// 256-channel input read twice, the 64-channel intermediates written and read
// back) and took ~245 us (profiles/r2_resnet50_fp8_ops_conv1x1.txt); fused it
// moves ~0.4 GB.
//
// One workgroup = one image, 8 waves in two roles, 4 output rows (224
// pixels = 14 pixel fragments of 16) per step; the schedule is at the kernel
// (two workgroup barriers per step):
//  * compute waves 0-3 (tile half wm, channel half wn): conv1 -> t1 rows
//    4k+1 .. 4k+4 (a 6-row LDS ring; rows -1 and 56 are conv2's zero
//    padding) from x rows staged in LDS, then conv2 over t1 rows 4k-1 .. 4k+4
//    -> t2 (two LDS buffers); conv1 weights in registers, conv2 weights
//    through a register ring (their only global loads);
//  * memory waves 4-7 (tile half, 128-channel half): the LDS-DMA of the
//    next step's x rows, conv3 of the previous step's t2 with the weights in
//    registers, + residual (loaded a step ahead) -> y stores, 16 channels
//    per lane (16-B e4m3 accesses).
// A memory wave shares its SIMD with a compute wave, and its vmcnt queue is
// its own: the compute waves never wait behind a store.
//
// History (tools/bottleneck_bench.py, B = 256, same-box resnet50_fp8 bench;
// profiles/r3_bottleneck_v2.txt, profiles/r3_bottleneck_v3.txt):
//  v1: every wave all three convs, x / weights / constants loaded from
//      HBM/L2 in the phase that used them, behind the previous stores:
//      257-273 us per block (111 us with every memory access knocked out),
//      at parity with the three unfused kernels;
//  v2: x staged by DMA a step ahead, weights and constants on chip:
//      193-210 us (+3% img/s with the fused kernel on);
//  v3: the two roles, 16-B residual / y accesses, residual a step ahead:
//      156-177 us; resnet50_fp8 103.2k -> 109.5-109.8k img/s fused.
#include "common.h"
#include "kernels.h"

#include <type_traits>

namespace dmlc {

namespace {

typedef int v8i __attribute__((ext_vector_type(8)));

struct BnArgs {
  const uint8_t* x;    // [B, 56, 56, 256] e4m3 (value = e4m3 * res_scale)
  const uint8_t* w1;   // [64][256] e4m3 (per-row scales folded into a1)
  const float* a1;     // [64] s_x * s_w1[n]
  const float* b1;     // [64]
  const bf16* wf2;     // conv2 weights, fragment order [2][18][2][64][8] (stream_frag_index, K = 576)
  const float* b2;     // [64]
  const bf16* wf3;     // conv3 weights, fragment order [8][2][2][64][8] (K = 64)
  const float* b3;     // [256]
  uint8_t* y;          // [B, 56, 56, 256] e4m3
  float res_scale;     // s_x
  float out_inv_scale; // 1 / s_y
  int stagger;         // start_stagger (common.h)
};

constexpr int kH = 56, kW = 56, kC = 256, kM = 64;
constexpr int kR = 4;                    // output rows per step
constexpr int kPix = kR * kW;            // 224 pixels per step
constexpr int kSteps = kH / kR;          // 14
constexpr int kMF = kPix / 32;           // 7 pixel fragments per wave (half a step)
constexpr int kHalf = (kW + 2) * 64;     // t1 slot: one 32-channel half, 58 columns x 64 B = 3712 B
constexpr int kSlot = 2 * kHalf;         // 7424 B per t1 row
constexpr int kRing = 6;                 // t1 rows 4k-1 .. 4k+4
constexpr int kT2 = kPix * kM * 2;       // 28672 B per t2 buffer (two)
constexpr int kXB = kPix * kC;           // 57344 B: conv1's 4 x rows (e4m3)
constexpr int kKS2 = 9 * kM / 32;        // 18 conv2 K steps
constexpr int kPD = 3;                   // conv2 weight register ring depth (divides kKS2)
constexpr int kXDma = kXB / 1024 / 4;    // 14 LDS-DMA instructions per memory wave per step
constexpr int kCst = 7 * kM * 4;         // a1, b1, b2 (64 floats each), b3 (256): 1792 B
constexpr int kST = kMF * 2;             // y stores per memory wave per step
constexpr size_t kLds = (size_t)kRing * kSlot + 2 * kT2 + kXB + kCst;  // 161024 B
static_assert(kLds <= 160 * 1024, "LDS budget");

template <int N>
__device__ __forceinline__ void vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
}

// values already within +-448
__device__ __forceinline__ uint32_t f32x4_to_fp8_sat(const float* f) {
  int v = __builtin_amdgcn_cvt_pk_fp8_f32(f[0], f[1], 0, false);
  v = __builtin_amdgcn_cvt_pk_fp8_f32(f[2], f[3], v, true);
  return (uint32_t)v;
}
__device__ __forceinline__ uint32_t f32x4_to_fp8(const float* f) {
  float c[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) c[i] = fminf(fmaxf(f[i], -448.f), 448.f);
  int v = __builtin_amdgcn_cvt_pk_fp8_f32(c[0], c[1], 0, false);
  v = __builtin_amdgcn_cvt_pk_fp8_f32(c[2], c[3], v, true);
  return (uint32_t)v;
}

__device__ __forceinline__ void fp8x4_to_f32(uint32_t u, float* f) {
  e4m3x4_to_f32(u, f);
}

// 16-B global load the compiler does not track: its wait is the kernel's own
// (counted vm_wait + pin), so no compiler wait lands behind a later DMA
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ u32x4 gload16(const void* p) {
  u32x4 v;
  asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(v) : "v"(p) : "memory");
  return v;
}
template <typename T>
__device__ __forceinline__ void pin(T& v) {
  asm volatile("" : "+v"(v));
}

__device__ __forceinline__ void load8(const float* p, float* v) {
  const float4 lo = *(const float4*)p, h4 = *(const float4*)(p + 4);
  v[0] = lo.x, v[1] = lo.y, v[2] = lo.z, v[3] = lo.w, v[4] = h4.x, v[5] = h4.y, v[6] = h4.z, v[7] = h4.w;
}

// t1 ring address of (staged column q, channel half h, 16-B chunk g): the
// conv3x3_block.hip layout (chunk c of (h, q) holds channels
// 8 (4h + (c ^ ((q >> 1) & 3))); pad columns q = 0, 57 stay zero)
__device__ __forceinline__ int t1_off(int q, int h, int g) { return h * kHalf + q * 64 + ((g ^ ((q >> 1) & 3)) << 4); }
// t2: pixel p's 8 chunks of 8 channels, chunk c at physical c ^ ((p >> 1) & 7)
// (every 16-lane group of a fragment read hits 16 distinct bank slots)
__device__ __forceinline__ int t2_off(int p, int c) { return p * 128 + ((c ^ ((p >> 1) & 7)) << 4); }
// x staging buffer: tile pixel p's 16 chunks of 16 channels, chunk c at
// physical c ^ (p & 15) (a fragment's 16 pixels, p & 15 = lane row: every
// 16-lane group of a ds_read_b128 covers the 16 chunk slots of a bank row)
__device__ __forceinline__ int xb_off(int p, int c) { return p * 256 + ((c ^ (p & 15)) << 4); }
// head kernel (bf16 64-channel x, 128-B rows): chunk c of pixel p at physical
// c ^ (p & 7) (conv1x1.hip's 128-B bf16 layout, tests/test_layouts_cpu.py)
__device__ __forceinline__ int xb_off_ds(int p, int c) { return p * 128 + ((c ^ (p & 7)) << 4); }

// Lane geometry shared by both roles: wave half wm owns the step's tile
// pixels 112 wm .. 112 wm + 111 (tile rows 2 wm, 2 wm + 1) as fragments
// f = 0..6, lane pixel p = 112 wm + 16 f + fr in tile row 2 wm + bit f of hi.
struct Geo {
  int col[kMF];
  int hi;
  __device__ __forceinline__ Geo(int wm, int fr) {
    hi = 0;
#pragma unroll
    for (int f = 0; f < kMF; ++f) {
      const int q = 16 * f + fr;  // pixel within the half tile
      col[f] = (112 * wm + q) % kW;
      hi |= (q / kW) << f;
    }
  }
};

// ---- compute role (waves 0-3: wave cw = 2 wm + wn): conv1 -> t1 ring,
// conv2 -> t2, on tile half wm and channel half wn (32 channels, perm32
// rows). Its only global loads are the conv2 weight ring's (no store ever
// sits in front of them in its vmcnt queue).
template <bool DS = false>
struct Compute {
  const BnArgs& a;
  char* ring;
  const char* xb;
  const float* cst;
  int wm, wn, fr, g, lane;
  Geo geo;
  // conv1 weights, resident: lane (rr, g) of fragment nf holds channel 32 wn +
  // perm32(16 nf + rr), k = 128 ks + 32 g .. +32 (e4m3) / DS: 32 ks + 8 g .. +8 (bf16)
  typename std::conditional<DS, bf16x8, v8i>::type w1f[2][2];
  bf16x8 wq[kPD][2];
  __amdgpu_buffer_rsrc_t w2rs;

  __device__ __forceinline__ Compute(const BnArgs& a_, char* ring_, const char* xb_, const float* cst_, int cw, int lane_)
      : a(a_), ring(ring_), xb(xb_), cst(cst_), wm(cw >> 1), wn(cw & 1), fr(lane_ & 15), g(lane_ >> 4), lane(lane_),
        geo(cw >> 1, lane_ & 15) {
#pragma unroll
    for (int nf = 0; nf < 2; ++nf) {
      const int ch = 32 * wn + 8 * (fr >> 2) + 4 * nf + (fr & 3);
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        if constexpr (DS) {
          w1f[nf][ks] = *(const bf16x8*)(a.w1 + (ch * kM + ks * 32 + g * 8) * 2);
        } else {
          const uint4 lo = *(const uint4*)(a.w1 + ch * kC + ks * 128 + g * 32);
          const uint4 h4 = *(const uint4*)(a.w1 + ch * kC + ks * 128 + g * 32 + 16);
          w1f[nf][ks] = v8i{(int)lo.x, (int)lo.y, (int)lo.z, (int)lo.w, (int)h4.x, (int)h4.y, (int)h4.z, (int)h4.w};
        }
      }
    }
    w2rs = wave_rsrc(a.wf2 + (long)wn * kKS2 * 2 * 512, kKS2 * 2 * 1024);
#pragma unroll
    for (int ks = 0; ks < kPD - 1; ++ks)
#pragma unroll
      for (int nf = 0; nf < 2; ++nf) wq[ks][nf] = w2load(ks * 2 + nf);
  }
  __device__ __forceinline__ bf16x8 w2load(int kf) {
    return __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(w2rs, lane * 16, kf * 1024, 0));
  }

  // t1 rows 4j+1 .. 4j+4 (rows outside the image: zeros) from the staged x rows
  __device__ __forceinline__ void conv1(int j) {
    float a1v[8], b1v[8];
    load8(cst + 32 * wn + 8 * g, a1v);
    load8(cst + kM + 32 * wn + 8 * g, b1v);
#pragma unroll
    for (int f = 0; f < kMF; ++f) {
      const int p = 112 * wm + 16 * f + fr;
      floatx4 acc[2] = {floatx4{0.f, 0.f, 0.f, 0.f}, floatx4{0.f, 0.f, 0.f, 0.f}};
      if constexpr (DS) {
        bf16x8 xv[2];
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) xv[ks] = *(const bf16x8*)(xb + xb_off_ds(p, 4 * ks + g));
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
          for (int nf = 0; nf < 2; ++nf)
            acc[nf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w1f[nf][ks], xv[ks], acc[nf], 0, 0, 0);
      } else {
        v8i xv[2];
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          const uint4 lo = *(const uint4*)(xb + xb_off(p, 8 * ks + 2 * g));
          const uint4 h4 = *(const uint4*)(xb + xb_off(p, 8 * ks + 2 * g + 1));
          xv[ks] = v8i{(int)lo.x, (int)lo.y, (int)lo.z, (int)lo.w, (int)h4.x, (int)h4.y, (int)h4.z, (int)h4.w};
        }
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
          for (int nf = 0; nf < 2; ++nf)
            acc[nf] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(w1f[nf][ks], xv[ks], acc[nf], 0, 0, 0, 127, 0,
                                                                       127);
      }
      const int r = 4 * j + 1 + 2 * wm + ((geo.hi >> f) & 1);
      const bool outside = (unsigned)r >= (unsigned)kH;
      // scale + bias as v_pk_fma_f32 on channel pairs, ReLU on the packed
      // bf16 (relu_bf16x8), rows outside the image zeroed on the packed words
      float v[8];
#pragma unroll
      for (int e = 0; e < 8; e += 2) {
        const f32x2 q = __builtin_elementwise_fma(f32x2{acc[e >> 2][e & 3], acc[e >> 2][(e & 3) + 1]},
                                                  f32x2{a1v[e], a1v[e + 1]}, f32x2{b1v[e], b1v[e + 1]});
        v[e] = q.x;
        v[e + 1] = q.y;
      }
      const uint4 pk = relu_bf16x8(pack8(v));
      *(uint4*)(ring + ((r + kRing) % kRing) * kSlot + t1_off(geo.col[f] + 1, wn, g)) =
          outside ? make_uint4(0, 0, 0, 0) : pk;
    }
  }

  // conv2 over t1 rows 4k-1 .. 4k+4 -> t2 buffer
  __device__ __forceinline__ void conv2(int k, char* t2) {
    // slot byte offsets of t1 rows 4k-1+i (wave-uniform; named scalars, not
    // an array: a per-lane select between array elements becomes a
    // dynamically indexed private array in scratch)
    const int s0 = ((4 * k - 1 + kRing) % kRing) * kSlot;
    auto sl = [&](int i) __attribute__((always_inline)) {  // i compile time
      const int v = s0 + i * kSlot;
      return v >= kRing * kSlot ? v - kRing * kSlot : v;
    };
    // the bias is the accumulators' starting value; ReLU on the packed bf16
    float b2v[8];
    load8(cst + 2 * kM + 32 * wn + 8 * g, b2v);
    floatx4 acc[kMF][2];
#pragma unroll
    for (int f = 0; f < kMF; ++f) {
      acc[f][0] = floatx4{b2v[0], b2v[1], b2v[2], b2v[3]};
      acc[f][1] = floatx4{b2v[4], b2v[5], b2v[6], b2v[7]};
    }
    bf16x8 xc[kMF], xn[kMF];
    auto load_k = [&](int ks, bf16x8* xd) __attribute__((always_inline)) {
      const int tap = ks >> 1, h = ks & 1;
      const int kh = tap / 3, kw = tap % 3;
#pragma unroll
      for (int f = 0; f < kMF; ++f) {
        const int so = ((geo.hi >> f) & 1) ? sl(2 * wm + kh + 1) : sl(2 * wm + kh);
        xd[f] = *(const bf16x8*)(ring + so + t1_off(geo.col[f] + kw, h, g));
      }
    };
    load_k(0, xc);
#pragma unroll
    for (int ks = 0; ks < kKS2; ++ks) {
      if (ks + 1 < kKS2) load_k(ks + 1, xn);
      {  // K step ks + PD - 1, wrapping into the next step's first ones
        const int kl = (ks + kPD - 1) % kKS2;
#pragma unroll
        for (int nf = 0; nf < 2; ++nf) wq[(ks + kPD - 1) % kPD][nf] = w2load(kl * 2 + nf);
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int f = 0; f < kMF; ++f)
#pragma unroll
        for (int nf = 0; nf < 2; ++nf)
          acc[f][nf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wq[ks % kPD][nf], xc[f], acc[f][nf], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
      if (ks + 1 < kKS2) {
#pragma unroll
        for (int f = 0; f < kMF; ++f) xc[f] = xn[f];
      }
    }
#pragma unroll
    for (int f = 0; f < kMF; ++f) {
      float v[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = acc[f][e >> 2][e & 3];
      *(uint4*)(t2 + t2_off(112 * wm + 16 * f + fr, 4 * wn + g)) = relu_bf16x8(pack8(v));
    }
  }
};

// ---- memory role (waves 4-7: wave mw = 2 wm + cb): the x-row DMA, the
// residual loads, conv3 (t2 of tile half wm -> 128 channels 128 cb .. +127,
// weights resident) and the y stores. Its vmcnt queue per step: residual
// loads, then the DMA, then the stores.
struct Memory {
  const BnArgs& a;
  char* xb;
  const float* cst;
  int mw, wm, cb, fr, g, lane;
  Geo geo;
  const uint8_t* xim;
  uint8_t* yim;
  uint32_t xvoff;
  bf16x8 w3[2][2][4];  // [channel pair-pass P][ks][nf]: channels 128 cb + 64 P .. +63

  __device__ __forceinline__ Memory(const BnArgs& a_, char* xb_, const float* cst_, int mw_, int lane_)
      : a(a_), xb(xb_), cst(cst_), mw(mw_), wm(mw_ >> 1), cb(mw_ & 1), fr(lane_ & 15), g(lane_ >> 4), lane(lane_),
        geo(mw_ >> 1, lane_ & 15) {
    xim = a.x + (long)blockIdx.x * kH * kW * kC;
    yim = a.y + (long)blockIdx.x * kH * kW * kC;
    // DMA instruction i = mw + 4d covers tile pixels 4i .. 4i+3 (one image
    // row: 56 % 4 == 0); lane: pixel 4i + (lane >> 4), physical chunk
    // lane & 15 = logical chunk (lane & 15) ^ ((4i + (lane >> 4)) & 15),
    // (4i) & 15 = (4 mw) & 15 for every d
    xvoff = (uint32_t)((lane >> 4) * kC + 16 * ((lane & 15) ^ ((4 * mw + (lane >> 4)) & 15)));
    // conv3 weights in the perm64 row order: row r of N fragment nf of
    // channel pair-pass P is channel 128 cb + 64 P + 16 (r >> 2) + 4 nf +
    // (r & 3), so a lane's 16 accumulators are 16 consecutive channels (16-B
    // e4m3 residual loads and y stores, 64 B per pixel per wave instruction).
    // Gathered from the perm32 fragment-order array (wf3: channel 8 (r' >> 2)
    // + 4 nf' + (r' & 3) of a 32-channel group at lane r' + 16 k-group).
#pragma unroll
    for (int P = 0; P < 2; ++P)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int nf = 0; nf < 4; ++nf) {
          const int c = 128 * cb + 64 * P + 16 * (fr >> 2) + 4 * nf + (fr & 3);
          const int grp = c >> 5, cc = c & 31;
          const int r0 = 4 * (cc >> 3) + (cc & 3), nf0 = (cc >> 2) & 1;
          w3[P][ks][nf] =
              *(const bf16x8*)((const char*)a.wf3 + ((grp * 2 + ks) * 2 + nf0) * 1024 + ((g << 4) | r0) * 16);
        }
    // 1 / s_y folded into the conv3 weights once (re-rounded to bf16), and
    // the bias (x 1 / s_y) is the MFMAs' accumulator input: an output value
    // is then one fma (the residual), one med3 and a quarter of a packed
    // convert, where it was two fma (conv3 is K = 64: its epilogue is most
    // of the kernel's VALU, which shares the SIMDs with the compute waves)
    const float inv = a.out_inv_scale;
#pragma unroll
    for (int P = 0; P < 2; ++P)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int nf = 0; nf < 4; ++nf) {
          float wv[8];
          unpack8(__builtin_bit_cast(uint4, w3[P][ks][nf]), wv);
#pragma unroll
          for (int e = 0; e < 8; ++e) wv[e] *= inv;
          w3[P][ks][nf] = __builtin_bit_cast(bf16x8, pack8(wv));
        }
  }

  // x rows 4j+1 .. 4j+4 (clamped into the image: rows outside it feed t1
  // rows that are written as zeros) -> staging buffer
  __device__ __forceinline__ void dma_x(int j) {
#pragma unroll
    for (int d = 0; d < kXDma; ++d) {
      const int i = mw + 4 * d, p0 = 4 * i;
      const int r = min(max(4 * j + 1 + p0 / kW, 0), kH - 1);
      const int off = __builtin_amdgcn_readfirstlane((r * kW + p0 % kW) * kC);
      dma16s(xim + off, xvoff, xb + i * 1024);
    }
  }

  __device__ __forceinline__ int pix(int k, int f) const {  // byte offset of fragment f's lane pixel, output rows 4k..
    return ((4 * k + 2 * wm + ((geo.hi >> f) & 1)) * kW + geo.col[f]) * kC;
  }

  u32x4 rv[kMF][2];  // residual of the next conv3 (loaded a step ahead)
  static constexpr int kRL = kMF * 2;  // residual loads per step

  // the residual of y rows 4k .. 4k+3 (16 channels per lane and pair-pass)
  __device__ __forceinline__ void load_rv(int k) {
#pragma unroll
    for (int f = 0; f < kMF; ++f)
#pragma unroll
      for (int P = 0; P < 2; ++P) rv[f][P] = gload16(xim + pix(k, f) + 128 * cb + 64 * P + 16 * g);
  }

  // conv3 over t2 -> y rows 4k .. 4k+3 (its residual landed: the caller's wait)
  __device__ __forceinline__ void conv3(int k, const char* t2) {
#pragma unroll
    for (int f = 0; f < kMF; ++f)
#pragma unroll
      for (int P = 0; P < 2; ++P) pin(rv[f][P]);
#pragma unroll
    for (int P = 0; P < 2; ++P) {
      const int c3 = 128 * cb + 64 * P + 16 * g;  // this lane's 16 channels
      // 1 / s_y folded into the weights (constructor), the bias and the
      // residual scale: an output value is one fma, one med3 (ReLU and the
      // e4m3 saturation) and a quarter of a packed convert
      const float inv = a.out_inv_scale, rsi = a.res_scale * inv;
      float b3v[16];
      load8(cst + 3 * kM + c3, b3v);
      load8(cst + 3 * kM + c3 + 8, b3v + 8);
#pragma unroll
      for (int e = 0; e < 16; ++e) b3v[e] *= inv;
#pragma unroll
      for (int f = 0; f < kMF; ++f) {
        const int p = 112 * wm + 16 * f + fr;
        bf16x8 xt[2];
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) xt[ks] = *(const bf16x8*)(t2 + t2_off(p, 4 * ks + g));
        floatx4 acc[4];
#pragma unroll
        for (int nf = 0; nf < 4; ++nf)
          acc[nf] = floatx4{b3v[4 * nf], b3v[4 * nf + 1], b3v[4 * nf + 2], b3v[4 * nf + 3]};
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
          for (int nf = 0; nf < 4; ++nf)
            acc[nf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w3[P][ks][nf], xt[ks], acc[nf], 0, 0, 0);
        const uint32_t rw[4] = {rv[f][P].x, rv[f][P].y, rv[f][P].z, rv[f][P].w};
        uint32_t q[4];
#pragma unroll
        for (int h = 0; h < 4; ++h) {  // channels c3 + 4h .. +3 = acc[h]
          float v[4], rf[4];
          fp8x4_to_f32(rw[h], rf);
#pragma unroll
          for (int i = 0; i < 4; i += 2) {  // the residual as v_pk_fma_f32
            const f32x2 q = __builtin_elementwise_fma(f32x2{rf[i], rf[i + 1]}, f32x2{rsi, rsi},
                                                      f32x2{acc[h][i], acc[h][i + 1]});
            v[i] = __builtin_amdgcn_fmed3f(q.x, 0.f, 448.f);
            v[i + 1] = __builtin_amdgcn_fmed3f(q.y, 0.f, 448.f);
          }
          q[h] = f32x4_to_fp8_sat(v);
        }
        // non-temporal y stores (L2 kept for the x re-reads)
        __builtin_nontemporal_store(u32x4{q[0], q[1], q[2], q[3]}, (u32x4*)(yim + pix(k, f) + c3));
      }
    }
  }
};

// Step k = 0 .. 14, two workgroup barriers each (S1 mid-step, S2 at the end):
//   compute: conv1(k) [x rows staged during step k-1]  | S1 | conv2(k) -> t2[k & 1] | S2
//   memory:                                           | S1 | residual loads, DMA of
//            conv1(k+1)'s x rows, conv3(k-1) over t2[(k-1) & 1], y stores, wait for the DMA | S2
// The x buffer is read before S1 and written after it; the two t2 buffers
// alternate; t1 rows written by conv1(k+1) replace rows conv2(k) finished
// with before S2.
__global__ __launch_bounds__(512, 1) void bottleneck56_kernel(BnArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint4 smem[];
  char* ring = (char*)smem;
  char* t2 = ring + kRing * kSlot;  // two buffers of kT2
  char* xb = t2 + 2 * kT2;
  float* cst = (float*)(xb + kXB);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  start_stagger(a.stagger);
  // zero the t1 ring (its pad columns stay zero for the whole kernel); the
  // per-channel constants -> LDS
  for (int i = tid; i < kRing * kSlot / 16; i += 512) ((uint4*)ring)[i] = make_uint4(0, 0, 0, 0);
  if (tid < kM) {
    cst[tid] = a.a1[tid];
    cst[kM + tid] = a.b1[tid];
    cst[2 * kM + tid] = a.b2[tid];
  }
  if (tid < 4 * kM) cst[3 * kM + tid] = a.b3[tid];
  if (wave < 4) {
    Compute<> c(a, ring, xb, cst, wave, lane);
    lds_barrier();  // B0: x rows of conv1(-1) staged (memory waves)
    c.conv1(-1);
    lds_barrier();  // B1
    lds_barrier();  // B2: x rows of conv1(0) staged
    for (int k = 0; k <= kSteps; ++k) {
      if (k < kSteps) c.conv1(k);
      lds_barrier();  // S1
      if (k < kSteps) c.conv2(k, t2 + (k & 1) * kT2);
      lds_barrier();  // S2
    }
  } else {
    Memory m(a, xb, cst, wave - 4, lane);
    m.dma_x(-1);
    vm_wait<0>();
    lds_barrier();  // B0
    lds_barrier();  // B1: conv1(-1) is done with the x buffer
    m.dma_x(0);
    vm_wait<0>();
    lds_barrier();  // B2
    for (int k = 0; k <= kSteps; ++k) {
      lds_barrier();  // S1: conv1(k) is done with the x buffer
      // vmcnt queue of a step: [this step's residual, loaded last step]
      // [DMA of conv1(k+1)'s x rows] [conv3(k-1)'s stores] [next residual]
      const bool dma = k + 1 < kSteps;
      if (dma) m.dma_x(k + 1);
      if (k >= 1) {
        if (dma) vm_wait<kXDma>();  // the residual (older than the DMA)
        else vm_wait<0>();
        m.conv3(k - 1, t2 + ((k - 1) & 1) * kT2);
      }
      if (k < kSteps) m.load_rv(k);
      if (dma) {  // the DMA has landed (the stores and the next residual may be in flight)
        if (k >= 1) vm_wait<kST + Memory::kRL>();
        else vm_wait<Memory::kRL>();
      }
      lds_barrier();  // S2
    }
    vm_wait<0>();  // no LDS-DMA may outlive the workgroup
  }
}


// ---- ResNet50 layer1.0's reduce + 3x3 convs as one kernel ("head"): x bf16
// [B,56,56,64] (the stem's output), t1 = relu(conv1x1 64->64 (x) + b1) and
// t2 = relu(conv3x3 64->64 (t1) + b2) with t1 in LDS, t2 (bf16 [B,56,56,64])
// stored for the block's expand conv (conv1x1.hip with the downsample as its
// second K block). The compute waves are bottleneck56's (bf16 conv1); the
// memory waves DMA the next step's x rows (128-B pixels, 8 per instruction)
// and copy the previous step's t2 from LDS to memory. Saves t1's round trip
// through HBM (2 x 103 MB at B = 256) and a launch.
constexpr int kXBh = kPix * kM * 2;         // 28672 B: 4 x rows of 64 bf16 channels
constexpr int kXDmah = kXBh / 1024 / 4;     // 7 LDS-DMA instructions per memory wave per step
constexpr int kSTh = kPix * 8 / 256;        // 7 t2 chunks (16 B) per memory lane per step
constexpr size_t kLdsH = (size_t)kRing * kSlot + 2 * kT2 + kXBh + kCst;  // 132352 B

struct HeadMemory {
  const BnArgs& a;
  char* xb;
  int mw, lane;
  const uint8_t* xim;
  uint8_t* yim;
  uint32_t xvoff;
  __device__ __forceinline__ HeadMemory(const BnArgs& a_, char* xb_, int mw_, int lane_)
      : a(a_), xb(xb_), mw(mw_), lane(lane_) {
    xim = a.x + (long)blockIdx.x * kH * kW * kM * 2;
    yim = a.y + (long)blockIdx.x * kH * kW * kM * 2;
    // instruction i covers pixels 8i .. 8i+7 of one image row (56 % 8 == 0);
    // lane: pixel 8i + (lane >> 3), physical chunk lane & 7 = logical
    // (lane & 7) ^ (lane >> 3)
    xvoff = (uint32_t)((lane >> 3) * 128 + 16 * ((lane & 7) ^ (lane >> 3)));
  }
  __device__ __forceinline__ void dma_x(int j) {  // x rows 4j+1 .. 4j+4 (clamped)
#pragma unroll
    for (int d = 0; d < kXDmah; ++d) {
      const int i = mw + 4 * d, p0 = 8 * i;
      const int r = min(max(4 * j + 1 + p0 / kW, 0), kH - 1);
      const int off = __builtin_amdgcn_readfirstlane((r * kW + p0 % kW) * 128);
      dma16s(xim + off, xvoff, xb + i * 1024);
    }
  }
  // t2 of output rows 4k .. 4k+3 (LDS, swizzled) -> y
  __device__ __forceinline__ void copy_t2(int k, const char* t2) {
#pragma unroll
    for (int i = 0; i < kSTh; ++i) {
      const int id = (i * 4 + mw) * 64 + lane;
      const int p = id >> 3, c = id & 7;
      const uint4 v = *(const uint4*)(t2 + t2_off(p, c));
      *(uint4*)(yim + ((4 * k + p / kW) * kW + p % kW) * 128 + c * 16) = v;
    }
  }
};

__global__ __launch_bounds__(512, 1) void bottleneck56_head_kernel(BnArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint4 smem[];
  char* ring = (char*)smem;
  char* t2 = ring + kRing * kSlot;  // two buffers of kT2
  char* xb = t2 + 2 * kT2;
  float* cst = (float*)(xb + kXBh);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  start_stagger(a.stagger);
  for (int i = tid; i < kRing * kSlot / 16; i += 512) ((uint4*)ring)[i] = make_uint4(0, 0, 0, 0);
  if (tid < kM) {
    cst[tid] = 1.f;  // (no conv1 alpha: bf16 weights carry the BN scale)
    cst[kM + tid] = a.b1[tid];
    cst[2 * kM + tid] = a.b2[tid];
  }
  if (wave < 4) {
    Compute<true> c(a, ring, xb, cst, wave, lane);
    lds_barrier();  // B0: x rows of conv1(-1) staged
    c.conv1(-1);
    lds_barrier();  // B1
    lds_barrier();  // B2: x rows of conv1(0) staged
    for (int k = 0; k <= kSteps; ++k) {
      if (k < kSteps) c.conv1(k);
      lds_barrier();  // S1
      if (k < kSteps) c.conv2(k, t2 + (k & 1) * kT2);
      lds_barrier();  // S2
    }
  } else {
    HeadMemory m(a, xb, wave - 4, lane);
    m.dma_x(-1);
    vm_wait<0>();
    lds_barrier();  // B0
    lds_barrier();  // B1: conv1(-1) is done with the x buffer
    m.dma_x(0);
    vm_wait<0>();
    lds_barrier();  // B2
    for (int k = 0; k <= kSteps; ++k) {
      lds_barrier();  // S1: conv1(k) is done with the x buffer
      const bool dma = k + 1 < kSteps;
      if (dma) m.dma_x(k + 1);
      if (k >= 1) m.copy_t2(k - 1, t2 + ((k - 1) & 1) * kT2);
      if (dma) {  // the DMA has landed (this step's t2 stores may be in flight)
        if (k >= 1) vm_wait<kSTh>();
        else vm_wait<0>();
      }
      lds_barrier();  // S2
    }
    vm_wait<0>();  // no LDS-DMA may outlive the workgroup
  }
}

}  // namespace

bool bottleneck56_supported(int H, int W, int C, int Cm) { return H == kH && W == kW && C == kC && Cm == kM; }

void bottleneck56(const void* x, const void* w1, const float* a1, const float* b1, const void* wf2, const float* b2,
                  const void* wf3, const float* b3, void* y, float res_scale, float out_inv_scale, int B,
                  hipStream_t s) {
  if (B <= 0) return;
  if (!x || !w1 || !a1 || !b1 || !wf2 || !b2 || !wf3 || !b3 || !y ||
      (((uintptr_t)x | (uintptr_t)w1 | (uintptr_t)wf2 | (uintptr_t)wf3 | (uintptr_t)y) & 15))
    throw std::invalid_argument("bottleneck56: null / misaligned operand");
  if (x == y) throw std::invalid_argument("bottleneck56: in-place not supported (the residual is re-read)");
  BnArgs a;
  a.stagger = kernel_stagger(kStagBottleneck);
  a.x = (const uint8_t*)x;
  a.w1 = (const uint8_t*)w1;
  a.a1 = a1;
  a.b1 = b1;
  a.wf2 = (const bf16*)wf2;
  a.b2 = b2;
  a.wf3 = (const bf16*)wf3;
  a.b3 = b3;
  a.y = (uint8_t*)y;
  a.res_scale = res_scale;
  a.out_inv_scale = out_inv_scale;
  hipLaunchKernelGGL(bottleneck56_kernel, dim3(B), dim3(512), kLds, s, a);
  DMLC_HIP_CHECK(hipGetLastError());
}

void bottleneck56_head(const void* x, const void* w1, const float* b1, const void* wf2, const float* b2, void* y,
                       int B, hipStream_t s) {
  if (B <= 0) return;
  if (!x || !w1 || !b1 || !wf2 || !b2 || !y || (((uintptr_t)x | (uintptr_t)w1 | (uintptr_t)wf2 | (uintptr_t)y) & 15))
    throw std::invalid_argument("bottleneck56_head: null / misaligned operand");
  if (x == y) throw std::invalid_argument("bottleneck56_head: in-place not supported");
  BnArgs a = {};
  a.stagger = kernel_stagger(kStagBottleneck);
  a.x = (const uint8_t*)x;
  a.w1 = (const uint8_t*)w1;
  a.b1 = b1;
  a.wf2 = (const bf16*)wf2;
  a.b2 = b2;
  a.y = (uint8_t*)y;
  hipLaunchKernelGGL(bottleneck56_head_kernel, dim3(B), dim3(512), kLdsH, s, a);
  DMLC_HIP_CHECK(hipGetLastError());
}

}  // namespace dmlc
