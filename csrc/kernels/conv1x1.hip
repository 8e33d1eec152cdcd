// Weight-stationary 1x1 convolution for the ResNet50 bottleneck convs
// (conv1 reduce, conv3 expand, the 1x1/s2 downsample), bf16 or e4m3 in and
// out, BN folded, optional residual, ReLU.
//
// Reference equivalent: the Bottleneck 1x1 convs of tch::vision::resnet50
// (BASELINE config 5; forward_t per query at src/services.rs:493). At B=256
// these convs move 100-500 MB each with K = 64..512: as 128x128 implicit-GEMM
// tiles (conv_igemm.hip) every tile runs 1-4 K-steps between its prologue and
// a 16-64 KB epilogue, and layer1's expand conv ran at ~1.8 TB/s (280 us vs a
// ~100 us HBM floor: profiles/r2_resnet50_ops.txt). Here:
//
//  * a workgroup owns a 4*NW-channel slice of the output; each of its 4 waves
//    keeps its NW channels' weights (NW x K, <= 16 KB) in VGPRs for the whole
//    kernel, so weights are read once per workgroup, not once per tile;
//  * the workgroup walks 64-pixel blocks of M = B*Ho*Wo (persistent grid,
//    the slices of one block on the same XCD so its input is fetched from HBM
//    once), its input rows (K bytes / 2K bytes per pixel) arriving by LDS-DMA
//    S blocks ahead; the residual of a block is loaded (asm, counted) with its
//    DMA and consumed in the epilogue;
//  * D = W x X on v_mfma_f32_16x16x32_bf16 or the block-scaled
//    v_mfma_scale_f32_16x16x128_f8f6f4 (unit scales): a lane ends with 8
//    consecutive channels of one pixel (weight rows permuted within 32-channel
//    groups), stored as one 16-B (bf16) / 8-B (e4m3) write.
//
// vmcnt retires in issue order and the compiler cannot see the asm loads, so
// every wait is explicit: per block a wave issues RES (the next block's
// residual loads), DMA (S-1 blocks ahead; dummy zero-page loads past the end
// keep the counts uniform) and ST (stores); the block's DMA has landed when at
// most (S-1)(ST+RES+DMA) newer operations are outstanding, its residual when
// at most 2 DMA + ST + RES are (the chained form's reduce stores, issued with
// the next block, add to both; every threshold comes from c1_plan below and
// is replayed against this issue order in tests/test_conv1x1_vmcnt_cpu.py).
// Only M % BM == 0 is supported (BM = 64, 32 for 1-KB rows: no partial
// blocks, so every wave issues the same instruction counts).
#include "common.h"
#include "kernels.h"

#include <algorithm>
#include <type_traits>

namespace dmlc {

namespace {

typedef int v8i __attribute__((ext_vector_type(8)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int N>
__device__ __forceinline__ void vm_wait() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}

// LDS reads/writes of this wave done, then the workgroup barrier (no
// compiler fence: it would add a vmcnt(0) and drain the DMA pipeline)
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
}

// Make the compiler treat v as (re)defined here, after a preceding wait:
// uses of an asm-loaded register cannot be hoisted above the wait.
template <typename T>
__device__ __forceinline__ void pin(T& v) {
  asm volatile("" : "+v"(v));
}


__device__ __forceinline__ void fp8x4_to_f32(uint32_t u, float* f) {
  e4m3x4_to_f32(u, f);
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

// Counted global loads the compiler does not track (no implicit vmcnt(0)
// waits in front of their uses: the kernel waits for them itself).
__device__ __forceinline__ u32x2 gload8(const void* p) {
  u32x2 v;
  asm volatile("global_load_dwordx2 %0, %1, off" : "=v"(v) : "v"(p) : "memory");
  return v;
}
__device__ __forceinline__ u32x4 gload16(const void* p) {
  u32x4 v;
  asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(v) : "v"(p) : "memory");
  return v;
}
__device__ __forceinline__ uint32_t gload4(const void* p) {
  uint32_t v;
  asm volatile("global_load_dword %0, %1, off" : "=v"(v) : "v"(p) : "memory");
  return v;
}

// Chunk swizzle of the staged input rows (16-B chunks, RB bytes per pixel):
// every 16-lane group of the B-fragment reads hits 16 distinct bank groups
// (tests/test_layouts_cpu.py::test_conv1x1_lds_conflict_free).
template <int RB, bool IN8>
__device__ __forceinline__ int swz1(int p) {
  if constexpr (RB == 128) return IN8 ? ((((p & 7) << 1) | ((p >> 3) & 1)) & 7) : (p & 7);
  else return p & 15;
}

struct C1Args {
  const void* x;       // [B, H, W, K] bf16 or e4m3
  const void* w;       // [Npad, Kpad] bf16 or e4m3 (BN folded; e4m3 with per-row scales)
  const float* bias;   // [Npad]
  const float* alpha;  // e4m3 input: [Npad] = s_in * s_w[n]
  const void* res;     // [M, N] (the output's dtype) or null
  void* y;             // [M, N]
  const void* zero;    // >= 16 zero bytes
  int B, H, W, Ho, Wo, N, Kpad;
  int nslices, nblocks;
  int relu;
  float res_scale, out_inv_scale;
  const void* x2;  // second input (K chunks cpr1 .. CPR-1 of a pixel), or null
  int cpr1;        // 16-B chunks of a pixel from x
  int stagger;     // start_stagger (common.h)
  // CH (chained reduce): the next bottleneck's reduce conv on this conv's
  // output block, read back from LDS: y2 = e4m3(relu(w2 x y * alpha2 + bias2) * out_inv_scale2)
  const void* w2;       // [N2][N] e4m3
  const float* alpha2;  // [N2]
  const float* bias2;   // [N2]
  void* y2;             // [M, N2] e4m3
  int N2, relu2;
  float out_inv_scale2;
};

// pixels per block: 64, or 32 for 1-KB input rows (stage = BM x RB bytes)
template <int RB>
constexpr int block_m() { return RB <= 512 ? 64 : 32; }

}  // namespace

// The block loop's vector-memory plan (kernels.h C1Plan): operation counts per
// wave per block and every s_waitcnt vmcnt threshold, computed once here for
// the kernel's template constants and for the host (conv1x1_plan:
// tests/test_conv1x1_vmcnt_cpu.py replays the kernel's issue order against it).
constexpr C1Plan c1_plan(bool in8, bool out8, int rb, int nw, bool res, int s, int wv, bool ch) {
  C1Plan p{};
  const int bm = rb <= 512 ? 64 : 32;
  const int nf = nw / 16;
  const bool w16 = out8 && nf >= 4;
  const int ng = w16 ? nf / 4 : nf >= 2 ? nf / 2 : 1;
  const int npf = bm / 16;
  p.s = s;
  p.dt = bm * rb / 16 / 64 / wv;
  p.rt = res ? npf * ng : 0;
  p.st2 = ch ? npf : 0;
  p.st = npf * ng + p.st2;
  p.pre = res && out8 && (wv == 8 || rb <= 256);
  // block it's rows were DMA'd S-1 blocks earlier; everything issued since:
  // (S-1) blocks of R + D + stores, and (CH) one more set of reduce stores
  // (the previous block's, issued after this block's R and D)
  p.n1 = (s - 1) * (p.st + p.rt + p.dt) + p.st2;
  p.n1_first = p.n1 - p.st2;  // CH, block S-1: block 0 issued no reduce stores
  p.pro_wait = p.pre ? p.rt + p.dt : p.dt;  // blocks < S-1: only this block's R, D in flight
  p.pro_wait_ch = p.pro_wait + p.st2;       // ... and (CH, it > 0) the reduce stores after them
  // PRE: block it's residual came with block it-1's R, before D(it-1), its
  // stores, R(it), D(it) and (CH) the reduce stores of it-2 and it-1
  p.res_wait = p.pre ? 2 * p.dt + p.st + p.rt + p.st2 : p.dt;
  return p;
}

C1Plan conv1x1_plan(bool in8, bool out8, int rb, int nw, bool res, int s, int wv, bool ch) {
  return c1_plan(in8, out8, rb, nw, res, s, wv, ch);
}

namespace {

// WV waves per workgroup: 4 (two workgroups per CU, <= 64 weight VGPRs per
// wave) or 8 (one per CU, <= 128 weight VGPRs per wave: twice the channels
// per wave and per workgroup, so a wide layer restages its input for fewer
// channel slices).
//
// CH (chained reduce, ResNet50 e4m3 layer2): this conv is a bottleneck's
// expand conv (e4m3, residual, all N = 512 output channels in one
// workgroup) and the next bottleneck's reduce conv (512 -> 128, e4m3, ReLU)
// runs on each finished 64-pixel output block while it is still on chip: the
// block goes to LDS next to its y store, and every wave computes 16 reduce
// channels from it (weights in 32 more VGPRs, 4 K steps). The reduce conv's
// separate launch re-read all of y from HBM (102.8 MB at B = 256).
template <bool IN8, bool OUT8, int RB, int NW, int S2, bool RES, int S, int WV, bool CH = false>
__global__ __launch_bounds__(64 * WV, WV == 4 ? 2 : 1) void conv1x1_kernel(C1Args a) {
  constexpr int kBM = block_m<RB>();
  constexpr int CPR = RB / 16;              // 16-B chunks per staged pixel row
  constexpr int KS = IN8 ? CPR / 8 : CPR / 4;  // K steps (128 e4m3 / 32 bf16 k each)
  constexpr int NF = NW / 16;               // N fragments per wave
  // e4m3 output with >= 4 N fragments: weight rows in the perm64 order, so a
  // lane's accumulators are 16 consecutive channels (16-B residual loads and
  // y stores, 64 B per pixel per wave instruction, instead of 8 B / 32 B)
  constexpr bool W16 = OUT8 && NF >= 4;
  constexpr int NG = W16 ? NF / 4 : NF >= 2 ? NF / 2 : 1;  // channel groups per lane
  constexpr int CPL = W16 ? 16 : NF >= 2 ? 8 : 4;          // channels per lane per group
  constexpr int NPF = kBM / 16;             // pixel fragments per block
  constexpr int STAGE = kBM * RB;
  constexpr C1Plan P = c1_plan(IN8, OUT8, RB, NW, RES, S, WV, CH);
  constexpr int DT = P.dt;                  // DMA instructions per wave per block
  constexpr int RT = P.rt;                  // residual loads per wave per block
  constexpr int NP2 = CH ? WV * NW : 0;     // chained reduce: its K (= N, e4m3 bytes per pixel)
  constexpr int KS2 = NP2 / 128;            // its K steps
  constexpr int ST2 = P.st2;                // the chained reduce's stores (of the previous block)
  constexpr int ST = P.st;                  // stores per wave per block
  // (CH: the previous block's reduce stores are issued after this block's
  // R and D, so one more ST2 sits between a block's DMA and its wait)
  constexpr int N1 = P.n1;
  static_assert(DT >= 1 && KS >= 1, "tile");
  static_assert(!CH || (IN8 && OUT8 && RES && W16 && NG == 1 && NP2 == 512 && S2 == 1), "chained reduce form");
  using WFrag = typename std::conditional<IN8, v8i, bf16x8>::type;

  extern __shared__ __attribute__((aligned(16))) uint4 smem[];
  char* stages = (char*)smem;
  char* ybuf = stages + S * STAGE;  // CH: the output block, [kBM][NP2] chunk-swizzled (c ^ (p & 15))

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  start_stagger(a.stagger);
  const int fr = lane & 15, g = lane >> 4;
  // block id -> (slice, first block): the slices of one M block on one XCD
  const int wgid = blockIdx.x;
  const int xcd = wgid & 7, r = wgid >> 3;
  const int slice = r % a.nslices;
  const int mstart = (r / a.nslices) * 8 + xcd;
  const int mstride = (int)gridDim.x / a.nslices;
  const int n0 = slice * WV * NW + wave * NW;  // this wave's first channel

  // ---- weights -> VGPRs: fragment f row rr = channel ch(f, rr); lane (rr, g)
  // holds k = 32*ks + 8g .. +8 (bf16) / 128*ks + 32g .. +32 (e4m3)
  auto ch_of = [](int f, int rr) {
    if constexpr (W16) return 64 * (f >> 2) + 16 * (rr >> 2) + 4 * (f & 3) + (rr & 3);
    else if constexpr (NF >= 2) return 32 * (f >> 1) + 8 * (rr >> 2) + 4 * (f & 1) + (rr & 3);
    else return rr;
  };
  // first channel of lane group j
  auto grp_ch = [&](int j) { return W16 ? 64 * j + 16 * g : NF >= 2 ? 32 * j + 8 * g : 4 * g; };
  WFrag wf[NF][KS];
  {
    const uint8_t* wb = (const uint8_t*)a.w;
    const int esz = IN8 ? 1 : 2;
#pragma unroll
    for (int f = 0; f < NF; ++f) {
      const uint8_t* row = wb + (size_t)(n0 + ch_of(f, fr)) * a.Kpad * esz;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        if constexpr (IN8) {
          const uint4 lo = *(const uint4*)(row + ks * 128 + g * 32);
          const uint4 hi = *(const uint4*)(row + ks * 128 + g * 32 + 16);
          wf[f][ks] = v8i{(int)lo.x, (int)lo.y, (int)lo.z, (int)lo.w, (int)hi.x, (int)hi.y, (int)hi.z, (int)hi.w};
        } else {
          wf[f][ks] = *(const bf16x8*)(row + (ks * 32 + g * 8) * 2);
        }
      }
    }
  }
  // this lane's channels: group j = n0 + 32j + 8g .. +7 (NF = 1: n0 + 4g .. +3).
  // e4m3 output: the 1 / s_out quantisation scale is folded into alpha, the
  // bias and the residual scale here, so an output value costs one fma (+ one
  // for the residual) and one med3 (ReLU and the +-448 saturation together)
  const float osc = OUT8 ? a.out_inv_scale : 1.f;
  const float rsc = a.res_scale * osc;
  const float relu_lo = a.relu ? 0.f : -448.f;  // e4m3 output: med3(v, relu_lo, 448)
  float bs[NG][CPL], al[NG][CPL];
#pragma unroll
  for (int j = 0; j < NG; ++j)
#pragma unroll
    for (int e = 0; e < CPL; ++e) {
      const int n = n0 + grp_ch(j) + e;
      bs[j][e] = a.bias[n] * osc;
      al[j][e] = (IN8 ? a.alpha[n] : 1.f) * osc;
    }

  // CH: the reduce conv's weights (channel 16 wave + fr, k = 128 ks + 32 g ..
  // +32 at lane (fr, g)) and constants (lane channels 16 wave + 4 g .. +3)
  v8i wf2[CH ? KS2 : 1];
  f32x2 al2[2], bs2[2];
  const float relu_lo2 = a.relu2 ? 0.f : -448.f;
  if constexpr (CH) {
    const uint8_t* row = (const uint8_t*)a.w2 + (size_t)(wave * 16 + fr) * NP2;
#pragma unroll
    for (int ks = 0; ks < KS2; ++ks) {
      const uint4 lo = *(const uint4*)(row + ks * 128 + g * 32);
      const uint4 hi = *(const uint4*)(row + ks * 128 + g * 32 + 16);
      wf2[ks] = v8i{(int)lo.x, (int)lo.y, (int)lo.z, (int)lo.w, (int)hi.x, (int)hi.y, (int)hi.z, (int)hi.w};
    }
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int n = wave * 16 + 4 * g + 2 * e;
      al2[e] = f32x2{a.alpha2[n], a.alpha2[n + 1]} * a.out_inv_scale2;
      bs2[e] = f32x2{a.bias2[n], a.bias2[n + 1]} * a.out_inv_scale2;
    }
  }

  // ---- staging: block m -> stage buffer (pixel p's RB bytes, chunk-swizzled)
  const long rowstride_in = (long)a.cpr1 * 16;  // x's pixel stride (all of K without x2)
  auto pixel_src = [&](int m) -> const uint8_t* {  // input pixel of output pixel m
    if constexpr (S2 == 1) {
      return (const uint8_t*)a.x + (long)m * rowstride_in;
    } else {
      const int hw = a.Ho * a.Wo;
      const int b = m / hw, rem = m - b * hw, oh = rem / a.Wo, ow = rem - oh * a.Wo;
      return (const uint8_t*)a.x + (((long)b * a.H + 2 * oh) * a.W + 2 * ow) * rowstride_in;
    }
  };
  auto issue_dma = [&](int blk, int st) __attribute__((always_inline)) {
    char* dst = stages + st * STAGE;
    const bool live = blk < a.nblocks;
#pragma unroll
    for (int d = 0; d < DT; ++d) {
      const int i = (d * WV + wave) * 64 + lane;  // chunk index in the stage
      const int p = i / CPR, pc = i % CPR;
      const int lc = pc ^ swz1<RB, IN8>(p);  // logical chunk stored at physical pc
      const void* src = a.zero;
      if (live) {
        if (lc < a.cpr1)
          src = pixel_src(blk * kBM + p) + lc * 16;
        else  // concatenated second input (stride 1: same pixel index)
          src = (const uint8_t*)a.x2 + ((long)(blk * kBM + p) * (CPR - a.cpr1) + (lc - a.cpr1)) * 16;
      }
      dma16(src, dst + (d * WV + wave) * 1024);
    }
  };
  // residual of block blk: lane (fr, g), pixel fragment pf, group j
  const int out_esz = OUT8 ? 1 : 2;
  auto res_ptr = [&](int blk, int pf, int j) {
    const long m = (long)blk * kBM + pf * 16 + fr;
    const int n = n0 + grp_ch(j);
    return (const uint8_t*)a.res + (m * a.N + n) * out_esz;
  };
  typedef typename std::conditional<
      OUT8, typename std::conditional<(CPL == 16), u32x4, typename std::conditional<(CPL == 8), u32x2, uint32_t>::type>::type,
      typename std::conditional<(CPL == 8), u32x4, u32x2>::type>::type RV;
  // PRE (e4m3 output with a residual): the residual of a block is loaded one
  // block ahead, into the other of two register sets (the block loop is
  // unrolled by two so each set stays in fixed registers), so its latency
  // hides under a whole block, not just the block's own MFMAs. (bf16: the
  // 64-channel forms have no registers for a second set; each block loads
  // its own residual with its DMA.)
  constexpr bool PRE = P.pre;  // (RES && OUT8 && (WV == 8 || RB <= 256): the 4-wave 512-B form has no registers either)
  static_assert(!CH || PRE, "the chained reduce form loads its residual a block ahead");
  RV rv0[NPF][NG], rv1[NPF][NG];
  auto load_res = [&](int blk, RV (&rv)[NPF][NG]) __attribute__((always_inline)) {
    const bool live = blk < a.nblocks;  // (past the end: the zero page, so every wave issues RT loads)
#pragma unroll
    for (int pf = 0; pf < NPF; ++pf)
#pragma unroll
      for (int j = 0; j < NG; ++j) {
        const void* p = live ? (const void*)res_ptr(blk, pf, j) : a.zero;
        if constexpr (OUT8 && CPL == 16) rv[pf][j] = gload16(p);
        else if constexpr (OUT8 && CPL == 8) rv[pf][j] = gload8(p);
        else if constexpr (OUT8) rv[pf][j] = gload4(p);
        else if constexpr (CPL == 8) rv[pf][j] = gload16(p);
        else rv[pf][j] = gload8(p);
      }
  };

  // prologue: the first block's residual, then blocks 0 .. S-2's rows
  if constexpr (PRE) load_res(mstart, rv0);
#pragma unroll
  for (int s = 0; s < S - 1; ++s) issue_dma(mstart + s * mstride, s);

  // ---- CH: the chained reduce of block blk from ybuf (issued at the start of
  // the next block, between its loads and its DMA wait, so it runs under
  // that latency; every wave wrote its share of ybuf before the barrier that
  // opens that block, and none writes ybuf again before the block's second
  // barrier: one buffer suffices)
  auto reduce = [&](int blk) __attribute__((always_inline)) {
    floatx4 acc2[NPF];
#pragma unroll
    for (int pf = 0; pf < NPF; ++pf) acc2[pf] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < KS2; ++ks) {
      v8i xb[NPF];
#pragma unroll
      for (int pf = 0; pf < NPF; ++pf) {
        const int p = pf * 16 + fr, c0 = ks * 8 + 2 * g;
        const char* row = ybuf + p * NP2;
        const uint4 lo = *(const uint4*)(row + ((c0 ^ (p & 15)) << 4));
        const uint4 hi = *(const uint4*)(row + (((c0 + 1) ^ (p & 15)) << 4));
        xb[pf] = v8i{(int)lo.x, (int)lo.y, (int)lo.z, (int)lo.w, (int)hi.x, (int)hi.y, (int)hi.z, (int)hi.w};
      }
#pragma unroll
      for (int pf = 0; pf < NPF; ++pf)
        acc2[pf] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(wf2[ks], xb[pf], acc2[pf], 0, 0, 0, 127, 0, 127);
    }
#pragma unroll
    for (int pf = 0; pf < NPF; ++pf) {
      const long m = (long)blk * kBM + pf * 16 + fr;
      float v[4];
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const f32x2 r = __builtin_elementwise_fma(f32x2{acc2[pf][2 * e], acc2[pf][2 * e + 1]}, al2[e], bs2[e]);
        v[2 * e] = __builtin_amdgcn_fmed3f(r.x, relu_lo2, 448.f);
        v[2 * e + 1] = __builtin_amdgcn_fmed3f(r.y, relu_lo2, 448.f);
      }
      *(uint32_t*)((uint8_t*)a.y2 + m * a.N2 + wave * 16 + 4 * g) = f32x4_to_fp8_sat(v);
    }
  };

  // per block a wave issues R [RT] (PRE: the next block's), D(block + S-1)
  // [DT], (CH) the previous block's reduce stores [ST2], then after the MFMAs
  // its stores [ST - ST2]. The block's rows have landed when at most N1 =
  // (S-1)(RT+DT+ST) + ST2 newer operations are outstanding; its residual when
  // at most 2 DT + ST + RT + ST2 (PRE: issued one block earlier, after
  // D(block + S-2)) / DT are (C1Plan).
  auto block = [&](int blk, int it, RV (&rv)[NPF][NG], RV (&rvn)[NPF][NG]) __attribute__((always_inline)) {
    const int st = it % S;
    lds_barrier();  // every wave is done with stage (it-1) % S: the DMA below reuses it
    if constexpr (PRE) load_res(blk + mstride, rvn);
    else if constexpr (RES) load_res(blk, rv);
    issue_dma(blk + (S - 1) * mstride, (it + S - 1) % S);
    if constexpr (CH) {
      if (it > 0) reduce(blk - mstride);
    }
    if (it < S - 1) {  // prologue blocks: only this block's issues (CH: + the reduce stores) may stay in flight
      if (CH && it > 0) vm_wait<P.pro_wait_ch>();
      else vm_wait<P.pro_wait>();
    } else if (CH && it == S - 1) {
      vm_wait<P.n1_first>();  // (block 0 had no reduce to issue)
    } else {
      vm_wait<N1>();
    }
    lds_barrier();  // every wave's share of block blk's rows has landed
    // ---- MFMAs: acc[pf][f] = D[channel ch(f, 4g+i)][pixel 16pf + fr]
    const char* sb = stages + st * STAGE;
    floatx4 acc[NPF][NF];
#pragma unroll
    for (int pf = 0; pf < NPF; ++pf)
#pragma unroll
      for (int f = 0; f < NF; ++f) acc[pf][f] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      WFrag xb[NPF];
#pragma unroll
      for (int pf = 0; pf < NPF; ++pf) {
        const int p = pf * 16 + fr;
        const char* row = sb + p * RB;
        if constexpr (IN8) {
          const int c0 = ks * 8 + 2 * g;
          const uint4 lo = *(const uint4*)(row + ((c0 ^ swz1<RB, IN8>(p)) << 4));
          const uint4 hi = *(const uint4*)(row + (((c0 + 1) ^ swz1<RB, IN8>(p)) << 4));
          xb[pf] = v8i{(int)lo.x, (int)lo.y, (int)lo.z, (int)lo.w, (int)hi.x, (int)hi.y, (int)hi.z, (int)hi.w};
        } else {
          xb[pf] = *(const bf16x8*)(row + (((ks * 4 + g) ^ swz1<RB, IN8>(p)) << 4));
        }
      }
#pragma unroll
      for (int pf = 0; pf < NPF; ++pf)
#pragma unroll
        for (int f = 0; f < NF; ++f) {
          if constexpr (IN8)
            acc[pf][f] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(wf[f][ks], xb[pf], acc[pf][f], 0, 0, 0,
                                                                           127, 0, 127);
          else
            acc[pf][f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[f][ks], xb[pf], acc[pf][f], 0, 0, 0);
        }
    }

    // ---- epilogue
    if constexpr (RES) {
      if constexpr (PRE) {
        if (it >= S - 1) vm_wait<P.res_wait>();  // this block's residual (earlier blocks: waited above)
      } else {
        vm_wait<P.res_wait>();  // this block's residual (only the DMA issued after it may be in flight)
      }
#pragma unroll
      for (int pf = 0; pf < NPF; ++pf)
#pragma unroll
        for (int j = 0; j < NG; ++j) pin(rv[pf][j]);
    }
#pragma unroll
    for (int pf = 0; pf < NPF; ++pf) {
      const long m = (long)blk * kBM + pf * 16 + fr;
#pragma unroll
      for (int j = 0; j < NG; ++j) {
        float v[CPL];
        // channel pairs (2e, 2e+1) sit in consecutive accumulator registers:
        // scale + bias (and the e4m3 residual below) as v_pk_fma_f32, two
        // channels an instruction
#pragma unroll
        for (int e = 0; e < CPL; e += 2) {
          const floatx4& q = W16 ? acc[pf][4 * j + (e >> 2)] : NF >= 2 ? acc[pf][2 * j + (e >> 2)] : acc[pf][0];
          const f32x2 raw = {q[e & 3], q[(e & 3) + 1]};
          f32x2 r;
          if constexpr (IN8 || OUT8)
            r = __builtin_elementwise_fma(raw, f32x2{al[j][e], al[j][e + 1]}, f32x2{bs[j][e], bs[j][e + 1]});
          else
            r = raw + f32x2{bs[j][e], bs[j][e + 1]};
          v[e] = r.x;
          v[e + 1] = r.y;
        }
        if constexpr (RES) {
          float rf[CPL];
          if constexpr (OUT8) {
            if constexpr (CPL == 16) {
              fp8x4_to_f32(rv[pf][j].x, rf);
              fp8x4_to_f32(rv[pf][j].y, rf + 4);
              fp8x4_to_f32(rv[pf][j].z, rf + 8);
              fp8x4_to_f32(rv[pf][j].w, rf + 12);
            } else if constexpr (CPL == 8) {
              fp8x4_to_f32(rv[pf][j].x, rf);
              fp8x4_to_f32(rv[pf][j].y, rf + 4);
            } else {
              fp8x4_to_f32(rv[pf][j], rf);
            }
#pragma unroll
            for (int e = 0; e < CPL; e += 2) {
              const f32x2 r = __builtin_elementwise_fma(f32x2{rf[e], rf[e + 1]}, f32x2{rsc, rsc}, f32x2{v[e], v[e + 1]});
              v[e] = r.x;
              v[e + 1] = r.y;
            }
          } else {
            if constexpr (CPL == 8) {
              const u32x4 q = rv[pf][j];
              unpack8(make_uint4(q.x, q.y, q.z, q.w), rf);
            } else {
              const u32x2 q = rv[pf][j];
              rf[0] = __uint_as_float(q.x << 16);
              rf[1] = __uint_as_float(q.x & 0xffff0000u);
              rf[2] = __uint_as_float(q.y << 16);
              rf[3] = __uint_as_float(q.y & 0xffff0000u);
            }
#pragma unroll
            for (int e = 0; e < CPL; ++e) v[e] += rf[e];
          }
        }
        const int n = n0 + grp_ch(j);
        uint8_t* yp = (uint8_t*)a.y + (m * a.N + n) * out_esz;
        if constexpr (OUT8) {  // (already scaled by 1 / s_out)
#pragma unroll
          for (int e = 0; e < CPL; ++e) v[e] = __builtin_amdgcn_fmed3f(v[e], relu_lo, 448.f);
          if constexpr (CPL == 16) {
            const uint4 q4 = make_uint4(f32x4_to_fp8_sat(v), f32x4_to_fp8_sat(v + 4), f32x4_to_fp8_sat(v + 8),
                                        f32x4_to_fp8_sat(v + 12));
            *(uint4*)yp = q4;
            if constexpr (CH) {  // and into the chained reduce's input block
              const int p = pf * 16 + fr, c = n >> 4;
              *(uint4*)(ybuf + p * NP2 + ((c ^ (p & 15)) << 4)) = q4;
            }
          } else if constexpr (CPL == 8) *(uint2*)yp = make_uint2(f32x4_to_fp8_sat(v), f32x4_to_fp8_sat(v + 4));
          else *(uint32_t*)yp = f32x4_to_fp8_sat(v);
        } else if constexpr (CPL == 8) {
          *(uint4*)yp = pack8_relu(v, a.relu);  // ReLU on the packed bf16
        } else {
          if (a.relu) {
#pragma unroll
            for (int e = 0; e < CPL; ++e) v[e] = __builtin_amdgcn_fmed3f(v[e], 0.f, __builtin_inff());
          }
          *(uint2*)yp = make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3]));
        }
      }
    }
  };
  int it = 0;
  if constexpr (PRE) {
    for (int blk = mstart; blk < a.nblocks; blk += 2 * mstride, it += 2) {
      block(blk, it, rv0, rv1);
      if (blk + mstride < a.nblocks) block(blk + mstride, it + 1, rv1, rv0);
    }
  } else {
    for (int blk = mstart; blk < a.nblocks; blk += mstride, ++it) block(blk, it, rv0, rv0);
  }
  if constexpr (CH) {
    if (it > 0) {  // the last block's reduce
      lds_barrier();
      int last = mstart;
      while (last + mstride < a.nblocks) last += mstride;
      reduce(last);
    }
  }
  vm_wait<0>();  // no LDS-DMA may outlive the workgroup
}

// Register-resident weights of a wave: NW x RB bytes <= 16 KB (64 VGPRs),
// and with 8 waves also the 32 KB of 32 bf16 1-KB rows (128 VGPRs: ResNet50
// layer4's expand conv). Other 32 KB forms spilled (fp8 1-KB rows at 32
// channels, 512-B rows at 64 channels).
constexpr bool weights_fit(int wv, bool in8, int rb, int nw) {
  return nw * rb <= 16384 || (wv == 8 && !in8 && rb == 1024 && nw == 32);
}

// (waves per workgroup, channels per wave, staged row bytes) for a shape, or
// nw = 0. The fewest channel slices win (every slice restages the whole
// input: ResNet50 layer4's expand conv ran 32 slices at 4 waves x 16
// channels); at equal slices the 4-wave form (two workgroups per CU).
struct Pick {
  int wv = 4, nw = 0, rb = 0;
};

Pick pick(const ConvArgs& a) {
  Pick p;
  if (a.KH != 1 || a.KW != 1 || a.pad != 0 || (a.stride != 1 && a.stride != 2) || a.stem || a.out_f32 ||
      a.split_k > 1)
    return p;
  const int esz = a.in_fp8 ? 1 : 2;
  if (a.x2 && (a.in_fp8 || a.stride != 1 || a.cin2 <= 0 || a.cin2 % 8)) return p;
  if (a.Cin + (a.x2 ? a.cin2 : 0) != a.Kpad || a.N != a.Npad || a.ldo != a.N) return p;
  const int rb = a.Kpad * esz;
  if (rb != 128 && rb != 256 && rb != 512 && rb != 1024) return p;
  if (a.in_fp8 && a.Cin % 128) return p;
  const long M = (long)a.B * a.Ho * a.Wo;
  if (M % (rb <= 512 ? 64 : 32)) return p;
  // strided 1-KB rows (ResNet50 layer4.0 downsample, 32 channel slices each
  // re-staging every input block): 72 us vs 57 us on the implicit GEMM
  if (a.stride == 2 && rb > 512) return p;
  int best = 0;
  for (int wv : {4, 8})
    for (int nw : {64, 32, 16}) {
      if (a.N % (wv * nw)) continue;
      if (!weights_fit(wv, a.in_fp8, rb, nw)) continue;
      const int slices = a.N / (wv * nw);
      if (!best || slices < best) {
        best = slices;
        p.wv = wv;
        p.nw = nw;
        p.rb = rb;
      }
      break;  // the widest nw that fits this wave count
    }
  return p;
}

struct L1 {
  dim3 grid;
  size_t lds;
  hipStream_t s;
  C1Args c;
  int wv, nw, rb;
};

template <bool IN8, bool OUT8, int RB, int S2, bool RES, int WV>
void launch_wv(const L1& l) {
  constexpr int S = RB <= 256 ? 3 : 2;
  const dim3 block(64 * WV);
  if constexpr (weights_fit(WV, IN8, RB, 64)) {
    if (l.nw == 64) {
      hipLaunchKernelGGL((conv1x1_kernel<IN8, OUT8, RB, 64, S2, RES, S, WV>), l.grid, block, l.lds, l.s, l.c);
      return;
    }
  }
  if constexpr (weights_fit(WV, IN8, RB, 32)) {
    if (l.nw == 32) {
      hipLaunchKernelGGL((conv1x1_kernel<IN8, OUT8, RB, 32, S2, RES, S, WV>), l.grid, block, l.lds, l.s, l.c);
      return;
    }
  }
  hipLaunchKernelGGL((conv1x1_kernel<IN8, OUT8, RB, 16, S2, RES, S, WV>), l.grid, block, l.lds, l.s, l.c);
}

template <bool IN8, bool OUT8, int RB, int S2, bool RES>
void launch_nw(const L1& l) {
  if (l.wv == 8) launch_wv<IN8, OUT8, RB, S2, RES, 8>(l);
  else launch_wv<IN8, OUT8, RB, S2, RES, 4>(l);
}

template <bool IN8, bool OUT8, int S2, bool RES>
void launch_rb(const L1& l) {
  if (l.rb == 128) launch_nw<IN8, OUT8, 128, S2, RES>(l);
  else if (l.rb == 256) launch_nw<IN8, OUT8, 256, S2, RES>(l);
  else if (l.rb == 512) launch_nw<IN8, OUT8, 512, S2, RES>(l);
  else launch_nw<IN8, OUT8, 1024, S2, RES>(l);
}

}  // namespace

bool conv1x1_supported(const ConvArgs& a) { return pick(a).nw > 0; }

bool conv1x1_chain_supported(const ConvArgs& a, const ConvArgs& r) {
  const Pick pk = pick(a);
  // the expand conv: e4m3 in and out, residual, 128-B input rows, all 512
  // channels in one 8-wave workgroup; the reduce conv: 1x1 / stride 1 on its
  // output (K = 512 e4m3), 128 e4m3 output channels = 16 per wave
  return pk.nw == 64 && pk.wv == 8 && pk.rb == 128 && a.N == 512 && a.in_fp8 && a.out_fp8 && a.res && !a.x2 &&
         a.stride == 1 && conv1x1_supported(r) && r.in_fp8 && r.out_fp8 && !r.res && !r.x2 && r.stride == 1 &&
         r.Kpad == a.N && r.Cin == a.N && r.N == 128 && r.ldo == 128 && r.B == a.B && r.H == a.Ho && r.W == a.Wo &&
         r.alpha && r.bias && r.w && r.y;
}

void conv1x1_chain(const ConvArgs& a, const ConvArgs& r, int num_cus, hipStream_t s) {
  if (!conv1x1_chain_supported(a, r)) throw std::invalid_argument("conv1x1_chain: unsupported pair");
  if (!a.x || !a.w || !a.bias || !a.y || !a.zero || !a.alpha ||
      (((uintptr_t)a.x | (uintptr_t)a.w | (uintptr_t)a.y | (uintptr_t)a.res | (uintptr_t)r.w | (uintptr_t)r.y) & 15))
    throw std::invalid_argument("conv1x1_chain: null / misaligned operand");
  C1Args c{};
  c.x = a.x;
  c.x2 = nullptr;
  c.cpr1 = a.Cin / 16;
  c.w = a.w;
  c.bias = a.bias;
  c.alpha = a.alpha;
  c.res = a.res;
  c.y = a.y;
  c.zero = a.zero;
  c.B = a.B;
  c.H = a.H;
  c.W = a.W;
  c.Ho = a.Ho;
  c.Wo = a.Wo;
  c.N = a.N;
  c.Kpad = a.Kpad;
  c.relu = a.relu;
  c.stagger = kernel_stagger(kStagConv1x1);
  c.res_scale = a.res_scale;
  c.out_inv_scale = a.out_inv_scale;
  c.nslices = 1;
  c.nblocks = (int)((long)a.B * a.Ho * a.Wo / 64);
  c.w2 = r.w;
  c.alpha2 = r.alpha;
  c.bias2 = r.bias;
  c.y2 = r.y;
  c.N2 = r.N;
  c.relu2 = r.relu;
  c.out_inv_scale2 = r.out_inv_scale;
  const int q = std::max(1, std::min((c.nblocks + 7) / 8, num_cus / 8));
  const size_t lds = 3 * 64 * 128 + 64 * 512;
  hipLaunchKernelGGL((conv1x1_kernel<true, true, 128, 64, 1, true, 3, 8, true>), dim3(8 * q), dim3(512), lds, s, c);
  DMLC_HIP_CHECK(hipGetLastError());
}

void conv1x1(const ConvArgs& a, int num_cus, hipStream_t s) {
  const Pick pk = pick(a);
  if (!pk.nw) throw std::invalid_argument("conv1x1: unsupported shape");
  if (!a.x || !a.w || !a.bias || !a.y || !a.zero || (a.in_fp8 && !a.alpha) ||
      (((uintptr_t)a.x | (uintptr_t)a.w | (uintptr_t)a.y | (uintptr_t)a.res) & 15))
    throw std::invalid_argument("conv1x1: null / misaligned operand");
  C1Args c;
  c.x = a.x;
  c.x2 = a.x2;
  c.cpr1 = a.Cin * (a.in_fp8 ? 1 : 2) / 16;
  if (a.x2 && ((uintptr_t)a.x2 & 15)) throw std::invalid_argument("conv1x1: misaligned second input");
  c.w = a.w;
  c.bias = a.bias;
  c.alpha = a.alpha;
  c.res = a.res;
  c.y = a.y;
  c.zero = a.zero;
  c.B = a.B;
  c.H = a.H;
  c.W = a.W;
  c.Ho = a.Ho;
  c.Wo = a.Wo;
  c.N = a.N;
  c.Kpad = a.Kpad;
  c.relu = a.relu;
  c.stagger = kernel_stagger(kStagConv1x1);
  c.res_scale = a.res_scale;
  c.out_inv_scale = a.out_inv_scale;
  c.nslices = a.N / (pk.wv * pk.nw);
  const int bm = pk.rb <= 512 ? 64 : 32;
  c.nblocks = (int)((long)a.B * a.Ho * a.Wo / bm);
  // persistent grid: a multiple of 8 * nslices, about 2 (4 waves) or 1 (8
  // waves) workgroups per CU
  const int per_cu = pk.wv == 4 ? 2 : 1;
  const int q = std::max(1, std::min((c.nblocks + 7) / 8, (per_cu * num_cus) / (8 * c.nslices)));
  const dim3 grid(8 * c.nslices * q);
  const size_t lds = (size_t)(pk.rb <= 256 ? 3 : 2) * bm * pk.rb;
  const bool res = a.res != nullptr;
  const int key = (a.in_fp8 ? 1 : 0) | (a.out_fp8 ? 2 : 0) | (res ? 4 : 0) | (a.stride == 2 ? 8 : 0);
  const L1 l{grid, lds, s, c, pk.wv, pk.nw, pk.rb};
  // the (in, out, residual, stride) combinations ResNet50 needs
  switch (key) {
    case 0: launch_rb<false, false, 1, false>(l); break;  // bf16 -> bf16 (reduce convs of the bf16 model)
    case 4: launch_rb<false, false, 1, true>(l); break;   // bf16 -> bf16 + residual (bf16 expand)
    case 8: launch_rb<false, false, 2, false>(l); break;  // bf16 downsample
    case 1: launch_rb<true, false, 1, false>(l); break;   // e4m3 -> bf16 (fp8 reduce convs)
    case 2: launch_rb<false, true, 1, false>(l); break;   // bf16 -> e4m3 (layer1.0 downsample)
    case 6: launch_rb<false, true, 1, true>(l); break;    // bf16 -> e4m3 + residual (fp8 expand)
    case 11: launch_rb<true, true, 2, false>(l); break;   // e4m3 -> e4m3 / s2 (fp8 downsample)
    case 3: launch_rb<true, true, 1, false>(l); break;    // e4m3 -> e4m3
    case 7: launch_rb<true, true, 1, true>(l); break;     // e4m3 -> e4m3 + residual (expand after an e4m3 3x3)
    default: throw std::invalid_argument("conv1x1: unsupported dtype / residual / stride combination");
  }
  DMLC_HIP_CHECK(hipGetLastError());
}

}  // namespace dmlc
