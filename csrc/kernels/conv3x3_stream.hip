// Direct 3x3 / pad 1 convolution (stride 1 or 2) with the input image resident
// in LDS, BN folded, optional residual, ReLU. ResNet18 at batch >= 32 runs
// every 3x3 conv from layer2 on through it:
//   stride 1: layer2 (28x28x128), layer3 (14x14x256), layer4 (7x7x512)
//   stride 2: layer2.0.conv1 (56x56x64 -> 28x28x128), layer3.0.conv1 (28x28x128
//             -> 14x14x256), layer4.0.conv1 (14x14x256 -> 7x7x512); these also
//             compute the block's 1x1/s2 downsample conv when asked (its input
//             is the 3x3's tap (1,1), already resident: one more output, no
//             second pass over the block input)
//
// Reference equivalent: those convs + bn + (residual) + relu of
// tch::vision::resnet18, run per query by `forward_t` at src/services.rs:493.
// As an implicit GEMM (conv_igemm.hip) every output tile re-fetches its 3x3
// input window per tap (9x the input bytes through L2, from cold inputs in the
// model) and small-N tiles re-fetch the weights per tile. Here a workgroup owns
// HS output rows of one image (or IMG whole images) and C_out / NSP channels:
//
//  * Its input rows (the strip plus the halo rows inside the image) go HBM ->
//    LDS once by LDS-DMA and stay resident; taps that fall outside the image
//    read one zero pixel instead of staged zero padding. Chunks are XOR-
//    swizzled per pixel (see the staging loop) so every fragment read is
//    bank-conflict free and costs one VALU add. Stride 2 stores each input row
//    with its even columns first, then its odd ones.
//  * The folded weights stream through LDS in 32-deep K-tiles. Every wave
//    streams just the 32 output-channel rows it uses through a private 3-stage
//    LDS-DMA ring and waits only on its own vmcnt: the K loop has no workgroup
//    barrier. (With one shared ring the per-K-tile barrier, and the LDS read
//    latency it exposed, held the loop at ~50% MFMA busy: without MFMAs the
//    barrier/read skeleton alone took 35 of 60 us.)
//  * 8 waves (2 per SIMD) = WM pixel groups x 8/WM channel groups of 32 (2 N
//    fragments of 16). D = W x X. The weight rows are permuted when staged (row
//    16nf + r of a wave's tile holds channel 8(r>>2) + 4nf + (r&3) of its
//    group), so a lane ends with 8 consecutive output channels of one pixel:
//    16-B residual loads and stores.
//  * The K loop is software-pipelined: the operands of K-tile t+1 are read
//    while the MFMAs of t run.
// Design history and measurements: profiles/r1_stream_conv.log.
#include <atomic>

#include "common.h"
#include "kernels.h"

namespace dmlc {

namespace {

template <int N>
__device__ __forceinline__ void vm_wait() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}

struct StreamConvArgs {
  const bf16* x;      // [B, S*H, S*W, CI]
  const bf16* w;      // [CO, 9*CI], k = (kh*3 + kw)*CI + c
  const float* bias;  // [CO]
  const bf16* res;    // [B, H, W, CO] or null
  bf16* y;            // [B, H, W, CO]
  const bf16* zero;   // >= 16 zero bytes
  // fused 1x1 / stride-S downsample (DS kernels): yd = wd x (tap (1,1) input) + bd
  const bf16* wd;     // [CO, CI]
  const float* bd;    // [CO]
  bf16* yd;           // [B, H, W, CO]
  // WR kernels: weights in fragment order, [CO/32][KT][2][64 lanes][8] (lane l of
  // fragment nf of channel group g, K-tile t holds channel 32g + perm32(16nf +
  // (l & 15)), k = 32t + 8(l >> 4) .. +7), loaded straight into VGPRs
  const bf16* wf;
  const bf16* wdf;    // WR + DS: the downsample weights in the same order, [CO/32][CI/32][2][64][8]
  int B;
  int relu;
  unsigned long long* stamps;  // debug: per-workgroup phase stamps (100 MHz), or null
  // Fused global average pool (whole-image workgroups only): pool[b][c] =
  // mean over the image's pixels of the (post-ReLU) output, bf16 (what the
  // unfused avgpool kernel writes); with store_y = 0 the activation itself is
  // not written (nothing else reads it).
  bf16* pool;
  int store_y;
  // e4m3 output (ResNet50's bottleneck 3x3 -> its e4m3 expand conv): y holds
  // round(relu(v) * out_inv_scale) as e4m3 bytes [B, H, W, CO]; 0 = bf16
  float out_inv_scale;
  int stagger;  // start_stagger (common.h)
};

struct alignas(8) u32x2s {
  uint32_t x, y;
};
// 4 floats (>= -448, <= 448) -> 4 e4m3 bytes
__device__ __forceinline__ uint32_t e4m3x4(float a, float b, float c, float d) {
  int v = __builtin_amdgcn_cvt_pk_fp8_f32(fmaxf(a, -448.f), fmaxf(b, -448.f), 0, false);
  v = __builtin_amdgcn_cvt_pk_fp8_f32(fmaxf(c, -448.f), fmaxf(d, -448.f), v, true);
  return (uint32_t)v;
}

// Weight-row permutation inside a wave's 32-row tile: row n = 16nf + r holds
// channel 8(r>>2) + 4nf + (r&3) of the group, so the lane with accumulator
// rows 4fq..4fq+3 of fragments 0 and 1 owns the 8 consecutive channels
// 8fq .. 8fq+7.
__device__ __forceinline__ int perm32(int n) {
  const int nf = n >> 4, r = n & 15;
  return 8 * (r >> 2) + 4 * nf + (r & 3);
}

// Weight-tile chunk swizzle (physical 16-B chunk of logical chunk c of a 64-B
// row n), as conv_bigtile.hip: conflict-free for the fragment reads (lane
// reads chunk fq of row 16nf + fr).
__device__ __forceinline__ int wswz(int n, int c) { return c ^ (3 * ((n >> 2) & 1)); }

// Input chunk swizzle of a staged pixel with key K (see the staging loop).
template <int CPX>
__device__ __forceinline__ int xswz(int K) {
  if constexpr (CPX >= 16)
    return (K & 7) << 1;
  else
    return ((K >> 1) & 3) << 1;
}

// Geometry shared by the kernel and its launcher: output H x W, stride S, a
// workgroup owns HS output rows of one image (PARTS = H / HS > 1) or IMG whole
// images (PARTS == 1).
template <int H, int W, int CI, int HS, int IMG, int S, int ND>
struct StreamGeom {
  static constexpr int PARTS = H / HS;
  static_assert(PARTS == 1 || IMG == 1, "several images per workgroup only as whole images");
  static constexpr int HI = S * H, WI = S * W;         // input rows / columns
  // staged rows: the strip's S*(HS-1)+1 rows plus a halo row above and below,
  // one of which is outside the image when a stride-1 image has two strips
  static constexpr int XR = PARTS == 1                 ? IMG * HI
                            : (S == 1 && PARTS == 2) ? HS + 1
                            : (S * (HS - 1) + 3 < HI ? S * (HS - 1) + 3 : HI);
  static constexpr int PXB = CI * 2;                   // bytes per input pixel
  static constexpr int ROWB = WI * PXB;                // bytes per staged row
  static constexpr int ZB = XR * ROWB;                 // zero pixel
  static constexpr int XBYTES = ZB + PXB;              // input region
  static constexpr int WST = 32 * 32 * 2;              // a wave's weight stage: 32 rows x 32 k
  static constexpr size_t LDS = (size_t)XBYTES + (size_t)8 * ND * WST;
};

template <int H, int W, int CI, int CO, int HS, int IMG, int NSP, int WM, int S, int ND, bool DS, bool WR,
          int PD = 4, int NG = 1, int PRIO = 0>
__global__ __launch_bounds__(512, 1) void conv3x3_stream_kernel(StreamConvArgs a) {
  using G = StreamGeom<H, W, CI, HS, IMG, S, ND>;
  constexpr int BK = 32;                     // K-tile depth = one MFMA k-step
  constexpr int NPIX = IMG * HS * W;         // output pixels per workgroup (the last group may have fewer)
  constexpr int MFT = (NPIX + 15) / 16;      // pixel fragments (the last one partly padding)
  constexpr int MF = (MFT + WM - 1) / WM;    // per wave
  // NG = 2 (register weights only): a wave owns two 32-channel groups, so each
  // X fragment read from LDS feeds 4 MFMAs instead of 2 (the LDS read skeleton
  // alone was ~24 of the 14x14x256 conv's 43 us loop, profiles/r1_stream_conv.log)
  static_assert(NG == 1 || (NG == 2 && WR), "two channel groups per wave need the register weights");
  constexpr int WN = 32 * NG;                // channels per wave
  constexpr int NF = 2 * NG;                 // N fragments per wave
  constexpr int HI = G::HI, WI = G::WI;
  constexpr int PXB = G::PXB, ROWB = G::ROWB, ZB = G::ZB, WST = G::WST;
  constexpr int CPX = CI / 8;                // 16-B chunks per input pixel
  constexpr int XI = WI * CPX / 64;          // LDS-DMA instructions per input row
  constexpr int KT = 9 * CI / BK;            // K-tiles
  constexpr int CT = CI / BK;                // K-tiles per tap
  // A block's downsample conv reads exactly the 3x3 conv's tap (1,1) input
  // (x[S r, S c]), which is resident here: its CT K-tiles follow the 3x3's KT
  // in the same weight stream, on tap (1,1)'s X fragments, into accd.
  constexpr int KT2 = KT + (DS ? CT : 0);
  // WR: each wave's weight fragments come from HBM/L2 in fragment order
  // straight into a PD-deep register ring (no LDS stage, no DMA wait)
  static_assert(!WR || CT % PD == 0, "WR: PD divides the K-tiles per tap");
  constexpr int GW = WST / 1024;             // weight DMA instructions per wave per K-tile
  static_assert(CO == 8 / WM * WN * NSP && WI * CPX % 64 == 0 && H % HS == 0 && CPX >= 8, "geometry");
  // (128-B pixels rely on the even/odd column halves starting on the same
  // window parity; pixels of >= 256 B fill whole bank windows)
  static_assert(S == 1 || (S == 2 && (WI % 4 == 0 || CPX >= 16) && HI % 2 == 0), "stride");
  static_assert(ND == 3 && KT >= ND, "the loop's waits assume a 3-stage ring");
  static_assert(MF + NF <= 15, "lgkmcnt range of the pipelined loop");

  extern __shared__ __attribute__((aligned(16))) uint4 smem[];
  char* xs = (char*)smem;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave % WM, wc = wave / WM;  // pixel group, channel group
  const int fr = lane & 15, fq = lane >> 4;
  const char* wpriv = xs + G::XBYTES + wave * (ND * WST);
  constexpr int PARTS = G::PARTS;
  // channel split fastest: the XCDs (blocks are dealt to them round-robin)
  // each hold one split's weight rows in their L2
  const int ns = blockIdx.x % NSP, rest = blockIdx.x / NSP;
  const int bg = rest / PARTS, part = rest - bg * PARTS;
  const int b = bg * IMG, nimg = min(IMG, a.B - b);         // first image, images here
  const int r0 = part * HS;                                 // first output row
  const int rs = PARTS == 1 ? 0 : max(S * r0 - 1, 0);       // first staged input row
  const int nrows = PARTS == 1 ? nimg * HI : min(S * (r0 + HS - 1) + 1, HI - 1) - rs + 1;
  const int npix = IMG == 1 ? NPIX : nimg * HS * W;
  const int ch0 = ns * (CO / NSP) + wc * WN;                // this wave's first output channel
  const bf16* img = a.x + (long)b * HI * WI * CI;
  // A scalar memory op still pending in the loop (a debug stamp, or a kernel
  // argument whose s_load the compiler hoists into the loop's preheader) shares
  // lgkmcnt with the LDS reads and completes out of order, which turns every
  // counted LDS wait into lgkmcnt(0): consume them here.
  const int relu = a.relu;
  asm volatile("" ::"s"(relu));
  start_stagger(a.stagger);
  unsigned long long t_start = 0, t_first = 0;
  if (a.stamps) {
    t_start = __builtin_amdgcn_s_memrealtime();
    asm volatile("" ::"s"(t_start));
  }

  // ---- input rows rs .. rs+nrows-1 (several images back to back when
  // PARTS == 1). Staged pixel = input (y, x) of the workgroup's image i; its
  // key K is chosen so that for output pixel p at tap (kh, kw) it is p + a tap
  // constant: consecutive along a fragment even where it wraps an output row.
  //   stride 1: K = (staged row)*W + x;
  //   stride 2: K = i*H*W + (((y+1)>>1) - r0)*W + ((x+1)>>1)
  //             ((y+1)>>1 is the output row for kh 0/1 and one less for kh 2).
  // Chunk c sits at physical chunk c ^ xswz(K). A ds_read_b128 16-lane group
  // holds fragment pixels 0-3,12-15 at k-group g and 4-11 at g^1 (g even):
  //  * pixels of >= 256 B fill a whole 64-bank window; with xswz = (K&7)<<1
  //    pixels j and j+8 (one of each set) share the pair index (c>>1)^(K&7)
  //    and differ in the low bit, and the 8 pair indices are distinct;
  //  * 128-B pixels (64 channels) take the window half given by the pixel's
  //    parity, which follows K's parity along a fragment (stride 2 stores each
  //    row's even columns first: consecutive outputs read alternating halves);
  //    within a half xswz = ((K>>1)&3)<<1 does the same pairing.
  // All 16 bank slots for any fragment offset. (The first layout, padded
  // column & 15 under an XOR, collided whenever a fragment started at an odd
  // key or wrapped a row: 39% of LDS cycles were bank conflicts.)
  // Instruction k = row*XI + j goes to wave k % 8.
  for (int k = wave; k < nrows * XI; k += 8) {
    const int i = k / XI, j = k - i * XI;
    const int ci = j * 64 + lane;  // chunk of the staged row
    const int q = ci / CPX, pp = ci - q * CPX;  // physical column, chunk
    const int x = S == 1 ? q : (q < WI / 2 ? 2 * q : 2 * (q - WI / 2) + 1);
    int K;
    if constexpr (S == 1) {
      K = i * W + x;
    } else {
      const int ii = PARTS == 1 ? i / HI : 0, y = PARTS == 1 ? i - ii * HI : rs + i;
      K = ii * (H * W) + (((y + 1) >> 1) - r0) * W + ((x + 1) >> 1);
    }
    const int pc = pp ^ xswz<CPX>(K);  // logical chunk at physical pp
    dma16(img + ((long)(rs + i) * WI + x) * CI + 8 * pc, xs + i * ROWB + j * 1024);
  }
  if (wave == 0 && lane < CPX) dma16(a.zero, xs + ZB);

  // ---- this wave's 32 weight rows of K-tile t -> its stage st (rows permuted,
  // chunks swizzled): per-lane byte offsets into the weights, the K-tile
  // advance in the scalar base
  uint32_t woff[GW], woffd[GW];
#pragma unroll
  for (int g = 0; g < GW; ++g) {
    const int ci = g * 64 + lane, n = ci >> 2, pc = ci & 3;
    woff[g] = (uint32_t)(((ch0 + perm32(n)) * (9 * CI) + 8 * wswz(n, pc)) * 2);
    woffd[g] = (uint32_t)(((ch0 + perm32(n)) * CI + 8 * wswz(n, pc)) * 2);
  }
  const bf16* wbase = a.w;
  auto load_wtile = [&](int t, int st) __attribute__((always_inline)) {
    if constexpr (WR) return;
    if (DS && t >= KT) {
#pragma unroll
      for (int g = 0; g < GW; ++g) dma16s(a.wd + (t - KT) * BK, woffd[g], wpriv + st * WST + g * 1024);
    } else {
#pragma unroll
      for (int g = 0; g < GW; ++g) dma16s(wbase + t * BK, woff[g], wpriv + st * WST + g * 1024);
    }
  };
  bf16x8 wq[WR ? PD : 1][NF];
  // fragment nf of K-tile t (the downsample's tiles follow the 3x3's): buffer
  // loads, lane offset in a VGPR and the fragment offset a scalar
  // (non-WR kernels get descriptors of null pointers they never use)
  // (a wave's NG groups are consecutive in the fragment-order array: group j
  // of the wave starts j * KT * 2 fragments after the first)
  const __amdgpu_buffer_rsrc_t wrs = wave_rsrc(a.wf + (long)(ch0 / 32) * KT * 2 * 512, WR ? NG * KT * 2 * 1024 : 0);
  const __amdgpu_buffer_rsrc_t wdrs =
      wave_rsrc(a.wdf + (long)(ch0 / 32) * CT * 2 * 512, (WR && DS) ? NG * CT * 2 * 1024 : 0);
  auto wfrag = [&](int t, int nf) __attribute__((always_inline)) {
    const bool d = DS && t >= KT;
    const int kt = d ? CT : KT, tt = d ? t - KT : t;
    return __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(
                                          d ? wdrs : wrs, lane * 16, ((nf >> 1) * kt * 2 + tt * 2 + (nf & 1)) * 1024,
                                          0));
  };
  if constexpr (WR) {
#pragma unroll
    for (int t = 0; t < PD - 1; ++t)
#pragma unroll
      for (int nf = 0; nf < NF; ++nf) wq[t][nf] = wfrag(t, nf);
  } else {
#pragma unroll
    for (int t = 0; t < ND - 1; ++t) load_wtile(t, t);
  }

  // ---- per-lane constants: pixel p = 16(wm*MF + f) + fr (clamped for padding
  // lanes / a dummy last fragment: they compute a duplicate, never stored).
  // xoff = the staged offset of the tap-(1,1) input pixel; its low 4 bits flag
  // the image's first/last row and column, whose outside taps read the zero
  // pixel (stride 2 never leaves the image at the bottom or right).
  int xoff[MF];
#pragma unroll
  for (int f = 0; f < MF; ++f) {
    const int p = min(16 * (wm * MF + f) + fr, npix - 1);
    const int pi = p % (HS * W), ii = p / (HS * W), prow = pi / W, pcol = pi - prow * W, r = r0 + prow;
    const int row = ii * HI + S * r - rs;  // (stride 2: even input column 2 pcol sits at slot pcol)
    xoff[f] = (row * WI + pcol) * PXB | (r == 0 ? 1 : 0) | (S == 1 && r == H - 1 ? 2 : 0) | (pcol == 0 ? 4 : 0) |
              (S == 1 && pcol == W - 1 ? 8 : 0);
    asm volatile("" : "+v"(xoff[f]));  // keep it live: rematerialising p / W in the loop cost ~100 VALU per K-tile
  }
  floatx4 acc[MF][NF], accd[DS ? MF : 1][NF];
#pragma unroll
  for (int f = 0; f < MF; ++f)
#pragma unroll
    for (int nf = 0; nf < NF; ++nf) acc[f][nf] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int f = 0; f < (DS ? MF : 1); ++f)
#pragma unroll
    for (int nf = 0; nf < NF; ++nf) accd[f][nf] = floatx4{0.f, 0.f, 0.f, 0.f};

  // per-tap fragment bases xa[f] and lane swizzle tsw = 16 fq ^ 16 xswz(K):
  // K = p + ktap with p & 15 == fr for every real pixel (fragments start at
  // multiples of 16), so it is one lane value per tap for all fragments
  // (clamped lanes read a permuted chunk of their clamped pixel: in bounds,
  // never stored)
  const int kbase = fr + (S == 1 ? (r0 - rs) * W : 0);
  int xa[MF], tsw = 0;
  auto set_tap = [&](int tap) __attribute__((always_inline)) {
    const int kh = tap / 3, kw = tap - kh * 3;
    const int tm = (kh == 0 ? 1 : 0) | (kh == 2 ? 2 : 0) | (kw == 0 ? 4 : 0) | (kw == 2 ? 8 : 0);
    // staged column offset of tap column kw (stride 2: odd columns start at WI/2)
    const int dq = S == 1 ? kw - 1 : (kw == 0 ? WI / 2 - 1 : kw == 1 ? 0 : WI / 2);
    const int toff = ((kh - 1) * WI + dq) * PXB;
#pragma unroll
    for (int f = 0; f < MF; ++f) xa[f] = (xoff[f] & tm) ? ZB : (xoff[f] & ~15) + toff;
    const int ktap = S == 1 ? (kh - 1) * W + kw - 1 : (kh == 2 ? W : 0) + (kw == 2 ? 1 : 0);
    tsw = (fq << 4) ^ (xswz<CPX>(kbase + ktap) << 4);
  };
  const uint32_t wlane = fr * (BK * 2) + (wswz(fr, fq) << 4);
  auto wread = [&](bf16x8* wf, int st) __attribute__((always_inline)) {
#pragma unroll
    for (int nf = 0; nf < NF; ++nf) wf[nf] = *(const bf16x8*)(wpriv + st * WST + nf * 16 * (BK * 2) + wlane);
  };
  // fragment f of the current tap's K-tile cc (the in-pixel offset is < PXB,
  // so the add is an OR)
  auto xread = [&](int f, int cc) __attribute__((always_inline)) {
    return *(const bf16x8*)(xs + xa[f] + (tsw ^ (cc * BK * 2)));
  };

  // ---- software-pipelined K loop (one 32-deep k-step per K-tile), no
  // workgroup barrier: the operands of K-tile t+1 are read while the MFMAs of t
  // run, each X fragment's next read right after its own MFMAs, the weight
  // fragments at the start of the tile. Iteration t first waits for the
  // wave's own DMA of t+1 (issued one iteration earlier), then refills the
  // stage of t-1 (read during t-2, consumed by t-1's MFMAs) with t+2.
  // PRIO (A/B): waves 4-7 (the second-dispatched half, the arbitration
  // loser of every SIMD pair) at priority 1 for the whole K loop
  if constexpr (PRIO)
    if (wave >= 4) __builtin_amdgcn_s_setprio(1);
  set_tap(0);
  if constexpr (WR)
    vm_wait<(PD - 1) * NF>();  // own input rows (the weight loads were issued after them)
  else
    vm_wait<(ND - 2) * GW>();  // own input rows and K-tile 0
  __builtin_amdgcn_s_barrier();  // every wave's input rows
  asm volatile("" ::: "memory");
  if (a.stamps) {
    t_first = __builtin_amdgcn_s_memrealtime();
    asm volatile("" ::"s"(t_first));
  }
  bf16x8 wf[NF], xf[MF];
  if constexpr (!WR) wread(wf, 0);
#pragma unroll
  for (int f = 0; f < MF; ++f) xf[f] = xread(f, 0);
  int st = 0;
  for (int tap = 0; tap < 9; ++tap) {
#pragma unroll
    for (int cc = 0; cc < CT; ++cc) {
      const int t = tap * CT + cc;
      if constexpr (WR) {
        if (t + PD - 1 < KT2)
#pragma unroll
          for (int nf = 0; nf < NF; ++nf) wq[(cc + PD - 1) % PD][nf] = wfrag(t + PD - 1, nf);
      } else {
        if (t + 1 < KT2) vm_wait<0>();
        if (t + ND - 1 < KT2) load_wtile(t + ND - 1, st == 0 ? ND - 1 : st - 1);
      }
      const int st1 = st == ND - 1 ? 0 : st + 1;
      // next K-tile's X: same tap at cc+1, or the next tap's first (the
      // final iteration re-reads a valid tile, unused; with DS it reads the
      // downsample's first, tap (1,1))
      if (cc + 1 == CT && tap + 1 < 9) set_tap(tap + 1);
      if (DS && cc + 1 == CT && tap == 8) set_tap(4);
      const int cn = cc + 1 == CT ? 0 : cc + 1;
      bf16x8 wn[NF];
      if constexpr (!WR) wread(wn, st1);
      // everything but the two weight reads just issued: the X fragments (read
      // during the previous K-tile) have landed. One wait instead of the
      // compiler's one per fragment.
      __builtin_amdgcn_s_waitcnt(0xC07F | ((WR ? 0 : NF) << 8));
#pragma unroll
      for (int f = 0; f < MF; ++f) {
#pragma unroll
        for (int nf = 0; nf < NF; ++nf)
          acc[f][nf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(WR ? wq[cc % PD][nf] : wf[nf], xf[f], acc[f][nf], 0, 0,
                                                               0);
        xf[f] = xread(f, cn);
      }
      if constexpr (!WR) __builtin_amdgcn_sched_group_barrier(0x100, NF, 0);
#pragma unroll
      for (int f = 0; f < MF; ++f) {
        __builtin_amdgcn_sched_group_barrier(0x008, NF, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      }
      if constexpr (!WR) {
#pragma unroll
        for (int nf = 0; nf < NF; ++nf) wf[nf] = wn[nf];
      }
      st = st1;
    }
  }
  if constexpr (DS) {  // the downsample's K-tiles, same pipeline
#pragma unroll
    for (int cc = 0; cc < CT; ++cc) {
      const int t = KT + cc;
      if constexpr (WR) {  // KT % PD == 0: tile t sits in slot cc % PD
        if (t + PD - 1 < KT2)
#pragma unroll
          for (int nf = 0; nf < NF; ++nf) wq[(cc + PD - 1) % PD][nf] = wfrag(t + PD - 1, nf);
      } else {
        if (t + 1 < KT2) vm_wait<0>();
        if (t + ND - 1 < KT2) load_wtile(t + ND - 1, st == 0 ? ND - 1 : st - 1);
      }
      const int st1 = st == ND - 1 ? 0 : st + 1;
      const int cn = cc + 1 == CT ? 0 : cc + 1;
      bf16x8 wn[NF];
      if constexpr (!WR) wread(wn, st1);
      __builtin_amdgcn_s_waitcnt(0xC07F | ((WR ? 0 : NF) << 8));
#pragma unroll
      for (int f = 0; f < MF; ++f) {
#pragma unroll
        for (int nf = 0; nf < NF; ++nf)
          accd[f][nf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(WR ? wq[cc % PD][nf] : wf[nf], xf[f], accd[f][nf], 0,
                                                                0, 0);
        xf[f] = xread(f, cn);
      }
      if constexpr (!WR) __builtin_amdgcn_sched_group_barrier(0x100, NF, 0);
#pragma unroll
      for (int f = 0; f < MF; ++f) {
        __builtin_amdgcn_sched_group_barrier(0x008, NF, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      }
      if constexpr (!WR) {
#pragma unroll
        for (int nf = 0; nf < NF; ++nf) wf[nf] = wn[nf];
      }
      st = st1;
    }
  }

  unsigned long long t_loop = 0;
  if (a.stamps) {
    t_loop = __builtin_amdgcn_s_memrealtime();
    asm volatile("" ::"s"(t_loop));
  }
  // ---- epilogue: lane holds channels ch0 + 8fq .. +7 of its pixel. All
  // residual loads are issued first (the operand registers are free now):
  // loaded one per fragment, each waited on before its store, they cost
  // 4-5 us per workgroup.
  // (NG = 2: the same for channel group j at +32 j, fragments 2j, 2j+1)
  const long base = ((long)b * H + r0) * W * CO + ch0 + 8 * fq;
  float bs[NG][8];
#pragma unroll
  for (int j = 0; j < NG; ++j)
#pragma unroll
    for (int e = 0; e < 8; ++e) bs[j][e] = a.bias[ch0 + 32 * j + 8 * fq + e];
  uint4 rv[MF][NG];
  if (a.res) {
#pragma unroll
    for (int f = 0; f < MF; ++f) {
      const int p = min(16 * (wm * MF + f) + fr, npix - 1);
#pragma unroll
      for (int j = 0; j < NG; ++j) rv[f][j] = *(const uint4*)(a.res + base + 32 * j + (long)p * CO);
    }
  }
  // fused avgpool: per-lane sums per image of the workgroup (PARTS == 1)
  // (whole images with one pixel group per wave: a wave's lanes see every
  // pixel of its images; the host allows the pool only on such variants)
  constexpr bool POOLABLE = G::PARTS == 1 && WM == 1;
  constexpr int PIMG = G::PARTS == 1 ? IMG : 1;
  float psum[NG][PIMG][8];
#pragma unroll
  for (int j = 0; j < NG; ++j)
#pragma unroll
    for (int i = 0; i < PIMG; ++i)
#pragma unroll
      for (int e = 0; e < 8; ++e) psum[j][i][e] = 0.f;
#pragma unroll
  for (int f = 0; f < MF; ++f) {
    const int p = 16 * (wm * MF + f) + fr;
    if (p >= npix) continue;
#pragma unroll
    for (int j = 0; j < NG; ++j) {
      const long off = base + 32 * j + (long)p * CO;
      float v[8];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[e] = acc[f][2 * j][e] + bs[j][e];
        v[4 + e] = acc[f][2 * j + 1][e] + bs[j][4 + e];
      }
      if (a.res) {
        float r[8];
        unpack8(rv[f][j], r);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += r[e];
      }
      const uint4 packed = pack8_relu(v, relu);
      if (a.out_inv_scale > 0.f) {  // e4m3 bytes at element offset off
        float q[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) q[e] = fminf((relu ? fmaxf(v[e], 0.f) : v[e]) * a.out_inv_scale, 448.f);
        u32x2s o;
        o.x = e4m3x4(q[0], q[1], q[2], q[3]);
        o.y = e4m3x4(q[4], q[5], q[6], q[7]);
        *(u32x2s*)((uint8_t*)a.y + off) = o;
      } else if (a.store_y) {
        *(uint4*)(a.y + off) = packed;
      }
      if constexpr (POOLABLE) {
        if (a.pool) {  // the bf16 activation's values, as the unfused avgpool reads them
          float q[8];
          unpack8(packed, q);
          const int im = PIMG == 1 ? 0 : p / (H * W);
#pragma unroll
          for (int i = 0; i < PIMG; ++i)
            if (i == im)
#pragma unroll
              for (int e = 0; e < 8; ++e) psum[j][i][e] += q[e];
        }
      }
    }
  }
  if constexpr (POOLABLE) {
    if (a.pool) {  // reduce over the 16 pixel lanes fr of each channel group fq
#pragma unroll
      for (int j = 0; j < NG; ++j)
#pragma unroll
        for (int i = 0; i < PIMG; ++i)
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            float t = psum[j][i][e];
            t += __shfl_xor(t, 8, 64);
            t += __shfl_xor(t, 4, 64);
            t += __shfl_xor(t, 2, 64);
            t += __shfl_xor(t, 1, 64);
            psum[j][i][e] = t * (1.f / (H * W));
          }
      if (fr == 0 && (WM == 1 || wm == 0)) {
#pragma unroll
        for (int j = 0; j < NG; ++j)
#pragma unroll
          for (int i = 0; i < PIMG; ++i)
            if (i < nimg) {
              *(uint4*)(a.pool + (long)(b + i) * CO + ch0 + 32 * j + 8 * fq) = pack8(psum[j][i]);
            }
      }
    }
  }
  if constexpr (DS) {
#pragma unroll
    for (int j = 0; j < NG; ++j) {
      float bd[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) bd[e] = a.bd[ch0 + 32 * j + 8 * fq + e];
#pragma unroll
      for (int f = 0; f < MF; ++f) {
        const int p = 16 * (wm * MF + f) + fr;
        if (p >= npix) continue;
        float v[8];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[e] = accd[f][2 * j][e] + bd[e];
          v[4 + e] = accd[f][2 * j + 1][e] + bd[4 + e];
        }
        *(uint4*)(a.yd + base + 32 * j + (long)p * CO) = pack8(v);
      }
    }
  }
  if (a.stamps && tid == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    unsigned long long* sp = a.stamps + blockIdx.x * 4;
    sp[0] = t_start;
    sp[1] = t_first;
    sp[2] = t_loop;
    sp[3] = __builtin_amdgcn_s_memrealtime();
  }
}

template <int H, int W, int CI, int CO, int HS, int IMG, int NSP, int WM, int S, bool WR = false, int PD = 4,
          int NG = 1, int PRIO = 0>
void launch_stream(const StreamConvArgs& a, hipStream_t s) {
  using G = StreamGeom<H, W, CI, HS, IMG, S, 3>;
  constexpr size_t lds = WR ? (size_t)G::XBYTES : G::LDS;
  static_assert(lds <= 160 * 1024, "LDS budget");
  const int grid = (a.B + IMG - 1) / IMG * (H / HS) * NSP;
  if constexpr (WR) {
    if constexpr (S == 2) {
      if (a.yd) {
        hipLaunchKernelGGL((conv3x3_stream_kernel<H, W, CI, CO, HS, IMG, NSP, WM, S, 3, true, true, PD, NG, PRIO>),
                           dim3(grid), dim3(512), lds, s, a);
        return;
      }
    }
      hipLaunchKernelGGL((conv3x3_stream_kernel<H, W, CI, CO, HS, IMG, NSP, WM, S, 3, false, true, PD, NG, PRIO>),
                         dim3(grid), dim3(512), lds, s, a);
    return;
  } else {
    if constexpr (S == 2) {
      if (a.yd) {
        hipLaunchKernelGGL((conv3x3_stream_kernel<H, W, CI, CO, HS, IMG, NSP, WM, S, 3, true, false>), dim3(grid),
                           dim3(512), lds, s, a);
        return;
      }
    }
    hipLaunchKernelGGL((conv3x3_stream_kernel<H, W, CI, CO, HS, IMG, NSP, WM, S, 3, false, false>), dim3(grid),
                       dim3(512), lds, s, a);
  }
}

// Tuning hook for tools/conv_bench.py A/B runs (0 = the default kernels), bits:
// 1 = the 14x14x256 register-weight kernel with a 2-deep weight ring (PD 2);
// 2 = the stride-2 register-weight 28x28x128 kernel with two channel groups
// per wave (NG 2); 4 = the stride-2 14x14x256 one with one (NG 1, half the
// channels per workgroup); 8 = the 7x7x512 stride-1 register-weight kernel
// with an 8-deep weight ring (16 deep spills); 32 = waves 4-7 at priority 1 in
// the register-weight kernels of layers 3-4.
std::atomic<int> g_stream_variant{0};

}  // namespace

void conv3x3_stream_set_variant(int v) { g_stream_variant = v; }

// Whole-image workgroups (the fused avgpool): layer4's 7x7x512 stride-1 conv.
bool conv3x3_stream_pool_supported(int Hin, int Win, int Cin, int Cout, int stride) {
  return stride == 1 && Hin == 7 && Win == 7 && Cin == 512 && Cout == 512;
}

bool conv3x3_stream_supported(int Hin, int Win, int Cin, int Cout, int stride) {
  if (stride == 1)
    return Cin == Cout && ((Hin == 28 && Win == 28 && Cin == 128) || (Hin == 14 && Win == 14 && Cin == 256) ||
                           (Hin == 7 && Win == 7 && Cin == 512) || (Hin == 56 && Win == 56 && Cin == 64));
  if (stride == 2)
    return (Cout == 2 * Cin && ((Hin == 56 && Win == 56 && Cin == 64) || (Hin == 28 && Win == 28 && Cin == 128) ||
                                (Hin == 14 && Win == 14 && Cin == 256))) ||
           // ResNet50 layer2.0.conv2 (the bottleneck's strided 3x3)
           (Cout == Cin && Hin == 56 && Win == 56 && Cin == 128);
  return false;
}

// Register weights only where the LDS-ring variant leaves VGPRs for the ring:
// the 28x28x128 / 14x14x256 kernels (240 / 248 VGPRs) spill 17-57 VGPRs with
// even a 2-deep register ring (pointer or buffer-load addressing) and ran
// 1.7-2x slower (profiles/r1_stream_conv.log).
bool conv3x3_stream_uses_frag(int Hin, int Win, int Cin, int Cout, int stride) {
  // 56x56x64 / s2 (K-tiles per tap = 2, so a 2-deep ring): 83.8 vs 71.0 us
  // with the LDS ring (a 4-deep ring with all 20 K-tiles unrolled: 73.8),
  // not used; 28x28x128 / s2: 48.6 vs 53.6 us
  if (stride == 2)
    return (Cout == 2 * Cin && ((Hin == 28 && Win == 28 && Cin == 128) || (Hin == 14 && Cin == 256))) ||
           (Cout == Cin && Hin == 56 && Win == 56 && Cin == 128);
  // (28x28x128 in quarter images and 14x14x256 in 2 channel splits, both 7
  // fragments per wave so the register ring fits, measured 70.2 / 60.2 vs
  // 67.9 / 56.4 us with the LDS ring: kept out)
  // 14x14x256 with two channel groups per wave (NG = 2: WM = 2 pixel halves x
  // 4 x 64 channels, 7 fragments per wave, X reads per MFMA halved)
  return stride == 1 && Cin == Cout && ((Hin == 7 && Win == 7 && Cin == 512) || (Hin == 14 && Win == 14 && Cin == 256));
}

void conv3x3_stream(const void* x, const void* w, const float* bias, const void* res, void* y, const void* zero,
                    int B, int Hin, int Win, int Cin, int Cout, int stride, bool relu, hipStream_t s,
                    unsigned long long* stamps, const void* wd, const float* bd, void* yd, const void* wfrag,
                    const void* wdfrag, void* pool, bool store_y, float out_inv_scale) {
  if (B <= 0) return;
  if (out_inv_scale > 0.f && (res || pool || yd || !store_y))
    throw std::invalid_argument("conv3x3_stream: e4m3 output without residual, pool or downsample only");
  if ((pool || !store_y) && !conv3x3_stream_pool_supported(Hin, Win, Cin, Cout, stride))
    throw std::invalid_argument("conv3x3_stream: fused avgpool needs whole-image workgroups");
  if (pool && ((uintptr_t)pool & 15)) throw std::invalid_argument("conv3x3_stream: misaligned pool");
  if (!conv3x3_stream_supported(Hin, Win, Cin, Cout, stride))
    throw std::invalid_argument("conv3x3_stream: unsupported shape");
  if (!x || !w || !bias || !y || !zero ||
      (((uintptr_t)x | (uintptr_t)w | (uintptr_t)y | (uintptr_t)zero | (uintptr_t)res) & 15))
    throw std::invalid_argument("conv3x3_stream: null / misaligned operand");
  StreamConvArgs a;
  a.x = (const bf16*)x;
  a.w = (const bf16*)w;
  a.bias = bias;
  a.res = (const bf16*)res;
  a.y = (bf16*)y;
  a.zero = (const bf16*)zero;
  a.B = B;
  a.relu = relu;
  a.stamps = stamps;
  a.stagger = kernel_stagger(kStagStream);
  a.wd = (const bf16*)wd;
  a.bd = bd;
  a.yd = (bf16*)yd;
  a.wf = (const bf16*)wfrag;
  a.wdf = (const bf16*)wdfrag;
  a.pool = (bf16*)pool;
  a.store_y = store_y ? 1 : 0;
  a.out_inv_scale = out_inv_scale > 0.f ? out_inv_scale : 0.f;
  if (wfrag && (!conv3x3_stream_uses_frag(Hin, Win, Cin, Cout, stride) || ((uintptr_t)wfrag & 15) ||
                (yd && (!wdfrag || ((uintptr_t)wdfrag & 15)))))
    throw std::invalid_argument("conv3x3_stream: no register-weight variant for this call");
  if (yd && (stride != 2 || !wd || !bd || (((uintptr_t)wd | (uintptr_t)yd) & 15)))
    throw std::invalid_argument("conv3x3_stream: fused downsample needs stride 2 and aligned wd / yd");
  // LDS per workgroup: staged input rows + zero pixel + 8 waves x 3 x 2 KB weight stages
  if (stride == 1 && Cin == 64)  // layer1: 8-row strips (10 x 56 x 128 B = 70 KB), 4 pixel x 2 channel groups
    launch_stream<56, 56, 64, 64, 8, 1, 1, 4, 1>(a, s);
  else if (stride == 1 && Cin == 128)  // layer2: half an image (15 x 28 x 256 B = 105 KB)
    launch_stream<28, 28, 128, 128, 14, 1, 1, 2, 1>(a, s);
  else if (stride == 1 && Cin == 256 && wfrag) {  // layer3, register weights, 2 pixel halves x 4 groups of 64 channels
    if (g_stream_variant & 1)  // (tests: a 2-deep weight ring, the same MFMA order)
      launch_stream<14, 14, 256, 256, 14, 1, 1, 2, 1, true, 2, 2>(a, s);
    else
      launch_stream<14, 14, 256, 256, 14, 1, 1, 2, 1, true, 4, 2>(a, s);
  }
  else if (stride == 1 && Cin == 256)  // layer3: a whole image (14 x 14 x 512 B = 98 KB)
    launch_stream<14, 14, 256, 256, 14, 1, 1, 1, 1>(a, s);
  else if (stride == 1 && wfrag) {  // layer4, weights in fragment order straight into VGPRs
    // (two 64-channel groups per wave measured slower here: 2 images x 2
    // pixel halves 58.7 us, 1 image x 8 groups 60.9 us vs 53.0 us)
    launch_stream<7, 7, 512, 512, 7, 2, 2, 1, 1, true>(a, s);
  }
  else if (stride == 1)  // layer4: two whole images x half the output channels (2 x 49 x 1 KB = 98 KB)
    launch_stream<7, 7, 512, 512, 7, 2, 2, 1, 1>(a, s);
  else if (Cin == 128 && Hin == 56 && wfrag)  // ResNet50 layer2.0.conv2: 4 output rows (9 x 56 x 256 B = 129 KB)
    launch_stream<28, 28, 128, 128, 4, 1, 1, 2, 2, true>(a, s);
  else if (Cin == 128 && Hin == 56)  // the same with the LDS weight ring: 2 output rows (5 rows = 72 KB + 48 KB)
    launch_stream<28, 28, 128, 128, 2, 1, 1, 2, 2>(a, s);
  else if (Cin == 64)  // layer2.0.conv1: a quarter image (15 x 56 x 128 B = 105 KB)
    launch_stream<28, 28, 64, 128, 7, 1, 1, 2, 2>(a, s);
  else if (Cin == 128 && wfrag) {
    // variant bit 2: two 32-channel groups per wave (2 pixel halves x 4 x 64
    // channels, an X fragment read feeds 4 MFMAs instead of 2; 8 fragments
    // for the 7 of a half image): 50.7 vs 49.4 us at B = 256, not used
    if (g_stream_variant & 2)
      launch_stream<14, 14, 128, 256, 7, 1, 1, 2, 2, true, 4, 2>(a, s);
    else
      launch_stream<14, 14, 128, 256, 7, 1, 1, 1, 2, true>(a, s);
  }
  else if (Cin == 128)  // layer3.0.conv1: half an image (15 x 28 x 256 B = 105 KB)
    launch_stream<14, 14, 128, 256, 7, 1, 1, 1, 2>(a, s);
  else if (wfrag) {
    // a whole image x all 512 channels, 64 per wave (NG 2): 43.0 vs 49.0 us
    // at B = 256 with the fused downsample for half the channels per
    // workgroup, 32 per wave (variant bit 4; profiles/r3_stream_s2_ng2.txt)
    if (g_stream_variant & 4)
      launch_stream<7, 7, 256, 512, 7, 1, 2, 1, 2, true>(a, s);
    else
      launch_stream<7, 7, 256, 512, 7, 1, 1, 1, 2, true, 4, 2>(a, s);
  }
  else  // layer4.0.conv1: a whole image (14 x 14 x 512 B = 98 KB) x half the output channels
    launch_stream<7, 7, 256, 512, 7, 1, 2, 1, 2>(a, s);
  DMLC_HIP_CHECK(hipGetLastError());
}

}  // namespace dmlc
