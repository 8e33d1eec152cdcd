// Direct 3x3 / stride 1 / pad 1 convolution with the input image resident in
// LDS, for ResNet18 layer2 (28x28x128: layer2.0.conv2, layer2.1.conv{1,2}) and
// layer3 (14x14x256: layer3.0.conv2, layer3.1.conv{1,2}), BN folded, optional
// residual, ReLU.
//
// Reference equivalent: those convs + bn + (residual) + relu of
// tch::vision::resnet18, run per query by `forward_t` at src/services.rs:493.
// As an implicit GEMM (conv_igemm.hip) every output tile re-fetches its 3x3
// input window per tap: 9x the input bytes through L2, and in the model the
// input is cold (written by the previous layer), so these convs ran at 113-128
// us against 85 us on L2-hot inputs. Here one workgroup owns HS output rows of
// one image (layer2: half an image, 392 pixels; layer3: the whole image, 196):
//
//  * Its input rows (the strip plus the halo rows inside the image) go HBM ->
//    LDS once by LDS-DMA and stay resident; taps that fall outside the image
//    read one zero pixel instead of staged zero padding. Chunks are XOR-
//    swizzled per pixel (see the staging loop) so every fragment read is
//    bank-conflict free and costs one VALU add.
//  * The folded weights (C x 9C bf16, 295 KB / 1.2 MB, shared by every CU and
//    L2-resident) stream through LDS in 32-deep K-tiles. Every wave streams
//    just the 32 output-channel rows it uses through a private 3-stage LDS-DMA
//    ring and waits only on its own vmcnt: the K loop has no workgroup
//    barrier. (With one shared ring the per-K-tile barrier, and the LDS read
//    latency it exposed, held the loop at ~50% MFMA busy: without MFMAs the
//    barrier/read skeleton alone took 35 of 60 us.)
//  * 8 waves (2 per SIMD) = WM pixel groups x 8/WM channel groups of 32 (2 N
//    fragments of 16), 13 pixel fragments each: layer2 WM=2 (its two pixel
//    halves each stream the channel group's rows), layer3 WM=1. D = W x X. The
//    weight rows are permuted when staged (row 16nf + r of a wave's tile holds
//    channel 8(r>>2) + 4nf + (r&3) of its group), so a lane ends with 8
//    consecutive output channels of one pixel: 16-B residual loads and stores.
//  * The K loop is software-pipelined: the operands of K-tile t+1 are read
//    while the MFMAs of t run.
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
  const bf16* x;      // [B, H, W, C]
  const bf16* w;      // [C, 9*C], k = (kh*3 + kw)*C + c
  const float* bias;  // [C]
  const bf16* res;    // [B, H, W, C] or null
  bf16* y;            // [B, H, W, C]
  const bf16* zero;   // >= 16 zero bytes
  int B;
  int relu;
  unsigned long long* stamps;  // debug: per-workgroup phase stamps (100 MHz), or null
};

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

// Geometry shared by the kernel and its launcher: a workgroup owns HS output
// rows of one image (PARTS = H / HS > 1), or IMG whole images (PARTS == 1),
// and C / NSP of the output channels.
template <int H, int W, int C, int HS, int IMG, int ND>
struct StreamGeom {
  static constexpr int PARTS = H / HS;
  static_assert(PARTS == 1 || IMG == 1, "several images per workgroup only as whole images");
  static constexpr int XR = PARTS == 1 ? IMG * H : PARTS == 2 ? HS + 1 : HS + 2;  // max staged rows
  static constexpr int PXB = C * 2;                    // bytes per pixel
  static constexpr int ROWB = W * PXB;                 // bytes per staged row
  static constexpr int ZB = XR * ROWB;                 // zero pixel
  static constexpr int XBYTES = ZB + PXB;              // input region
  static constexpr int WST = 32 * 32 * 2;              // a wave's weight stage: 32 rows x 32 k
  static constexpr size_t LDS = (size_t)XBYTES + (size_t)8 * ND * WST;
};

// One workgroup = HS output rows x W columns of one image (or IMG images),
// C / NSP output channels.
template <int H, int W, int C, int HS, int IMG, int NSP, int WM, int ND>
__global__ __launch_bounds__(512, 1) void conv3x3_stream_kernel(StreamConvArgs a) {
  using G = StreamGeom<H, W, C, HS, IMG, ND>;
  constexpr int BK = 32;                     // K-tile depth = one MFMA k-step
  constexpr int NPIX = IMG * HS * W;         // output pixels per workgroup (the last group may have fewer)
  constexpr int MFT = (NPIX + 15) / 16;      // pixel fragments (the last one partly padding)
  constexpr int MF = (MFT + WM - 1) / WM;    // per wave
  constexpr int WN = 32;                     // channels per wave
  constexpr int NF = 2;                      // N fragments per wave
  constexpr int PXB = G::PXB, ROWB = G::ROWB, ZB = G::ZB, WST = G::WST;
  constexpr int CPX = C / 8;                 // 16-B chunks per pixel
  constexpr int XI = W * CPX / 64;           // LDS-DMA instructions per input row
  constexpr int KT = 9 * C / BK;             // K-tiles
  constexpr int CT = C / BK;                 // K-tiles per tap
  constexpr int GW = WST / 1024;             // weight DMA instructions per wave per K-tile
  static_assert(C == 8 / WM * WN * NSP && W * CPX % 64 == 0 && H % HS == 0 && PXB >= 256, "geometry");
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
  const int rs = PARTS == 1 ? 0 : max(r0 - 1, 0);
  const int nrows = PARTS == 1 ? nimg * H : min(r0 + HS, H - 1) - rs + 1;  // staged input rows
  const int npix = IMG == 1 ? NPIX : nimg * HS * W;
  const int ch0 = ns * (C / NSP) + wc * WN;                 // this wave's first output channel
  const bf16* img = a.x + (long)b * H * W * C;
  // A scalar memory op still pending in the loop (a debug stamp, or a kernel
  // argument whose s_load the compiler hoists into the loop's preheader) shares
  // lgkmcnt with the LDS reads and completes out of order, which turns every
  // counted LDS wait into lgkmcnt(0): consume them here.
  const int relu = a.relu;
  asm volatile("" ::"s"(relu));
  unsigned long long t_start = 0, t_first = 0;
  if (a.stamps) {
    t_start = __builtin_amdgcn_s_memrealtime();
    asm volatile("" ::"s"(t_start));
  }

  // ---- input rows rs .. rs+nrows-1. Staged pixel (i, q) has key K = i*W + q,
  // which for output pixel p at tap (kh, kw) is p + const: consecutive along a
  // fragment even where it wraps an output row. Chunk c sits at physical chunk
  // c ^ ((K & 7) << 1). A ds_read_b128 16-lane group holds fragment pixels
  // 0-3,12-15 at k-group g and 4-11 at g^1 (g even): pixels j and j+8 (one of
  // each set) share the pair index (c>>1) ^ (K&7) and differ in the low bit,
  // and the 8 pair indices are distinct: all 16 bank slots for any fragment
  // offset. (The first layout, padded column & 15 under an XOR, collided
  // whenever a fragment started at an odd key or wrapped a row: 39% of LDS
  // cycles were bank conflicts.) A read is one VALU add off a per-tap base.
  // (Pixels padded by 32 B put chunk c of key K in slot (2K + c) mod 16,
  // also conflict-free and with reads at immediate offsets, but the fully
  // unrolled loop that needs spilled registers.) Instruction k = row*XI + j
  // goes to wave k % 8.
  for (int k = wave; k < nrows * XI; k += 8) {
    const int i = k / XI, j = k - i * XI;
    const int ci = j * 64 + lane;  // chunk of the staged row
    const int q = ci / CPX, pp = ci - q * CPX;
    const int pc = pp ^ (((i * W + q) & 7) << 1);  // logical chunk at physical pp
    dma16(img + ((long)(rs + i) * W + q) * C + 8 * pc, xs + i * ROWB + j * 1024);
  }
  if (wave == 0 && lane < CPX) dma16(a.zero, xs + ZB);

  // ---- this wave's 32 weight rows of K-tile t -> its stage st (rows permuted,
  // chunks swizzled): per-lane byte offsets into the weights, the K-tile
  // advance in the scalar base
  uint32_t woff[GW];
#pragma unroll
  for (int g = 0; g < GW; ++g) {
    const int ci = g * 64 + lane, n = ci >> 2, pc = ci & 3;
    woff[g] = (uint32_t)(((ch0 + perm32(n)) * (9 * C) + 8 * wswz(n, pc)) * 2);
  }
  const bf16* wbase = a.w;
  auto load_wtile = [&](int t, int st) __attribute__((always_inline)) {
#pragma unroll
    for (int g = 0; g < GW; ++g) dma16s(wbase + t * BK, woff[g], wpriv + st * WST + g * 1024);
  };
#pragma unroll
  for (int t = 0; t < ND - 1; ++t) load_wtile(t, t);

  // ---- per-lane constants: pixel p = 16(wm*MF + f) + fr (clamped for padding
  // lanes / a dummy last fragment: they compute a duplicate, never stored).
  // The swizzle term ((p + const) & 7) << 5 has p & 7 == fr & 7 for every real
  // pixel (fragments start at multiples of 16), so it is one lane value per
  // tap for all fragments (clamped lanes read a permuted chunk of their
  // clamped pixel: in bounds, never stored). The low 4 bits of xoff flag the
  // image's first/last row and column, whose outside taps read the zero pixel.
  // Several images are staged back to back, so keys stay consecutive.
  int xoff[MF];
#pragma unroll
  for (int f = 0; f < MF; ++f) {
    const int p = min(16 * (wm * MF + f) + fr, npix - 1);
    const int pi = p % (HS * W), prow = pi / W, pcol = pi - prow * W, r = r0 + prow;
    xoff[f] = (p - pi + (r - rs) * W + pcol) * PXB | (r == 0 ? 1 : 0) | (r == H - 1 ? 2 : 0) | (pcol == 0 ? 4 : 0) |
              (pcol == W - 1 ? 8 : 0);
    asm volatile("" : "+v"(xoff[f]));  // keep it live: rematerialising p / W in the loop cost ~100 VALU per K-tile
  }
  floatx4 acc[MF][NF];
#pragma unroll
  for (int f = 0; f < MF; ++f)
#pragma unroll
    for (int nf = 0; nf < NF; ++nf) acc[f][nf] = floatx4{0.f, 0.f, 0.f, 0.f};

  // per-tap fragment bases xa[f] and lane swizzle tsw = 16 fq ^ ((K & 7) << 5)
  const int key = 32 * ((fr + (r0 - rs) * W) & 7);
  int xa[MF], tsw = 0;
  auto set_tap = [&](int tap) __attribute__((always_inline)) {
    const int kh = tap / 3, kw = tap - kh * 3;
    const int tm = (kh == 0 ? 1 : 0) | (kh == 2 ? 2 : 0) | (kw == 0 ? 4 : 0) | (kw == 2 ? 8 : 0);
    const int toff = ((kh - 1) * W + (kw - 1)) * PXB;
#pragma unroll
    for (int f = 0; f < MF; ++f) xa[f] = (xoff[f] & tm) ? ZB : (xoff[f] & ~15) + toff;
    tsw = (fq << 4) ^ ((key + 32 * ((kh - 1) * W + kw - 1)) & 0xE0);
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
  set_tap(0);
  vm_wait<(ND - 2) * GW>();  // own input rows and K-tile 0
  __builtin_amdgcn_s_barrier();  // every wave's input rows
  asm volatile("" ::: "memory");
  if (a.stamps) {
    t_first = __builtin_amdgcn_s_memrealtime();
    asm volatile("" ::"s"(t_first));
  }
  bf16x8 wf[NF], xf[MF];
  wread(wf, 0);
#pragma unroll
  for (int f = 0; f < MF; ++f) xf[f] = xread(f, 0);
  int st = 0;
  for (int tap = 0; tap < 9; ++tap) {
#pragma unroll
    for (int cc = 0; cc < CT; ++cc) {
      const int t = tap * CT + cc;
      if (t + 1 < KT) vm_wait<0>();
      if (t + ND - 1 < KT) load_wtile(t + ND - 1, st == 0 ? ND - 1 : st - 1);
      const int st1 = st == ND - 1 ? 0 : st + 1;
      // next K-tile's X: same tap at cc+1, or the next tap's first (the
      // final iteration re-reads a valid tile, unused)
      if (cc + 1 == CT && tap + 1 < 9) set_tap(tap + 1);
      const int cn = cc + 1 == CT ? 0 : cc + 1;
      bf16x8 wn[NF];
      wread(wn, st1);
      // everything but the two weight reads just issued: the X fragments (read
      // during the previous K-tile) have landed. One wait instead of the
      // compiler's one per fragment.
      __builtin_amdgcn_s_waitcnt(0xC07F | (NF << 8));
#pragma unroll
      for (int f = 0; f < MF; ++f) {
#pragma unroll
        for (int nf = 0; nf < NF; ++nf)
          acc[f][nf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[nf], xf[f], acc[f][nf], 0, 0, 0);
        xf[f] = xread(f, cn);
      }
      __builtin_amdgcn_sched_group_barrier(0x100, NF, 0);
#pragma unroll
      for (int f = 0; f < MF; ++f) {
        __builtin_amdgcn_sched_group_barrier(0x008, NF, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      }
#pragma unroll
      for (int nf = 0; nf < NF; ++nf) wf[nf] = wn[nf];
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
  const long base = ((long)b * H + r0) * W * C + ch0 + 8 * fq;
  float bs[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) bs[e] = a.bias[ch0 + 8 * fq + e];
  uint4 rv[MF];
  if (a.res) {
#pragma unroll
    for (int f = 0; f < MF; ++f) {
      const int p = min(16 * (wm * MF + f) + fr, npix - 1);
      rv[f] = *(const uint4*)(a.res + base + (long)p * C);
    }
  }
#pragma unroll
  for (int f = 0; f < MF; ++f) {
    const int p = 16 * (wm * MF + f) + fr;
    if (p >= npix) continue;
    const long off = base + (long)p * C;
    float v[8];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      v[e] = acc[f][0][e] + bs[e];
      v[4 + e] = acc[f][1][e] + bs[4 + e];
    }
    if (a.res) {
      float r[8];
      unpack8(rv[f], r);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] += r[e];
    }
    if (relu) {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = fmaxf(v[e], 0.f);
    }
    *(uint4*)(a.y + off) = pack8(v);
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

template <int H, int W, int C, int HS, int IMG, int NSP, int WM>
void launch_stream(const StreamConvArgs& a, hipStream_t s) {
  constexpr size_t lds = StreamGeom<H, W, C, HS, IMG, 3>::LDS;
  static_assert(lds <= 160 * 1024, "LDS budget");
  const int grid = (a.B + IMG - 1) / IMG * (H / HS) * NSP;
  hipLaunchKernelGGL((conv3x3_stream_kernel<H, W, C, HS, IMG, NSP, WM, 3>), dim3(grid), dim3(512), lds, s, a);
}

}  // namespace

bool conv3x3_stream_supported(int H, int W, int Cin, int Cout) {
  return Cin == Cout && ((H == 28 && W == 28 && Cin == 128) || (H == 14 && W == 14 && Cin == 256) ||
                         (H == 7 && W == 7 && Cin == 512));
}

void conv3x3_stream(const void* x, const void* w, const float* bias, const void* res, void* y, const void* zero,
                    int B, int H, int W, int C, bool relu, hipStream_t s, unsigned long long* stamps) {
  if (B <= 0) return;
  if (!conv3x3_stream_supported(H, W, C, C)) throw std::invalid_argument("conv3x3_stream: unsupported shape");
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
  if (C == 128)  // layer2: half an image per workgroup (15 x 28 x 256 B = 105 KB) + 8 x 3 x 2 KB weight stages
    launch_stream<28, 28, 128, 14, 1, 1, 2>(a, s);
  else if (C == 256)  // layer3: a whole image per workgroup (14 x 14 x 512 B = 98 KB) + 8 x 3 x 2 KB weight stages
    launch_stream<14, 14, 256, 14, 1, 1, 1>(a, s);
  else  // layer4: two whole images x half the output channels per workgroup (2 x 49 x 1 KB = 98 KB) + rings
    launch_stream<7, 7, 512, 7, 2, 2, 1>(a, s);
  DMLC_HIP_CHECK(hipGetLastError());
}

}  // namespace dmlc
