// Direct 3x3 / stride 1 / pad 1 convolution for 128-channel 28x28 layers
// (ResNet layer2: layer2.0.conv2, layer2.1.conv{1,2}), BN folded, optional
// residual, ReLU.
//
// Reference equivalent: those convs + bn + (residual) + relu of
// tch::vision::resnet18, run per query by `forward_t` at src/services.rs:493.
// As an implicit GEMM (conv_igemm.hip) every output tile re-fetches its 3x3
// input window per tap: 9x the input bytes through L2, and in the model the
// input is cold (written by the previous layer), so these convs ran at 113-128
// us against 85 us on L2-hot inputs. Here one workgroup owns half an image
// (14 output rows = 392 pixels = 25 fragments of 16):
//
//  * Its 16 input rows (with the halo; zero rows/columns from a zero page) go
//    HBM -> LDS once by LDS-DMA and stay resident (120 KB). Pixel rows are
//    256 B (16 chunks of 8 channels); chunk c of padded column q sits at
//    physical chunk c ^ (q & 15), so the 16 pixels of a fragment read spread
//    over all 16 bank slots.
//  * The folded weights (128 x 1152 bf16 = 295 KB, shared by every CU and
//    L2-resident) stream once per workgroup through a 2-stage LDS-DMA ring of
//    64-deep K-tiles (128 rows x 128 B, chunks XOR-swizzled by (row>>1)&7 as
//    in conv_igemm.hip); a K-tile is 52 MFMAs per wave, 2 waves per SIMD: long enough to hide
//    the next tile's L2 fetch. (A 4-row step variant re-streamed the weights
//    7x per image and was L2-bound at 115 us.)
//  * 8 waves (2 per SIMD: one's LDS reads hide under the other's MFMAs) = 2
//    pixel halves (13 fragments) x 4 channel quarters (2 N fragments of 16);
//    with all 25 fragments in one wave the accumulators took 512 registers
//    and every MFMA pair waited on its own LDS read. D = W x X. The
//    weight rows are permuted when staged (LDS row 32w + 16nf + r holds
//    channel 32w + 8(r>>2) + 4nf + (r&3)), so a lane ends with 8 consecutive
//    output channels of one pixel: 16-B residual loads and output stores.
#include "common.h"
#include "kernels.h"

namespace dmlc {

namespace {

typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef const __attribute__((address_space(1))) void* gbl_ptr_t;

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
  int relu;
};

// Weight-row permutation: LDS row n of wave group g = n / WN (WN = 16*NF
// channels per wave), n_local = 16*nf + r, holds output channel
// g*WN + 32*(nf>>1) + 8*(r>>2) + 4*(nf&1) + (r&3): the lane with accumulator
// rows 4fq..4fq+3 of fragments (2j, 2j+1) then owns 8 consecutive channels
// g*WN + 32j + 8fq .. +7.
template <int WN>
__device__ __forceinline__ int perm_row(int n) {
  const int g = n / WN, nl = n % WN, nf = nl >> 4, r = nl & 15;
  return g * WN + 32 * (nf >> 1) + 8 * (r >> 2) + 4 * (nf & 1) + (r & 3);
}

// Weight-stage chunk swizzle (physical 16-B chunk of logical chunk c, row n):
// 128-B rows (BK = 64): c ^ ((n>>1)&7) as conv_igemm.hip; 64-B rows (BK =
// 32): c ^ (3*((n>>2)&1)) as conv_bigtile.hip. Both conflict-free for the
// fragment reads (lane reads chunk fq of row base+fr, base % 16 == 0).
template <int BK>
__device__ __forceinline__ int wswz(int n, int c) {
  if constexpr (BK == 64)
    return c ^ ((n >> 1) & 7);
  else
    return c ^ (3 * ((n >> 2) & 1));
}

// One workgroup = HS output rows x W columns of one image, all C channels;
// 8 waves = 2 pixel halves x 4 channel quarters.
template <int H, int W, int C, int HS, int BK>
__global__ __launch_bounds__(512, 1) void conv3x3_stream_kernel(StreamConvArgs a) {
  constexpr int NPIX = HS * W;               // output pixels per workgroup
  constexpr int MFT = (NPIX + 15) / 16;      // pixel fragments (the last one partly padding)
  constexpr int MF = (MFT + 1) / 2;          // per wave (2 pixel halves)
  constexpr int WN = C / 4;                  // channels per wave
  constexpr int NF = WN / 16;                // N fragments per wave
  constexpr int XR = HS + 2;                 // resident input rows (with the halo)
  constexpr int Q = W + 2;                   // padded columns
  constexpr int CPX = C / 8;                 // 16-B chunks per pixel
  constexpr int ROWB = Q * C * 2;            // bytes per staged input row
  constexpr int XI = (Q * CPX + 63) / 64;    // LDS-DMA instructions per input row
  constexpr int KT = 9 * C / BK;             // K-tiles
  constexpr int CT = C / BK;                 // K-tiles per tap
  constexpr int WCH = BK / 8;                // 16-B chunks per weight row
  constexpr int WSTAGE = C * BK * 2;         // bytes per weight stage
  constexpr int GW = C * WCH / 64 / 8;       // weight DMA instructions per wave per K-tile
  static_assert(C % 64 == 0 && CPX >= 16 && NF % 2 == 0 && H % HS == 0, "geometry");
  static_assert(C * WCH % 512 == 0, "weight stage splits into 8 waves x 64 lanes");

  extern __shared__ __attribute__((aligned(16))) uint4 smem[];
  char* xs = (char*)smem;
  char* wring = xs + XR * ROWB;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int mh = wave & 1, wn = wave >> 1;  // pixel half, channel quarter
  const int fr = lane & 15, fq = lane >> 4;
  constexpr int PARTS = H / HS;
  const int b = blockIdx.x / PARTS, part = blockIdx.x - b * PARTS;
  const int r0 = part * HS;  // first output row
  const bf16* img = a.x + (long)b * H * W * C;

  // ---- input rows r0-1 .. r0+HS (outside rows/columns are zeros), chunk c of
  // padded column q at physical chunk c ^ (q & 15): instruction k = row*XI + j
  // goes to wave k % 8
  for (int k = wave; k < XR * XI; k += 8) {
    const int xr = k / XI, j = k - xr * XI;
    const int r = r0 - 1 + xr;
    const int i = j * 64 + lane;  // chunk of the padded row
    const int q = i / CPX, pc = i - q * CPX;
    const bool ok = (unsigned)r < (unsigned)H && q >= 1 && q <= W;
    const bf16* src = ok ? img + ((long)r * W + (q - 1)) * C + 8 * (pc ^ (q & 15)) : a.zero;
    if (i < Q * CPX)
      __builtin_amdgcn_global_load_lds((gbl_ptr_t)src, (lds_ptr_t)(xs + xr * ROWB + j * 1024), 16, 0, 0);
  }

  // ---- weight K-tile t (k = BK*t ..) -> stage st (rows permuted, chunks swizzled)
  auto load_wtile = [&](int t, int st) __attribute__((always_inline)) {
#pragma unroll
    for (int p = 0; p < GW; ++p) {
      const int qi = wave * GW + p;  // 1 KB instruction of the stage
      const int i = qi * 64 + lane;
      const int n = i / WCH, pc = i - n * WCH;
      const bf16* src = a.w + (long)perm_row<WN>(n) * (9 * C) + t * BK + 8 * wswz<BK>(n, pc);
      __builtin_amdgcn_global_load_lds((gbl_ptr_t)src, (lds_ptr_t)(wring + st * WSTAGE + qi * 1024), 16, 0, 0);
    }
  };
  load_wtile(0, 0);

  // ---- per-lane constants: pixel p = 16(mh*MF + f) + fr (clamped for padding
  // lanes / a dummy last fragment: they compute a duplicate, never stored)
  int xoff[MF];  // LDS byte offset of (input row prow, padded column pcol) = tap (0, 0)
  int key[MF];   // padded column of tap (0, 0): the chunk swizzle key is (key + kw) & 15
#pragma unroll
  for (int f = 0; f < MF; ++f) {
    const int p = min(16 * (mh * MF + f) + fr, NPIX - 1);
    const int prow = p / W, pcol = p - prow * W;
    xoff[f] = prow * ROWB + pcol * (C * 2);
    key[f] = pcol;
  }
  const uint32_t wrow = (uint32_t)(WN * wn + fr) * (BK * 2);
  float bs[NF / 2][8];  // bias of this lane's channels WN*wn + 32j + 8fq + e
#pragma unroll
  for (int j = 0; j < NF / 2; ++j)
#pragma unroll
    for (int e = 0; e < 8; ++e) bs[j][e] = a.bias[WN * wn + 32 * j + 8 * fq + e];

  floatx4 acc[MF][NF];
#pragma unroll
  for (int f = 0; f < MF; ++f)
#pragma unroll
    for (int nf = 0; nf < NF; ++nf) acc[f][nf] = floatx4{0.f, 0.f, 0.f, 0.f};

  // ---- K loop: 2-stage weight ring, the DMA of K-tile t+1 issued after the
  // barrier that retires every wave's reads of K-tile t-1
  for (int t = 0; t < KT; ++t) {
    vm_wait<0>();  // this wave's DMAs of K-tile t (and, at t = 0, of the input rows)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (t + 1 < KT) load_wtile(t + 1, (t + 1) & 1);

    const int tap = t / CT, cc = t - tap * CT;
    const int kh = tap / 3, kw = tap - kh * 3;
    const int toff = kh * ROWB + kw * (C * 2);
    const char* ws = wring + (t & 1) * WSTAGE + wrow;
#pragma unroll
    for (int ks = 0; ks < BK / 32; ++ks) {
      bf16x8 wf[NF];
#pragma unroll
      for (int nf = 0; nf < NF; ++nf)
        wf[nf] = *(const bf16x8*)(ws + nf * 16 * (BK * 2) + (wswz<BK>(fr, ks * 4 + fq) << 4));
      const int cbase = cc * WCH + ks * 4 + fq;
#pragma unroll
      for (int f = 0; f < MF; ++f) {
        const int ch = cbase ^ ((key[f] + kw) & 15);
        const bf16x8 xf = *(const bf16x8*)(xs + xoff[f] + toff + (ch << 4));
#pragma unroll
        for (int nf = 0; nf < NF; ++nf)
          acc[f][nf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[nf], xf, acc[f][nf], 0, 0, 0);
      }
    }
  }

  // ---- epilogue: lane holds channels WN*wn + 32j + 8fq .. +7 of its pixel
  const long base = ((long)b * H + r0) * W * C + WN * wn + 8 * fq;
#pragma unroll
  for (int f = 0; f < MF; ++f) {
    const int p = 16 * (mh * MF + f) + fr;
    if (p >= NPIX) continue;
#pragma unroll
    for (int j = 0; j < NF / 2; ++j) {
      const long off = base + (long)p * C + 32 * j;
      float v[8];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[e] = acc[f][2 * j][e] + bs[j][e];
        v[4 + e] = acc[f][2 * j + 1][e] + bs[j][4 + e];
      }
      if (a.res) {
        float r[8];
        unpack8(*(const uint4*)(a.res + off), r);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += r[e];
      }
      if (a.relu) {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = fmaxf(v[e], 0.f);
      }
      *(uint4*)(a.y + off) = pack8(v);
    }
  }
}

}  // namespace

bool conv3x3_stream_supported(int H, int W, int Cin, int Cout) {
  return Cin == Cout && ((H == 28 && W == 28 && Cin == 128) || (H == 14 && W == 14 && Cin == 256));
}

void conv3x3_stream(const void* x, const void* w, const float* bias, const void* res, void* y, const void* zero,
                    int B, int H, int W, int C, bool relu, hipStream_t s) {
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
  a.relu = relu;
  if (C == 128) {  // layer2: half an image per workgroup (16 x 30 x 256 B rows + 2 x 16 KB weight stages)
    const size_t lds = (size_t)(14 + 2) * (28 + 2) * 128 * 2 + (size_t)2 * 128 * 64 * 2;
    hipLaunchKernelGGL((conv3x3_stream_kernel<28, 28, 128, 14, 64>), dim3(2 * B), dim3(512), lds, s, a);
  } else {  // layer3: a whole image per workgroup (16 x 16 x 512 B rows + 2 x 16 KB weight stages = 160 KB)
    const size_t lds = (size_t)(14 + 2) * (14 + 2) * 256 * 2 + (size_t)2 * 256 * 32 * 2;
    hipLaunchKernelGGL((conv3x3_stream_kernel<14, 14, 256, 14, 32>), dim3(B), dim3(512), lds, s, a);
  }
  DMLC_HIP_CHECK(hipGetLastError());
}

}  // namespace dmlc
