// Implicit-GEMM convolution on CDNA4 bf16 MFMA (v_mfma_f32_16x16x32_bf16).
//
// Replaces the libtorch CPU conv/BN/ReLU/linear ops that the reference runs
// per query inside `forward_t` (reference: src/services.rs:493, models built at
// src/services.rs:513-524). GEMM view: M = B*Ho*Wo output pixels, N = Cout,
// K = KH*KW*Cin with activations in NHWC so every 8-wide k chunk is 16
// contiguous bytes.
//
// Design (gfx950):
//  * 256-thread workgroups = 4 waves of 64; each wave owns a 64x64 output
//    sub-tile = 4x4 MFMA 16x16 tiles (16 fp32x4 accumulators).
//  * Operand tiles go HBM/L2 -> LDS with global_load_lds_dwordx4 (LDS-DMA,
//    no VGPR staging, no ds_write): each wave-instruction fills 8 LDS rows of
//    128 B. Im2col padding is handled by pointing the lanes of out-of-image
//    taps at a 16-B zero page, so the DMA never needs a per-lane mask.
//  * LDS rows are XOR-swizzled per 16-B chunk (phys = chunk ^ ((row>>1)&7)) so
//    the ds_read_b128 fragment reads (16 rows x same chunk per lane group) are
//    bank-conflict free; because LDS-DMA writes lane-linearly, the swizzle is
//    applied to the per-lane SOURCE address and undone on the read.
//  * Two LDS stages, one barrier per 64-deep K-tile: the DMA of tile t+1 is
//    issued before the MFMAs of tile t.
//  * The MFMA is issued "swapped": A operand = weight rows (n), B operand =
//    activation rows (m), so each lane ends with 4 consecutive output
//    channels of one pixel -> 8-byte packed bf16 stores straight to NHWC.
//  * Epilogue fuses folded-BN bias, residual add and ReLU.
//  * The 3-channel stems read a zero-padded packed-RGB bf16 image written by
//    the preprocess kernel: within an input row the KW taps x 3 channels of
//    one output pixel are contiguous, so k = kh*CPK*8 + kw*3 + c and each
//    16-B chunk is 8 consecutive (kw, c) values of one row (CPK = ceil(3KW/8)
//    chunks per kernel row; no bounds checks, 77% useful K for 7x7 instead
//    of 57% with 4-channel padding).
//  * Optional split-K writes fp32 partials that a small kernel reduces (used
//    when the tile grid cannot fill the 256 CUs, e.g. batch-1 latency runs
//    and the AlexNet classifier).
//  * blockIdx is remapped so consecutive tiles (which share activation rows)
//    run on the same XCD / L2.
#include "common.h"
#include "kernels.h"

#include <algorithm>
#include <type_traits>

namespace dmlc {

namespace {

typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef const __attribute__((address_space(1))) void* gbl_ptr_t;

__device__ __forceinline__ int swz(int row, int chunk) { return chunk ^ ((row >> 1) & 7); }
// e4m3 tiles: a lane's fragment is chunks 2fq and 2fq + 1 of its row, and
// with the bf16 swizzle rows 0 and 4 of a 16-lane read group met on one bank
// (45.7% of the fp8 kernel's LDS cycles were conflicts,
// profiles/r5_roofline_resnet50_fp8.txt); (row >> 1) & 5 gives every group
// of both reads 16 distinct bank slots (tests/test_layouts_cpu.py)
template <bool IN8>
__device__ __forceinline__ int swzk(int row, int chunk) {
  return IN8 ? chunk ^ ((row >> 1) & 5) : swz(row, chunk);
}

typedef int v8i __attribute__((ext_vector_type(8)));
__device__ __forceinline__ v8i cat8(uint4 lo, uint4 hi) {
  return v8i{(int)lo.x, (int)lo.y, (int)lo.z, (int)lo.w, (int)hi.x, (int)hi.y, (int)hi.z, (int)hi.w};
}

// e4m3 helpers (OCP, gfx950): 4 bytes <-> 4 floats; stores saturate at +-448.
__device__ __forceinline__ void fp8x4_to_f32(uint32_t u, float* f) {
  e4m3x4_to_f32(u, f);
}
__device__ __forceinline__ uint32_t f32x4_to_fp8(const float* f) {
  float c[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) c[i] = fminf(fmaxf(f[i], -448.f), 448.f);
  int v = __builtin_amdgcn_cvt_pk_fp8_f32(c[0], c[1], 0, false);
  v = __builtin_amdgcn_cvt_pk_fp8_f32(c[2], c[3], v, true);
  return (uint32_t)v;
}

__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  // Bijective: blocks b and b+8 share an XCD; give each XCD a contiguous
  // range of logical tiles.
  const int q = nwg / 8, r = nwg % 8;
  const int xcd = bid % 8, local = bid / 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + local;
}

// s_waitcnt vmcnt(N) with a compile-time N (the field is an immediate).
template <int N>
__device__ __forceinline__ void vm_wait() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}

// Leave at most min(D-1, remaining) tiles (G DMA instructions each) of this
// wave in flight. `remaining` = tiles issued after the one being waited for.
template <int D, int G>
__device__ __forceinline__ void wait_tiles(int remaining) {
  if constexpr (D >= 3) {
    if (remaining >= 2) { vm_wait<2 * G>(); return; }
  }
  if constexpr (D >= 2) {
    if (remaining >= 1) { vm_wait<G>(); return; }
  }
  vm_wait<0>();
}

// __launch_bounds__(256, 2): 2 waves/SIMD caps the unified register budget
// at 256, which keeps the 64 accumulator registers in arch VGPRs. Without
// it hipcc splits into AGPRs and shuffles ~100 v_accvgpr_* per K-tile
// (measured: 4.4 VALU per MFMA, 40% of wave cycles in waits).
// fp8 (IN8/OUT8, ResNet50 fp8 path): activations/weights/residual are OCP
// e4m3 bytes and a 128-B LDS row holds 128 k instead of 64, so one block-
// scaled v_mfma_scale_f32_16x16x128_f8f6f4 (2x the bf16 MFMA rate) covers a
// whole K-tile; a lane's A/B fragment is the 32 contiguous bytes of chunks
// 2*fq, 2*fq+1 of its row (any lane->k map works as long as A and B agree:
// tests/test_fp8_gpu.py). The epilogue dequantises with a per-channel
// alpha = s_in * s_w[n], adds bias and the residual (e4m3 x res_scale when
// the output is e4m3: in a ResNet block the residual has the output's
// dtype), applies ReLU and requantises with out_inv_scale (saturating).
template <int BM, int BN, int WM, int WN, int NS, bool PAIR, bool IN8 = false, bool OUT8 = false>
__global__ __launch_bounds__(256, 2) void conv_igemm_kernel(ConvArgs a, int kt_per_split, int k_tiles) {
  static_assert(!(PAIR && IN8), "the stem is bf16");
  using Elem = typename std::conditional<IN8, uint8_t, bf16>::type;
  constexpr int CE = IN8 ? 16 : 8;  // elements per 16-B chunk
  constexpr int BK = 8 * CE;        // elements per K-tile (one 128-B LDS row)
  static_assert(NS >= 2 && NS <= 4, "stages");
  constexpr int PA = BM / 32;  // A rows per lane (wave covers BM/4 rows = PA instrs of 8 rows)
  constexpr int PB = BN / 32;
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int TM = WTM / 16, TN = WTN / 16;
  static_assert(WM * WN == 4, "4 waves per block");
  static_assert(BM % 32 == 0 && BN % 32 == 0, "tile");
  constexpr int ROWB = 128;                          // bytes per LDS row
  constexpr int STAGE_B = (BM + BN) * ROWB;          // bytes per stage
  constexpr int A_CH = BM * 8;                       // chunks in the A part of a stage
  constexpr int STAGE_CH = (BM + BN) * 8;

  extern __shared__ __attribute__((aligned(16))) uint4 smem[];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave % WM, wn = wave / WM;

  const int M = a.B * a.Ho * a.Wo;
  const int n_tiles = a.Npad / BN;
  const int m_tiles = (M + BM - 1) / BM;
  const int nwg = n_tiles * m_tiles;
  // Persistent grids (NS == 2): block b walks tiles b, b+G, b+2G, ... (G =
  // gridDim.x, a multiple of 8 so b's XCD group is fixed), and the first
  // K-tile DMA of its next tile is issued before the epilogue of the current
  // one, so prologue latency and epilogue stores overlap.
  int tile_iter = blockIdx.x;
  int tile = xcd_remap(tile_iter, nwg);
  int m0 = (tile / n_tiles) * BM, n0 = (tile % n_tiles) * BN;

  const int split = blockIdx.y;
  const int kt0 = split * kt_per_split;
  const int kt1 = min(k_tiles, kt0 + kt_per_split);
  const int nk = kt1 - kt0;

  const Elem* __restrict__ x = (const Elem*)a.x;
  const Elem* __restrict__ w = (const Elem*)a.w;
  const Elem* zero = (const Elem*)a.zero;

  // Rows this lane stages. A: rows wave*BM/4 + p*8 + lane/8, B likewise.
  const int lrow = lane >> 3;
  const int pchunk = lane & 7;  // physical chunk written by this lane
  int hi0[PA], wi0[PA], abase[PA];
  int lcA[PA];
  int wboff[PB];
  // Per-tile staging state (input origin of every staged row, weight rows).
  auto setup_rows = [&](int m0_, int n0_) __attribute__((always_inline)) {
#pragma unroll
    for (int p = 0; p < PA; ++p) {
      const int r = wave * (BM / 4) + p * 8 + lrow;
      const int lc = swzk<IN8>(r, pchunk);
      lcA[p] = lc;
      const int m = m0_ + r;
      if (m < M) {
        const int hw = a.Ho * a.Wo;
        const int b = m / hw;
        const int rem = m - b * hw;
        const int ho = rem / a.Wo;
        const int wo = rem - ho * a.Wo;
        if constexpr (PAIR) {
          hi0[p] = ho * a.stride;
          wi0[p] = wo * a.stride;
          abase[p] = ((b * a.H + hi0[p]) * a.W + wi0[p]) * 3;  // packed RGB row image
        } else {
          hi0[p] = ho * a.stride - a.pad;
          wi0[p] = wo * a.stride - a.pad;
          abase[p] = ((b * a.H + hi0[p]) * a.W + wi0[p]) * a.Cin + lc * CE;
        }
      } else {
        hi0[p] = -(1 << 28);
        wi0[p] = 0;
        abase[p] = 0;
      }
    }
#pragma unroll
    for (int p = 0; p < PB; ++p) {
      const int r = wave * (BN / 4) + p * 8 + lrow;
      wboff[p] = (n0_ + r) * a.Kpad + swzk<IN8>(r, pchunk) * CE;
    }
  };
  setup_rows(m0, n0);
  const int CPK = (a.KW * 3 + 7) >> 3;  // stem: 16-B chunks per kernel row
  const int stem_chunks = a.KH * CPK;

  // Issue the LDS-DMA for K-tile t into stage `st`.
  auto stage = [&](int t, int st) __attribute__((always_inline)) {
    char* sbase = (char*)smem + st * STAGE_B;
    if constexpr (!PAIR) {
      const int ctiles = a.Cin / BK;
      const int tap = t / ctiles;
      const int c0 = (t - tap * ctiles) * BK;
      const int kh = tap / a.KW;
      const int kw = tap - kh * a.KW;
      const int off = (kh * a.W + kw) * a.Cin + c0;
#pragma unroll
      for (int p = 0; p < PA; ++p) {
        const bool ok = (unsigned)(hi0[p] + kh) < (unsigned)a.H && (unsigned)(wi0[p] + kw) < (unsigned)a.W;
        const Elem* src = ok ? x + abase[p] + off : zero;
        __builtin_amdgcn_global_load_lds((gbl_ptr_t)src,
                                         (lds_ptr_t)(sbase + (wave * (BM / 4) + p * 8) * ROWB), 16, 0, 0);
      }
    } else {
#pragma unroll
      for (int p = 0; p < PA; ++p) {
        const int q = t * 8 + lcA[p];  // chunk index along K
        const int kh = q / CPK;
        const int j = q - kh * CPK;
        const bool ok = q < stem_chunks && hi0[p] >= 0;
        // 4-B aligned (wi0 even, row length even): LDS-DMA needs dword alignment
        const Elem* src = ok ? x + abase[p] + kh * a.W * 3 + j * 8 : zero;
        __builtin_amdgcn_global_load_lds((gbl_ptr_t)src,
                                         (lds_ptr_t)(sbase + (wave * (BM / 4) + p * 8) * ROWB), 16, 0, 0);
      }
    }
    const Elem* wt = w + t * BK;
#pragma unroll
    for (int p = 0; p < PB; ++p)
      __builtin_amdgcn_global_load_lds((gbl_ptr_t)(wt + wboff[p]),
                                       (lds_ptr_t)(sbase + (BM + wave * (BN / 4) + p * 8) * ROWB), 16, 0, 0);
  };

  floatx4 acc[TN][TM];
#pragma unroll
  for (int i = 0; i < TN; ++i)
#pragma unroll
    for (int j = 0; j < TM; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fq = lane >> 4;

  auto compute = [&](int st) __attribute__((always_inline)) {
    const uint4* sb = smem + st * STAGE_CH;
    if constexpr (IN8) {
      // one 128-deep k-step: lane fragment = chunks 2fq, 2fq+1 (32 bytes)
      v8i af[TN], bm[TM];
#pragma unroll
      for (int i = 0; i < TN; ++i) {
        const int r = wn * WTN + i * 16 + fr;
        af[i] = cat8(sb[A_CH + r * 8 + swzk<IN8>(r, 2 * fq)], sb[A_CH + r * 8 + swzk<IN8>(r, 2 * fq + 1)]);
      }
#pragma unroll
      for (int j = 0; j < TM; ++j) {
        const int r = wm * WTM + j * 16 + fr;
        bm[j] = cat8(sb[r * 8 + swzk<IN8>(r, 2 * fq)], sb[r * 8 + swzk<IN8>(r, 2 * fq + 1)]);
      }
#pragma unroll
      for (int i = 0; i < TN; ++i)
#pragma unroll
        for (int j = 0; j < TM; ++j)  // formats 0/0 = e4m3; E8M0 scales 127 = 1.0
          acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(af[i], bm[j], acc[i][j], 0, 0, 0, 127, 0, 127);
      return;
    }
#pragma unroll
    for (int ks = 0; ks < BK / 32; ++ks) {
      bf16x8 af[TN], bm[TM];
#pragma unroll
      for (int i = 0; i < TN; ++i) {
        const int r = wn * WTN + i * 16 + fr;
        af[i] = __builtin_bit_cast(bf16x8, sb[A_CH + r * 8 + swzk<IN8>(r, ks * 4 + fq)]);
      }
#pragma unroll
      for (int j = 0; j < TM; ++j) {
        const int r = wm * WTM + j * 16 + fr;
        bm[j] = __builtin_bit_cast(bf16x8, sb[r * 8 + swzk<IN8>(r, ks * 4 + fq)]);
      }
#pragma unroll
      for (int i = 0; i < TN; ++i)
#pragma unroll
        for (int j = 0; j < TM; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bm[j], acc[i][j], 0, 0, 0);
    }
  };

  // NS-stage ring, prefetch distance D = NS-1 tiles. Iteration `it`:
  //   wait (counted) until this wave's DMA for tile `it` landed, leaving the
  //   younger tiles in flight; raw s_barrier (no vmcnt(0) drain) so every
  //   wave's part of tile `it` is visible and every wave has finished reading
  //   tile it-1; then refill tile it-1's stage with tile it+D and compute.
  constexpr int D = NS - 1;
  constexpr int G = PA + PB;  // LDS-DMA instructions per wave per tile

  // Epilogue. Lane holds D[n = 4*fq + r][m = fr] of each 16x16 tile.
  auto epilogue = [&](int m0e, int n0e) __attribute__((always_inline)) {
    if (gridDim.y > 1) {
      float* __restrict__ ws = a.ws + (size_t)split * M * a.Npad;
#pragma unroll
      for (int j = 0; j < TM; ++j) {
        const int m = m0e + wm * WTM + j * 16 + fr;
        if (m >= M) continue;
#pragma unroll
        for (int i = 0; i < TN; ++i) {
          const int n = n0e + wn * WTN + i * 16 + fq * 4;
          *(floatx4*)(ws + (size_t)m * a.Npad + n) = acc[i][j];
        }
      }
      return;
    }
    const bf16* __restrict__ res = (const bf16*)a.res;
#pragma unroll
    for (int j = 0; j < TM; ++j) {
      const int m = m0e + wm * WTM + j * 16 + fr;
      if (m >= M) continue;
#pragma unroll
      for (int i = 0; i < TN; ++i) {
        const int n = n0e + wn * WTN + i * 16 + fq * 4;
        if (n >= a.N) continue;
        float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
        if constexpr (IN8) {  // dequantise: s_in * s_w[n]
          const floatx4 al = *(const floatx4*)(a.alpha + n);
          v[0] *= al[0]; v[1] *= al[1]; v[2] *= al[2]; v[3] *= al[3];
        }
        if (a.bias) {
          const floatx4 bb = *(const floatx4*)(a.bias + n);
          v[0] += bb[0]; v[1] += bb[1]; v[2] += bb[2]; v[3] += bb[3];
        }
        const size_t o = (size_t)m * a.ldo + n;
        if (res) {
          if constexpr (OUT8) {  // the residual is the block's previous output: same dtype as y
            float rf[4];
            fp8x4_to_f32(*(const uint32_t*)((const uint8_t*)a.res + o), rf);
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] += rf[r] * a.res_scale;
          } else {
            const uint2 rv = *(const uint2*)(res + o);
            v[0] += __uint_as_float(rv.x << 16);
            v[1] += __uint_as_float(rv.x & 0xffff0000u);
            v[2] += __uint_as_float(rv.y << 16);
            v[3] += __uint_as_float(rv.y & 0xffff0000u);
          }
        }
        if (a.relu) {
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = fmaxf(v[r], 0.f);
        }
        if constexpr (OUT8) {
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] *= a.out_inv_scale;
          *(uint32_t*)((uint8_t*)a.y + o) = f32x4_to_fp8(v);
        } else if (a.out_f32) {
          *(floatx4*)((float*)a.y + o) = floatx4{v[0], v[1], v[2], v[3]};
        } else {
          *(uint2*)((bf16*)a.y + o) = make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3]));
        }
      }
    }
  };

  // bf16 epilogue staged through LDS (same scheme as conv_bigtile.hip): the
  // wave writes 16 rows x 64 cols of fp32 accumulators to its 4 KB of the
  // stage it just consumed (16-B chunks XOR-swizzled by row), then each lane
  // reads 8 consecutive channels of one row and adds bias and residual with
  // one 16-B load, applies ReLU and stores 16 B: a wave instruction covers 8
  // rows x 128 contiguous bytes instead of 16 rows x 32 B. Needs the caller
  // to have passed a barrier after every wave's last read of that stage.
  auto epilogue_lds = [&](int m0e, int n0e, int est) __attribute__((always_inline)) {
    float* wl = (float*)((char*)smem + est * STAGE_B) + wave * (16 * 64);
    const bf16* __restrict__ res = (const bf16*)a.res;
    const int q = lane & 7, rr = lane >> 3;
    const int nq = n0e + wn * WTN + q * 8;
    floatx4 bq0 = {0.f, 0.f, 0.f, 0.f}, bq1 = bq0, aq0 = {1.f, 1.f, 1.f, 1.f}, aq1 = aq0;
    if (a.bias && nq < a.N) {
      bq0 = *(const floatx4*)(a.bias + nq);
      bq1 = *(const floatx4*)(a.bias + nq + 4);
    }
    if constexpr (IN8) {  // dequantise: s_in * s_w[n], before the bias
      if (nq < a.N) {
        aq0 = *(const floatx4*)(a.alpha + nq);
        aq1 = *(const floatx4*)(a.alpha + nq + 4);
      }
    }
#pragma unroll
    for (int j = 0; j < TM; ++j) {
#pragma unroll
      for (int i = 0; i < TN; ++i) *(floatx4*)(wl + fr * 64 + (((i * 4 + fq) ^ fr) * 4)) = acc[i][j];
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int g = 0; g < 2; ++g) {
        const int row = g * 8 + rr;
        const floatx4 lo = *(const floatx4*)(wl + row * 64 + (((2 * q) ^ row) * 4));
        const floatx4 hi = *(const floatx4*)(wl + row * 64 + (((2 * q + 1) ^ row) * 4));
        const int m = m0e + wm * WTM + j * 16 + row;
        if (m >= M || nq >= a.N) continue;
        float v[8] = {lo[0] * aq0[0] + bq0[0], lo[1] * aq0[1] + bq0[1], lo[2] * aq0[2] + bq0[2],
                      lo[3] * aq0[3] + bq0[3], hi[0] * aq1[0] + bq1[0], hi[1] * aq1[1] + bq1[1],
                      hi[2] * aq1[2] + bq1[2], hi[3] * aq1[3] + bq1[3]};
        if constexpr (!IN8) {  // (exact: the multiply by 1 is not emitted for bf16 input)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            v[e] = lo[e] + bq0[e];
            v[4 + e] = hi[e] + bq1[e];
          }
        }
        const size_t o = (size_t)m * a.ldo + nq;
        if (res) {
          float r[8];
          if constexpr (OUT8) {  // the residual is the block's previous output: same dtype as y
            const uint2 rv = *(const uint2*)((const uint8_t*)a.res + o);
            fp8x4_to_f32(rv.x, r);
            fp8x4_to_f32(rv.y, r + 4);
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] += r[e] * a.res_scale;
          } else {
            unpack8(*(const uint4*)(res + o), r);
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] += r[e];
          }
        }
        if (a.relu) {
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = fmaxf(v[e], 0.f);
        }
        if constexpr (OUT8) {
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] *= a.out_inv_scale;
          *(uint2*)((uint8_t*)a.y + o) = make_uint2(f32x4_to_fp8(v), f32x4_to_fp8(v + 4));
        } else {
          *(uint4*)((bf16*)a.y + o) = pack8(v);
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // reads done before the next pass overwrites
    }
  };
  // 16-B rows need N, ldo multiples of 8 and 16-B aligned y / residual
  // (fp8 in / out too: alpha before the bias, 8-B e4m3 rows; 16-B bf16 rows)
  const bool lds_epi = !PAIR && WTN == 64 && gridDim.y == 1 && !a.out_f32 && a.N % 8 == 0 && a.ldo % 8 == 0 &&
                       (((uintptr_t)a.y | (uintptr_t)a.res) & (OUT8 ? 7 : 15)) == 0;

  if (nk <= 0 || tile_iter >= nwg) return;

  if constexpr (NS == 2) {
    // Flattened (tile, K-tile) stream over this block's tiles; the DMA for
    // the next item is issued right after each barrier, including across a
    // tile boundary (the next tile's first K-tile lands during this tile's
    // last MFMAs and epilogue).
    stage(kt0, 0);
    int st = 0;
    while (true) {
      int next_iter = -1;
      int m0c = m0, n0c = n0;
      for (int it = 0; it < nk; ++it) {
        vm_wait<0>();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if (it + 1 < nk) {
          stage(kt0 + it + 1, st ^ 1);
        } else if (a.persistent && tile_iter + (int)gridDim.x < nwg) {
          next_iter = tile_iter + gridDim.x;
          tile = xcd_remap(next_iter, nwg);
          m0 = (tile / n_tiles) * BM;
          n0 = (tile % n_tiles) * BN;
          setup_rows(m0, n0);  // the current tile issued all its DMA: safe to overwrite
          stage(kt0, st ^ 1);
        }
        compute(st);
        st ^= 1;
      }
      if (lds_epi) {
        // every wave has finished reading the stage it just computed (st ^ 1);
        // the next tile's first K-tile is landing in the other one
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        epilogue_lds(m0c, n0c, st ^ 1);
      } else {
        epilogue(m0c, n0c);
      }
      if (next_iter < 0) break;
      tile_iter = next_iter;
#pragma unroll
      for (int i = 0; i < TN; ++i)
#pragma unroll
        for (int j = 0; j < TM; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
    }
  } else {
#pragma unroll
    for (int s = 0; s < D; ++s)
      if (s < nk) stage(kt0 + s, s);
    int st = 0;
    for (int it = 0; it < nk; ++it) {
      wait_tiles<D, G>(min(D - 1, nk - 1 - it));
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      if (it + D < nk) {
        const int ls = st == 0 ? NS - 1 : st - 1;  // stage of tile it-1 == stage of tile it+D
        stage(kt0 + it + D, ls);
      }
      compute(st);
      st = st == NS - 1 ? 0 : st + 1;
    }
    epilogue(m0, n0);
  }
}

// Split-K reduction + fused epilogue. One thread per 4 output channels.
__global__ __launch_bounds__(256) void splitk_reduce_kernel(ConvArgs a, int M, int splits) {
  const int n4 = a.N / 4;
  const long total = (long)M * n4;
  for (long idx = blockIdx.x * 256L + threadIdx.x; idx < total; idx += (long)gridDim.x * 256) {
    const int m = (int)(idx / n4);
    const int n = (int)(idx - (long)m * n4) * 4;
    // all of a group's partial loads in flight at once (a plain loop waited
    // on each in turn: one L2 round trip per split, ~5 us per reduce at B=1)
    floatx4 s = {0.f, 0.f, 0.f, 0.f};
    const float* wp = a.ws + (size_t)m * a.Npad + n;
    const size_t sstride = (size_t)M * a.Npad;
    int k = 0;
    for (; k + 8 <= splits; k += 8) {
      floatx4 t[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) t[u] = *(const floatx4*)(wp + (size_t)(k + u) * sstride);
#pragma unroll
      for (int u = 0; u < 8; ++u) s += t[u];
    }
    for (; k + 4 <= splits; k += 4) {
      floatx4 t[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) t[u] = *(const floatx4*)(wp + (size_t)(k + u) * sstride);
#pragma unroll
      for (int u = 0; u < 4; ++u) s += t[u];
    }
    for (; k < splits; ++k) s += *(const floatx4*)(wp + (size_t)k * sstride);
    if (a.bias) s += *(const floatx4*)(a.bias + n);
    const size_t o = (size_t)m * a.ldo + n;
    if (a.res) {
      const uint2 rv = *(const uint2*)((const bf16*)a.res + o);
      s[0] += __uint_as_float(rv.x << 16);
      s[1] += __uint_as_float(rv.x & 0xffff0000u);
      s[2] += __uint_as_float(rv.y << 16);
      s[3] += __uint_as_float(rv.y & 0xffff0000u);
    }
    if (a.relu) {
#pragma unroll
      for (int r = 0; r < 4; ++r) s[r] = fmaxf(s[r], 0.f);
    }
    if (a.out_f32) {
      *(floatx4*)((float*)a.y + o) = s;
    } else {
      *(uint2*)((bf16*)a.y + o) = make_uint2(pack2(s[0], s[1]), pack2(s[2], s[3]));
    }
  }
}

struct TileCfg {
  int bm, bn, ns;
};

// Tile configurations (4 waves each, 64x64 per wave; ns = LDS stages):
//   0: 128x128 ns2   1: 256x64 ns2   2: 64x256 ns2
//   3: 128x128 ns3   4: 256x64 ns3   5: 64x256 ns3   6: 128x128 ns4
// (A register double-buffered fragment schedule on top of ns2 measured
// within +-3% of these and was dropped; ns3/ns4 lose 30% to the halved
// occupancy: profiles/r1_conv_bench_stages.log.)
//   7: 128x64 ns2 (waves 2x2 of 64x32)   8: 64x128 ns2 (waves 2x2 of 32x64)
//   9: 128x64 ns3  10: 64x128 ns3 (72 KB: deeper prefetch at 2 blocks per CU)
constexpr int kNumTiles = 11;
constexpr TileCfg kTiles[kNumTiles] = {{128, 128, 2}, {256, 64, 2}, {64, 256, 2}, {128, 128, 3}, {256, 64, 3},
                                       {64, 256, 3},  {128, 128, 4}, {128, 64, 2}, {64, 128, 2}, {128, 64, 3},
                                       {64, 128, 3}};

int pick_tile(const ConvArgs& a) {
  if (a.tile >= 0 && a.tile < kNumTiles) return a.tile;
  if (a.Npad % 128 != 0) return 1;
  const long M = (long)a.B * a.Ho * a.Wo;
  if (M <= 64 && a.Npad % 256 == 0) return 2;
  // N = 128 over many pixels (ResNet layer2): 64x128 tiles measured 5-11%
  // faster than 128x128 (profiles/r1_conv_tiles_ns3.log)
  if (a.Npad == 128 && M >= 64L * 1024) return 8;
  return 0;
}

template <int BM, int BN, int WM, int WN, int NS, bool IN8 = false, bool OUT8 = false>
void launch_cfg(const ConvArgs& a, int splits, int kt_per, int k_tiles, hipStream_t s) {
  const int M = a.B * a.Ho * a.Wo;
  int tiles = ((M + BM - 1) / BM) * (a.Npad / BN);
  ConvArgs b = a;
  if (NS == 2 && a.persistent && a.max_blocks >= 8 && tiles > a.max_blocks) {
    tiles = a.max_blocks / 8 * 8;  // multiple of 8: a block keeps its XCD group
  } else {
    b.persistent = false;
  }
  dim3 grid(tiles, splits);
  const size_t lds = (size_t)NS * (BM + BN) * 128;
  if constexpr (IN8 || OUT8)
    hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, WM, WN, NS, false, IN8, OUT8>), grid, dim3(256), lds, s, b, kt_per,
                       k_tiles);
  else if (a.stem)
    hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, WM, WN, NS, true>), grid, dim3(256), lds, s, b, kt_per, k_tiles);
  else
    hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, WM, WN, NS, false>), grid, dim3(256), lds, s, b, kt_per, k_tiles);
  DMLC_HIP_CHECK(hipGetLastError());
}

}  // namespace

int conv_out_dim(int in, int k, int stride, int pad) { return (in + 2 * pad - k) / stride + 1; }

int conv_kpad(int Cin, int KH, int KW, bool stem) {
  if (stem) {
    const int k = KH * ((KW * 3 + 7) / 8) * 8;
    return (k + 63) / 64 * 64;
  }
  return KH * KW * Cin;  // Cin % 64 == 0
}

int stem_row_width(int S, int pad, int KW, int stride) {
  // columns read by the last output pixel: ((Wo-1)*stride)*3 + CPK*8 values
  const int Wo = (S + 2 * pad - KW) / stride + 1;
  const int need = ((Wo - 1) * stride * 3 + ((KW * 3 + 7) / 8) * 8 + 2) / 3;
  int w = std::max(S + 2 * pad, need);
  return (w + 7) / 8 * 8;  // multiple of 8 pixels: 48-B aligned rows, even width
}

int conv_npad(int N) {
  if (N <= 64) return 64;
  if (N % 64 == 0) return N;  // 192, 320, ...: 256x64 tiles, no padding waste
  return (N + 127) / 128 * 128;
}

int conv_pick_split_k(const ConvArgs& a, int num_cus) {
  const int cfg = pick_tile(a);
  const int BM = kTiles[cfg].bm, BN = kTiles[cfg].bn;
  const long M = (long)a.B * a.Ho * a.Wo;
  const long tiles = ((M + BM - 1) / BM) * (a.Npad / BN);
  const int k_tiles = a.Kpad / 64;
  if (a.in_fp8 || a.out_fp8 || tiles >= num_cus / 2 || k_tiles < 16) return 1;
  int s = (int)((num_cus + tiles - 1) / tiles);
  // fc layers at throughput batches (AlexNet classifier, M = B <= 256: 64 / 16
  // tiles): 8 K slices (two rounds of workgroups) beat the one-round pick --
  // classifier.1 55 -> 47 us, classifier.6 28 -> 23 us at B=256; 16 is slower
  // again (profiles/r3_alexnet_fc_splitk.txt)
  const bool fc = a.H == 1 && a.W == 1 && a.KH == 1 && a.KW == 1 && a.Kpad >= 4096;
  if (fc) s = std::max(s, 8);
  // (fc layers may take K slices of 4 K-tiles: classifier.6, 16 tiles at
  // B = 256, 22.0 -> 20.2 us with 16 slices; tools/fc_bench.py,
  // profiles/r5_fc_splitk.txt)
  s = std::min(s, k_tiles / (fc ? 4 : 8));
  s = std::min(s, 16);
  return std::max(s, 1);
}

size_t conv_splitk_ws_elems(const ConvArgs& a) {
  if (a.split_k <= 1) return 0;
  return (size_t)a.split_k * a.B * a.Ho * a.Wo * a.Npad;
}

void conv2d_igemm(const ConvArgs& a, hipStream_t s) {
  if (a.stem) {
    if (a.Cin != 3) throw std::invalid_argument("conv2d_igemm: stem expects the packed RGB image (Cin == 3)");
  } else if (a.Cin % (a.in_fp8 ? 128 : 64) != 0) {
    throw std::invalid_argument("conv2d_igemm: Cin must be a multiple of 64 (128 for fp8)");
  }
  if ((a.in_fp8 || a.out_fp8) && (a.stem || a.split_k > 1 || a.out_f32))
    throw std::invalid_argument("conv2d_igemm: fp8 has no stem / split-K / fp32-output variant");
  if (a.in_fp8 && !a.alpha) throw std::invalid_argument("conv2d_igemm: fp8 input needs alpha");
  if (a.Kpad != conv_kpad(a.Cin, a.KH, a.KW, a.stem)) throw std::invalid_argument("conv2d_igemm: bad Kpad");
  if (a.N % 4 != 0 || a.N > a.Npad || a.ldo < a.N || a.ldo % 4 != 0)
    throw std::invalid_argument("conv2d_igemm: bad N/ldo");
  if (a.stem) {
    // x = zero-padded packed image [B, H, W, 3] (pad already applied, W = row
    // width in pixels). Every chunk read must stay inside its row and be
    // dword aligned: even stride and even row width.
    const int cpk = (a.KW * 3 + 7) / 8;
    if (a.Ho <= 0 || a.Wo <= 0 || (a.Ho - 1) * a.stride + a.KH > a.H ||
        (a.Wo - 1) * a.stride * 3 + cpk * 8 > a.W * 3 || (a.stride & 1) || (a.W & 1))
      throw std::invalid_argument("conv2d_igemm: stem geometry out of bounds / misaligned");
  } else if (a.Ho != conv_out_dim(a.H, a.KH, a.stride, a.pad) || a.Wo != conv_out_dim(a.W, a.KW, a.stride, a.pad)) {
    throw std::invalid_argument("conv2d_igemm: bad output dims");
  }
  if (!a.x || !a.w || !a.y || !a.zero) throw std::invalid_argument("conv2d_igemm: null operand");
  if (((uintptr_t)a.x | (uintptr_t)a.w | (uintptr_t)a.zero) & 15)
    throw std::invalid_argument("conv2d_igemm: operands must be 16-B aligned");
  const int cfg = pick_tile(a);
  const int BN = kTiles[cfg].bn;
  if (a.Npad % BN != 0) throw std::invalid_argument("conv2d_igemm: Npad not a multiple of BN");
  const long M = (long)a.B * a.Ho * a.Wo;
  if (M <= 0) return;
  if ((long)a.B * a.H * a.W * a.Cin >= (1L << 31) || M * a.ldo >= (1L << 31) ||
      (long)a.Npad * a.Kpad >= (1L << 31))
    throw std::invalid_argument("conv2d_igemm: tensor too large for 32-bit offsets");
  const int k_tiles = a.Kpad / (a.in_fp8 ? 128 : 64);
  int splits = std::max(1, a.split_k);
  if (splits > 1 && !a.ws) throw std::invalid_argument("conv2d_igemm: split-K needs a workspace");
  const int kt_per = (k_tiles + splits - 1) / splits;
  splits = (k_tiles + kt_per - 1) / kt_per;
  ConvArgs b = a;
  b.split_k = splits;
  if (a.in_fp8 || a.out_fp8) {  // fp8 is built for the 128x128 and 256x64 tiles only
    const int fcfg = (a.tile == 1 || a.Npad % 128 != 0) ? 1 : 0;
    if (a.Npad % kTiles[fcfg].bn != 0) throw std::invalid_argument("conv2d_igemm: Npad not a multiple of BN");
    const int v = (a.in_fp8 ? 2 : 0) + (a.out_fp8 ? 1 : 0) + (fcfg == 1 ? 4 : 0);
    switch (v) {
      case 1: launch_cfg<128, 128, 2, 2, 2, false, true>(b, 1, k_tiles, k_tiles, s); break;
      case 2: launch_cfg<128, 128, 2, 2, 2, true, false>(b, 1, k_tiles, k_tiles, s); break;
      case 3: launch_cfg<128, 128, 2, 2, 2, true, true>(b, 1, k_tiles, k_tiles, s); break;
      case 5: launch_cfg<256, 64, 4, 1, 2, false, true>(b, 1, k_tiles, k_tiles, s); break;
      case 6: launch_cfg<256, 64, 4, 1, 2, true, false>(b, 1, k_tiles, k_tiles, s); break;
      default: launch_cfg<256, 64, 4, 1, 2, true, true>(b, 1, k_tiles, k_tiles, s); break;
    }
    return;
  }
  switch (cfg) {
    case 0: launch_cfg<128, 128, 2, 2, 2>(b, splits, kt_per, k_tiles, s); break;
    case 1: launch_cfg<256, 64, 4, 1, 2>(b, splits, kt_per, k_tiles, s); break;
    case 2: launch_cfg<64, 256, 1, 4, 2>(b, splits, kt_per, k_tiles, s); break;
    case 3: launch_cfg<128, 128, 2, 2, 3>(b, splits, kt_per, k_tiles, s); break;
    case 4: launch_cfg<256, 64, 4, 1, 3>(b, splits, kt_per, k_tiles, s); break;
    case 5: launch_cfg<64, 256, 1, 4, 3>(b, splits, kt_per, k_tiles, s); break;
    case 6: launch_cfg<128, 128, 2, 2, 4>(b, splits, kt_per, k_tiles, s); break;
    case 7: launch_cfg<128, 64, 2, 2, 2>(b, splits, kt_per, k_tiles, s); break;
    case 8: launch_cfg<64, 128, 2, 2, 2>(b, splits, kt_per, k_tiles, s); break;
    case 9: launch_cfg<128, 64, 2, 2, 3>(b, splits, kt_per, k_tiles, s); break;
    default: launch_cfg<64, 128, 2, 2, 3>(b, splits, kt_per, k_tiles, s); break;
  }
  if (splits > 1) splitk_reduce(b, M, splits, s);
}

void splitk_reduce(const ConvArgs& a, long M, int splits, hipStream_t s) {
  const int blocks = (int)std::min<long>((M * (a.N / 4) + 255) / 256, 4096);
  hipLaunchKernelGGL(splitk_reduce_kernel, dim3(blocks), dim3(256), 0, s, a, (int)M, splits);
  DMLC_HIP_CHECK(hipGetLastError());
}

}  // namespace dmlc
