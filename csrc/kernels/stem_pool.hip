// Fused ResNet stem: conv 7x7/s2/p3 (BN folded) + ReLU + maxpool 3x3/s2/p1
// in one kernel, image in, pooled [B, Ho/2, Wo/2, 64] bf16 NHWC out.
//
// Reference equivalent: the first four modules of tch::vision::resnet18's
// forward (conv1, bn1, relu, maxpool) run by `forward_t` per query at
// src/services.rs:493. As two kernels (implicit-GEMM conv, then maxpool) the
// stem is the most memory-bound stage of ResNet18: the 112x112x64 conv
// output is written and re-read (2 x 411 MB at B=256) and the im2col tile
// re-fetches every input pixel ~12x from L2. Here each workgroup walks a
// strip of pooled rows of one image top to bottom:
//
//  * Input: the "paired" image from preprocess_u8(paired=true): rows of
//    Wq 16-B chunks, chunk p = padded pixels (2p, 2p+1) as [r g b r g b 0 0].
//    With stride 2, output column ow reads kernel row kh as the 4 chunks
//    p = ow..ow+3, so a 32-wide K step is exactly one kernel row and every
//    MFMA operand is one aligned ds_read_b128 straight from the staged input
//    row (no im2col copy). K = 7 rows x 32 = 224; weights are zero on the
//    pad slots (e = 6,7 and kw = 7).
//  * Staging: input rows go HBM -> LDS with global_load_lds_dwordx4 into a
//    ring of 21 rows; a step needs 13, the 8 rows of the next step are in
//    flight while the current one computes.
//  * Compute: 4 waves, wave w = one conv row, all 64 channels; weights
//    (64 x 224) live in registers for the whole kernel. D = X x W, so each
//    lane holds 4 consecutive output columns of one channel.
//  * Pool: the horizontal 3-max is then mostly lane-local: columns
//    4g..4g+3 of a lane give pooled columns 2g (plus column 4g-1, fetched
//    from the lane 16 below with two row-swap permutes) and 2g+1. The bias is
//    the accumulators' starting value; rounding to bf16 and ReLU are monotone,
//    so they run first and the max runs on packed bf16 pairs (hpool_packed),
//    and the results go to a 5-row LDS ring of pooled conv rows ([pw][64 ch],
//    16-B channel chunks XOR-swizzled by pw so the 4 row groups of a wave
//    hit different banks). The vertical 3-max over that ring writes two
//    pooled rows per step as 16-B stores. Post-ReLU values are >= 0, so
//    bf16 max is an unsigned 16-bit max and the zero row above the image is
//    neutral.
//
// Step t of a strip starting at pooled row ph0 computes conv rows
// c0 = 2*ph0 - 4 + 4t .. c0+3; step 0 only computes row 2*ph0-1 (the top
// halo), steps >= 1 emit pooled rows ph0 + 2(t-1) and ph0 + 2(t-1) + 1.
#include "common.h"
#include "kernels.h"

#include <algorithm>
#include <cstdlib>
#include <string>

namespace dmlc {

namespace {

typedef unsigned short ushort8 __attribute__((ext_vector_type(8)));
typedef float float2v __attribute__((ext_vector_type(2)));
typedef short short2v __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

constexpr int kRing = 21;  // staged input rows: 13 for a step + 8 in flight
// u8 input (fused preprocess): the 8 rows of the next step arrive as raw u8
// image rows in a small ring and are converted into the paired bf16 ring only
// after the current step's MFMAs, so the paired ring needs just 13 rows
// (and the workgroup still fits 2 per CU: ~73 KB of LDS at 224x224).
constexpr int kRingU8 = 13;
// raw u8 ring slot: the row at byte 16, zero pads before (16) and after (64)
// it, so the conversion's 28-byte windows (which start 12 bytes before the
// row and end up to 16 after it) read in-slot zeros at the edges: no
// per-dword bounds checks
constexpr int kU8Front = 16, kU8Pad = 80;
constexpr int kHp = 5;     // horizontally pooled conv rows: carried halo + 4
constexpr int kK = 224;    // 7 kernel rows x 4 chunks x 8
constexpr int kKD = 160;   // dense K: 7 kernel rows x 22 (7 px x rgb + 1 pad) -> 5 x 32
// Pooled-row LDS layout: [pw][64 ch] with a 144-B column stride (128 + 16 pad):
// the 4 row groups of a wave write columns 2 apart = 288 B = 8 banks apart,
// so the 16-bit stores are conflict-free and every address is a per-lane
// base plus an immediate.
constexpr int kHpCol = 144;

struct StemArgs {
  const bf16* x;      // [B, Hp, Wq, 8]
  const uint8_t* u8;  // fused preprocess: u8 HWC images [B, S, S, 3] (x unused)
  int S;
  const bf16* w;      // [64, 224]
  const bf16* w2;     // [64, 160] dense-K order (stem_roles_kernel<.., V & 2>), may be null
  const float* bias;  // [64]
  bf16* y;            // [B, PH, PW, 64]
  int Hp, Wq, PH, PW, strip;
  // The second half of the grid (at 2 workgroups per CU: each CU's second
  // workgroup) starts stagger x ~2048 cycles late. The two workgroups of a CU
  // otherwise run in lockstep: both in their MFMA phase, then both in the
  // barrier-separated VALU phase (vertical max, u8 conversion) with the
  // matrix pipes idle. 100.9 -> 93.0 us at B = 256 with 2
  // (profiles/r3_stem_knockouts.txt).
  int stagger;
  int rstagger;  // the one-image-per-workgroup kernel: start_stagger (common.h)
  // measurement hook (stem_conv_pool_set_stamps): per-step phase stamps of
  // the one-image-per-workgroup kernel's first kStemStampWgs workgroups
  // (100 MHz), or null
  unsigned long long* stamps;
};
constexpr int kStemStampWgs = 16;
constexpr int kStemStagger = 2;

template <int N>
__device__ __forceinline__ void vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}

// LDS address of a pointer into __shared__ memory.
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}

// 16-bit LDS stores issued as inline asm: the compiler's waitcnt pass would
// otherwise put an s_waitcnt vmcnt(0) in front of every LDS store (it cannot
// tell them apart from the in-flight LDS-DMA of the input ring), stalling
// the epilogue on the next step's prefetch. lds_barrier() waits lgkmcnt(0).
// `off` must fold to a constant (it becomes the instruction's offset field).
__device__ __forceinline__ void ds_write_lo16(uint32_t addr, uint32_t v, const int off) {
  asm volatile("ds_write_b16 %0, %1 offset:%2" ::"v"(addr), "v"(v), "i"(off));
}
__device__ __forceinline__ void ds_write_hi16(uint32_t addr, uint32_t v, const int off) {
  asm volatile("ds_write_b16_d16_hi %0, %1 offset:%2" ::"v"(addr), "v"(v), "i"(off));
}

__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
}

// y[l] = x[(l - 16) mod 64]: rotate the wave's four 16-lane rows down by one
// with the gfx950 row-swap permutes (VALU only; a ds_bpermute here made each
// of the 4 channel blocks of a fragment epilogue wait a full LDS round trip,
// and its lgkmcnt wait also drained the epilogue's own LDS stores).
// permlane32_swap(x, x): [0] = rows (0,1,0,1), [1] = rows (2,3,2,3);
// z = rows (2,3,0,1); permlane16_swap(z, x): [0] = (2,0,0,2), [1] = (3,1,1,3):
// odd rows from [0], even rows from [1].
// Semantics checked on the GPU by tools/probes/permlane_probe.hip.
__device__ __forceinline__ float rot_rows_down1(float x, int lane) {
  const unsigned u = __float_as_uint(x);
  const auto p32 = __builtin_amdgcn_permlane32_swap(u, u, false, false);
  const unsigned z = lane < 32 ? p32[1] : p32[0];
  const auto p16 = __builtin_amdgcn_permlane16_swap(z, u, false, false);
  return __uint_as_float((lane & 16) ? p16[0] : p16[1]);
}

// Horizontal 3-max + ReLU of one output-column fragment in packed bf16 (the
// bias is already in the accumulators: they start from it). Lane (r, g) holds
// columns 16f + 4g + i (i = 0..3) of channel 16n + r. Rounding is monotone,
// so round-then-max equals the fp32 max-then-round: each block converts its 4
// values (2 cvt), pooled column 8f + 2g + 1 = max(v1, v2, v3) and 8f + 2g =
// max(v0, v1, nb) come out of two packed i16 maxes over (v0, v1) | (v1, v2) |
// (nb, v3) and one ReLU, and
// nb (column 16f + 4g - 1: v3 of row g - 1, of row 3 of fragment f-1 for g
// = 0) moves between lanes as bf16 pairs, two channel blocks per row
// rotation instead of one fp32 each. 0 is the neutral left pad (values >= 0).
// 89.6 vs 90.9 us for the role-split stem at B = 256 against the fp32 max +
// bias-add epilogue (profiles/r4_stem_roles.txt).


template <int NB>
__device__ __forceinline__ void hpool_packed(const floatx4 (&acc)[NB], uint32_t (&prevq)[(NB + 1) / 2], int lane,
                                             int fq, uint32_t hbase, const int f, const int off) {
  uint32_t p01[NB], p23[NB];
#pragma unroll
  for (int n = 0; n < NB; ++n) {  // (no ReLU yet: see below)
    const float2v a = {acc[n][0], acc[n][1]}, b = {acc[n][2], acc[n][3]};
    p01[n] = __builtin_bit_cast(uint32_t, __builtin_convertvector(a, bf16x2));
    p23[n] = __builtin_bit_cast(uint32_t, __builtin_convertvector(b, bf16x2));
  }
  constexpr int NQ = (NB + 1) / 2;
  uint32_t r[NQ];
#pragma unroll
  for (int j = 0; j < NQ; ++j) {
    // (v3 of block 2j, v3 of block 2j+1)
    const uint32_t q = 2 * j + 1 < NB ? __builtin_amdgcn_perm(p23[2 * j + 1], p23[2 * j], 0x07060302u) : p23[2 * j];
    const uint32_t src = (f > 0 && fq == 3) ? prevq[j] : q;
    uint32_t rr = __float_as_uint(rot_rows_down1(__uint_as_float(src), lane));
    if (f == 0) rr = fq == 0 ? 0u : rr;
    r[j] = rr;
    prevq[j] = q;
  }
#pragma unroll
  for (int n = 0; n < NB; ++n) {
    // (nb, v3): nb from half (n & 1) of the rotated pair (a lone block's pair
    // carries its v3 in the high half)
    const uint32_t c = __builtin_amdgcn_perm(p23[n], r[n >> 1], (n & 1) || NB == 1 ? 0x07060302u : 0x07060100u);
    const uint32_t b12 = __builtin_amdgcn_alignbit(p23[n], p01[n], 16);  // (v1, v2)
    // signed 16-bit max on the raw bf16 bits: exact whenever the window's
    // maximum is >= 0 (non-negative bf16 order as int16 and above every
    // negative one); when all three are negative it returns some negative
    // value, which the ReLU after the max turns into 0 = relu(max) anyway.
    // One ReLU per pair of pooled columns instead of two per block of four
    // conv columns; the 0 left pad stays neutral (relu(max(0, a, b)) =
    // relu(max(a, b)))
    const short2v m = __builtin_elementwise_max(
        __builtin_elementwise_max(
            __builtin_elementwise_max(__builtin_bit_cast(short2v, p01[n]), __builtin_bit_cast(short2v, b12)),
            __builtin_bit_cast(short2v, c)),
        short2v{0, 0});
    const uint32_t packed = __builtin_bit_cast(uint32_t, m);
    ds_write_lo16(hbase, packed, off + n * 32);
    ds_write_hi16(hbase, packed, off + n * 32 + kHpCol);
  }
}

// The same epilogue without the cross-lane exchange (the dense-K stem when
// its LDS has room for an edge ring): pooled column 2G (G = the lane's
// 4-column group) is stored without its left neighbour, as
// relu(max(v0, v1)), and the lane stores relu(v3) of its group into the edge
// ring ([G][64 ch], same 144-B stride); the helpers' vertical pass takes
// max(., edge[G - 1]) for even pooled columns. Per block: 2 cvt, alignbit, 3
// packed max, and -- 3 16-bit stores instead of the row rotation's ~12
// instructions per pair of blocks (the stem's MFMA waves are issue-bound:
// profiles/r6_stem_dense.txt).
template <int NB>
__device__ __forceinline__ void hpool_edge(const floatx4 (&acc)[NB], uint32_t hbase, uint32_t ebase, const int off,
                                           const int eoff) {
#pragma unroll
  for (int n = 0; n < NB; ++n) {
    const float2v a = {acc[n][0], acc[n][1]}, b = {acc[n][2], acc[n][3]};
    const uint32_t p01 = __builtin_bit_cast(uint32_t, __builtin_convertvector(a, bf16x2));
    const uint32_t p23 = __builtin_bit_cast(uint32_t, __builtin_convertvector(b, bf16x2));
    const uint32_t b12 = __builtin_amdgcn_alignbit(p23, p01, 16);  // (v1, v2)
    // (relu v2, relu v3): signed 16-bit max on bf16 bits, exact against 0
    const short2v r23 = __builtin_elementwise_max(__builtin_bit_cast(short2v, p23), short2v{0, 0});
    const uint32_t c = __builtin_bit_cast(uint32_t, r23) & 0xffff0000u;  // (0, relu v3)
    // lo = max(v0, v1, 0), hi = max(v1, v2, relu v3) = relu(max(v1, v2, v3))
    const short2v m = __builtin_elementwise_max(
        __builtin_elementwise_max(__builtin_bit_cast(short2v, p01), __builtin_bit_cast(short2v, b12)),
        __builtin_bit_cast(short2v, c));
    const uint32_t packed = __builtin_bit_cast(uint32_t, m);
    // compiler-visible stores (its lgkmcnt waits then count them: inline-asm
    // stores issued after the next fragment's operand loads made its waits
    // drain those loads; the MFMA waves have no DMA in flight)
    typedef __attribute__((address_space(3))) uint16_t lds_u16;
    *(lds_u16*)(uintptr_t)(hbase + off + n * 32) = (uint16_t)packed;
    *(lds_u16*)(uintptr_t)(hbase + off + n * 32 + kHpCol) = (uint16_t)(packed >> 16);
    *(lds_u16*)(uintptr_t)(ebase + eoff + n * 32) = (uint16_t)(__builtin_bit_cast(uint32_t, r23) >> 16);
  }
}

// The whole geometry follows from the image size S = 32 NF (NF = output
// column fragments): compile-time constants, so the row / ring / column
// arithmetic is shifts and constant multiplies instead of v_mul_lo_u32 (a
// quarter-rate VALU op) on runtime sizes.
template <int NF>
struct StemGeom {
  static constexpr int S = 32 * NF, Ho = 16 * NF, PH = 8 * NF, PW = 8 * NF, Hp = S + 6;
  static constexpr int need = ((Ho - 1) * 6 + 26) / 3;  // stem_row_width(S, 3, 7, 2)
  static constexpr int Wr = ((S + 6 > need ? S + 6 : need) + 7) / 8 * 8;
  static constexpr int Wq = Wr / 2;  // paired 16-B chunks per staged row
  // the u8 conversion's last 28-byte window ends this far past the raw row
  static_assert(24 * ((Wq + 3) / 4) - 8 - 3 * S <= kU8Pad - kU8Front, "raw ring pad");
};

// CS (channel split, query batches): the workgroup computes 64 / CS of the
// 64 output channels (blockIdx.y picks which), so a batch too small to
// fill the CUs with strips runs CS x as many workgroups (each converts the
// same input rows: cheap next to the MFMAs it no longer does).
template <int NF, bool U8, int CS = 1>
__global__ __launch_bounds__(256, 2) void stem_conv_pool_kernel(
    StemArgs a) {
  using G = StemGeom<NF>;
  extern __shared__ __attribute__((aligned(16))) uint4 smem[];
  constexpr int RING = U8 ? kRingU8 : kRing;
  const int RB = G::Wq * 16;  // bytes per staged input row
  const int UB = G::S * 3;    // bytes per raw u8 image row (U8)
  const int UBS = UB + kU8Pad;  // raw ring slot
  char* ring = (char*)smem;
  char* hp = ring + RING * RB;
  char* u8ring = hp + kHp * G::PW * kHpCol;  // U8: raw rows, slot = row % RING
  const int HPB = G::PW * kHpCol;  // bytes per pooled conv row

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: row math in SGPRs
  const int fr = lane & 15, fq = lane >> 4;
  const int strips = G::PH / a.strip;
  const int b = blockIdx.x / strips;
  const int ph0 = (blockIdx.x - b * strips) * a.strip;
  const int T = a.strip / 2;  // steps 1..T emit pooled rows
  const bf16* img = a.x + (long)b * G::Hp * G::Wq * 8;
  constexpr int NB = 4 / CS;  // 16-channel blocks of this workgroup
  static_assert(CS == 1 || CS == 2 || CS == 4, "channel split");
  const int nb0 = CS == 1 ? 0 : blockIdx.y * NB;

  // This wave's share of a row list [lo, lo+cnt): rows lo+wave, lo+wave+4, ...
  // (U8: padded row r is image row r-3; rows outside the image are not
  // loaded, convert_rows writes them as zeros.)
  const uint8_t* uimg = U8 ? a.u8 + (long)b * G::S * G::S * 3 : nullptr;
  auto load_rows = [&](int lo, int cnt) __attribute__((always_inline)) {
    for (int i = wave; i < cnt; i += 4) {
      const int r = lo + i;
      if (r < 0) continue;
      if constexpr (U8) {
        const int iy = r - 3;
        if (iy < 0 || iy >= G::S) continue;
        const uint8_t* src = uimg + (long)iy * UB;
        char* dst = u8ring + (r % RING) * UBS + kU8Front;
        for (int c0 = 0; c0 < UB / 4; c0 += 64)
          if (c0 + lane < UB / 4)
            dma4(src + (c0 + lane) * 4, dst + c0 * 4);
      } else {
        const bf16* src = img + (long)r * G::Wq * 8;
        char* dst = ring + (r % RING) * RB;
        for (int c0 = 0; c0 < G::Wq; c0 += 64) {
          if (c0 + lane < G::Wq)
            dma16(src + (c0 + lane) * 8, dst + c0 * 16);
        }
      }
    }
  };
  // U8: raw rows [lo, lo+cnt) -> paired bf16 ring rows, exactly the
  // preprocess_u8(paired) values: chunk p = image columns 2p-3, 2p-2 as
  // [r g b r g b 0 0], (v/255 - mean)/std, zeros outside the image. A thread
  // converts 4 chunks (8 pixels = 24 bytes starting at byte 24k-9 of the
  // row) from 7 aligned dword reads starting at 24k-12.
  auto convert_rows = [&](int lo, int cnt) __attribute__((always_inline)) {
    const int G4 = (G::Wq + 3) / 4;
    const int items = cnt * G4;
    for (int it = tid; it < items; it += 256) {
      const int r = lo + it / G4;
      const int k = it - (it / G4) * G4;
      if (r < 0) continue;
      const int iy = r - 3;
      const bool row_in = iy >= 0 && iy < G::S;
      const char* srow = u8ring + (r % RING) * UBS + kU8Front;
      const int A = 24 * k - 12;
      // all 7 reads unconditional from one base (the slot's zero pads cover
      // the window's overhang at the row ends; a guarded read per dword had
      // compiled to an exec-masked branch each, the first with its own wait)
      uint32_t d[7];
#pragma unroll
      for (int j = 0; j < 7; ++j) d[j] = row_in ? *(const uint32_t*)(srow + A + 4 * j) : 0u;
      float v[32];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int ix = 8 * k - 3 + i;
        const bool in = row_in && ix >= 0 && ix < G::S;
#pragma unroll
        for (int c = 0; c < 3; ++c) {
          const int idx = 3 + 3 * i + c;
          const float cv = (float)((d[idx >> 2] >> (8 * (idx & 3))) & 0xffu);
          const float nv = imagenet_norm(c, cv);
          v[8 * (i >> 1) + 3 * (i & 1) + c] = in ? nv : 0.f;
        }
      }
      char* drow = ring + (r % RING) * RB;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        v[8 * q + 6] = v[8 * q + 7] = 0.f;
        if (4 * k + q < G::Wq) *(uint4*)(drow + (4 * k + q) * 16) = pack8(v + 8 * q);
      }
    }
  };

  // Weights in registers: wf[n][s] = W[16n + fr][32s + 8fq .. +8].
  bf16x8 wf[NB][7];
#pragma unroll
  for (int n = 0; n < NB; ++n)
#pragma unroll
    for (int s = 0; s < 7; ++s)
      wf[n][s] = *(const bf16x8*)(a.w + ((nb0 + n) * 16 + fr) * kK + s * 32 + fq * 8);
  float bs[NB];
#pragma unroll
  for (int n = 0; n < NB; ++n) bs[n] = a.bias[(nb0 + n) * 16 + fr];

  if (a.stagger && blockIdx.x >= gridDim.x / 2)  // (a wave-uniform scalar loop)
    for (int i = 0; i < a.stagger; ++i) __builtin_amdgcn_s_sleep(32);  // ~2048 cycles each
  if constexpr (U8) {  // the raw ring's pads stay zero (the DMA writes rows only)
    for (int o = tid * 16; o < RING * UBS; o += 256 * 16) *(uint4*)(u8ring + o) = make_uint4(0, 0, 0, 0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  }
  // Prologue: rows for step 0 (the 13 rows of c0(0), negative ones skipped).
  load_rows(4 * ph0 - 8, 13);
  vm_wait<0>();
  __builtin_amdgcn_s_barrier();
  if constexpr (U8) {
    convert_rows(4 * ph0 - 8, 13);
    lds_barrier();
  }

  for (int t = 0; t <= T; ++t) {
    const int c0 = 2 * ph0 - 4 + 4 * t;
    if (t < T) load_rows(2 * c0 + 13, 8);  // next step's new rows

    const int cr = c0 + wave;  // this wave's conv row
    char* hrow = hp + ((cr + kHp) % kHp) * HPB;
    if (t > 0 || wave == 3) {
      if (cr < 0) {  // row above the image: neutral zero row for the max
        for (int o = lane * 16; o < HPB; o += 64 * 16) *(uint4*)(hrow + o) = make_uint4(0, 0, 0, 0);
      } else {
        // Fragment-major: the 28 MFMAs of output columns 16f..16f+15 (7
        // kernel rows x 4 channel blocks), then that fragment's pooling
        // epilogue, which the scheduler can overlap with fragment f+1's
        // MFMAs. Only two fragments' accumulators are ever live.
        const char* rbase = ring + (fr + fq) * 16;
        int rows[7];
#pragma unroll
        for (int s = 0; s < 7; ++s) rows[s] = ((2 * cr + s) % RING) * RB;
        // per-lane store base: column 2g, channel chunk r/8, element r%8
        const uint32_t hbase = lds_addr(hrow) + fq * 2 * kHpCol + (fr >> 3) * 16 + (fr & 7) * 2 + nb0 * 32;
        uint32_t prevq[(NB + 1) / 2];  // column 16f+15 of the previous fragment, bf16 pairs of channel blocks
        bf16x8 xf[7];
#pragma unroll
        for (int s = 0; s < 7; ++s) xf[s] = *(const bf16x8*)(rbase + rows[s]);
#pragma unroll
        for (int f = 0; f < NF; ++f) {
          floatx4 acc[NB];
#pragma unroll
          for (int n = 0; n < NB; ++n)
            acc[n] = floatx4{bs[n], bs[n], bs[n], bs[n]};  // the bias first (hpool_packed)
#pragma unroll
          for (int s = 0; s < 7; ++s)
#pragma unroll
            for (int n = 0; n < NB; ++n)
              acc[n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xf[s], wf[n][s], acc[n], 0, 0, 0);
          // The next fragment's operands go out before this epilogue so the
          // reads land under it.
          if (f + 1 < NF) {
#pragma unroll
            for (int s = 0; s < 7; ++s)
              xf[s] = *(const bf16x8*)(rbase + rows[s] + (f + 1) * 256);
          }
          // horizontal 3-max over columns (2pw-1, 2pw, 2pw+1) + ReLU (the
          // bias is in the accumulators)
          hpool_packed<NB>(acc, prevq, lane, fq, hbase, f, f * 8 * kHpCol);
        }
      }
    }
    // One barrier between the MFMA phase and the pooled-row / conversion
    // phase: the next step's rows (issued at the top of the step) have landed
    // by now, so the wait for them moves ahead of it and the vertical max and
    // the u8 conversion share one phase (they touch disjoint LDS).
    vm_wait<0>();
    lds_barrier();
    if (t > 0) {  // vertical 3-max -> pooled rows ph, ph+1
      const int ph = ph0 + 2 * (t - 1);
      constexpr int CG = 8 / CS;  // this workgroup's 8-channel groups
      const int per_row = G::PW * CG;
      ushort8 m[4];  // 16*PW <= 1024 items: at most 4 per thread, reads issued together
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int it = tid + j * 256;
        if (it < 2 * per_row) {
          const int pr = it >= per_row;
          const int rem = it - pr * per_row;
          const int pw = rem / CG, cg = rem % CG + (CS == 1 ? 0 : CG * (int)blockIdx.y);
          const int r1 = 2 * (ph + pr) - 1;
          const int off = pw * kHpCol + cg * 16;
          const ushort8 v1 = *(const ushort8*)(hp + ((r1 + kHp) % kHp) * HPB + off);
          const ushort8 v2 = *(const ushort8*)(hp + ((r1 + 1) % kHp) * HPB + off);
          const ushort8 v3 = *(const ushort8*)(hp + ((r1 + 2) % kHp) * HPB + off);
          m[j] = __builtin_elementwise_max(__builtin_elementwise_max(v1, v2), v3);
        }
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int it = tid + j * 256;
        if (it < 2 * per_row) {
          const int pr = it >= per_row;
          const int rem = it - pr * per_row;
          *(ushort8*)(a.y + (((long)b * G::PH + ph + pr) * G::PW + rem / CG) * 64 +
                      (rem % CG + (CS == 1 ? 0 : CG * (int)blockIdx.y)) * 8) = m[j];
        }
      }
    }
    if constexpr (U8) {
      // the next step's raw rows landed; the paired rows they replace were
      // last read by this step's MFMAs (before the barrier above)
      if (t < T) convert_rows(2 * c0 + 13, 8);
    }
    // the next step's MFMAs overwrite pooled rows read above and read the
    // converted rows
    lds_barrier();
  }
}


// ---- Role-split stem (one workgroup per image, B >= the CU count): the same
// arithmetic as stem_conv_pool_kernel<NF, true>, but the VALU phase no longer
// stalls the matrix pipes. In the strip kernel every step is [MFMA +
// horizontal pool] | barrier | [vertical max + stores + u8 conversion] |
// barrier, and the VALU phase (~30% of the kernel by knock-outs,
// profiles/r3_stem_knockouts.txt) runs with the matrix pipes idle. Here 8
// waves: waves 0-3 (one per SIMD) only compute conv rows and their
// horizontal max into the hp ring; waves 4-7 (their SIMD partners) DMA raw
// rows, convert them for the next step and do the vertical max and stores of
// the previous step. One barrier per step:
//   step t (0..T+1, T = PH/2 steps of 4 conv rows):
//     MFMA waves (t <= T): conv rows 4t-4 .. 4t-1 (t = 0: only the zero row -1)
//       from paired rows 8t-8 .. 8t+4 -> hp rows;
//     helper waves: raw rows 8t+21 .. 8t+28 DMA'd (converted at t+2), pooled
//       rows 2(t-2), 2(t-2)+1 = max of hp rows 4t-9 .. 4t-5 (t >= 2) -> y,
//       paired rows 8t+5 .. 8t+12 converted (read by step t+1; t < T); then
//       each waits for its DMAs of step t-1 only (the stores and this step's
//       DMAs stay in flight).
// Rings: paired 21 rows (13 read + 8 written), hp 9 rows (4 written + 5
// read), raw 24 rows (8 converted + 16 in flight): 130 KB at 224x224.
constexpr int kRolesPairRing = 21, kRolesHpRing = 9, kRolesRawRing = 24;

// s_waitcnt vmcnt(n) for a wave-uniform runtime n (n > 15 waits for 15)
__device__ __forceinline__ void vm_wait_dyn(int n) {
  switch (n) {
#define DMLC_VMW(N) \
  case N: vm_wait<N>(); break;
    DMLC_VMW(1) DMLC_VMW(2) DMLC_VMW(3) DMLC_VMW(4) DMLC_VMW(5) DMLC_VMW(6) DMLC_VMW(7) DMLC_VMW(8) DMLC_VMW(9)
    DMLC_VMW(10) DMLC_VMW(11) DMLC_VMW(12) DMLC_VMW(13) DMLC_VMW(14)
#undef DMLC_VMW
    case 0: vm_wait<0>(); break;
    default: vm_wait<15>(); break;
  }
}

// V bit 1: the raw rows by 16-B LDS-DMA (one instruction per 672-B row
// instead of three 4-B ones; the u8 images must be 16-B aligned, which the
// launcher checks). (Knock-out timings of the phases: profiles/r4_stem_roles.txt,
// profiles/r6_stem_dense.txt.)
//
// V bit 2: dense K. The paired rows above hold [r g b r g b 0 0] chunks and
// a kernel row takes one 32-wide K step of 8 pixels: 7 x 32 = 224 K for 147
// taps (66% of the MFMAs useful). Dense rows hold the padded row as plain
// [px][rgb] bf16 (3 * (S + 6) elements, 48 B per 8 pixels: helper stores at
// a 48-B lane stride, conflict-free), and K runs over the 7 kernel rows'
// 22-element windows (7 px x rgb + 1 zero-weight slot): 154 of 160 = 5 K
// steps, 20 MFMAs a fragment instead of 28. Each operand is four ds_read_b32
// (one window dword each) at per-lane addresses computed once per conv row;
// which dword a lane group reads in which slot is stem_dense_cell
// (kernels.h): in every 32-lane half the same dword of an even and an odd
// kernel row, and odd rows sit 64 B (16 banks) further into their ring slot
// (slots a multiple of 128 B), so the two halves' 3 fr + u dword patterns
// never share a bank (18 of 20 slots; a lane pattern over one bank window
// costs the ds_read_b32 2 cycles a half-wave instead of 1). The pooling
// epilogue skips the cross-lane neighbour column when the edge ring fits
// (hpool_edge; RolesLds::EDGE). Weights: stem_dense_k_index (kernels.h),
// [64][160].
//
// LDS layout of the role-split stem (kernel and launcher): paired / dense
// ring, hp ring, edge ring (dense K, where it fits in 160 KB: S <= 224), raw
// ring.
template <int NF, bool DK>
struct RolesLds {
  using G = StemGeom<NF>;
  static constexpr int NG = 4 * NF + 1;            // dense rows: 8-pixel groups of the S + 6 padded pixels
  static constexpr int RB = DK ? NG * 48 : G::Wq * 16;  // bytes per paired / dense row
  // ring slot stride: dense slots a multiple of 128 B with room for the odd
  // rows' 64-B offset
  static constexpr int RBS = DK ? (RB + 64 + 127) / 128 * 128 : RB;
  static constexpr int HPB = G::PW * kHpCol;       // bytes per horizontally pooled conv row
  static constexpr int EPB = G::PW / 2 * kHpCol;   // edge row: relu(v3) per 4-column group
  static constexpr int UBS = G::S * 3 + kU8Pad;    // raw ring slot
  static constexpr int base = kRolesPairRing * RBS + kRolesHpRing * HPB + kRolesRawRing * UBS;
  static constexpr bool EDGE = DK && base + kRolesHpRing * EPB <= 160 * 1024;
  static constexpr int bytes = base + (EDGE ? kRolesHpRing * EPB : 0);
  static_assert(bytes <= 160 * 1024, "role-split LDS budget");
};

template <int NF, int V = 0>
__global__ __launch_bounds__(512, 1) void stem_roles_kernel(StemArgs a) {
  using G = StemGeom<NF>;
  extern __shared__ __attribute__((aligned(16))) uint4 smem[];
  constexpr bool DK = (V & 2) != 0;
  using L = RolesLds<NF, DK>;
  constexpr int NG = L::NG;
  static_assert(NG * 8 >= G::S + 6, "dense row groups");
  constexpr int RB = L::RB, RBS = L::RBS;
  constexpr bool EDGE = L::EDGE;
  static_assert(!DK || 12 * (16 * NF - 1) + 4 * 10 + 4 <= RB, "dense window reads stay in the row");
  constexpr int UB = G::S * 3;        // bytes per raw image row
  constexpr int UBS = L::UBS;         // raw ring slot
  constexpr int HPB = L::HPB, EPB = L::EPB;
  constexpr int T = G::PH / 2;
  char* ring = (char*)smem;
  char* hp = ring + kRolesPairRing * RBS;
  char* edge = hp + kRolesHpRing * HPB;  // (EDGE only)
  // byte offset of padded row r (>= 0) in the paired / dense ring
  auto row_off = [](int r) __attribute__((always_inline)) { return (r % kRolesPairRing) * RBS + (DK ? 64 * (r & 1) : 0); };
  char* u8ring = edge + (EDGE ? kRolesHpRing * EPB : 0);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  start_stagger(a.rstagger);
  const bool mfma_wave = wave < 4;
  const int hw = wave & 3, htid = tid & 255;  // helper wave / thread index among the helpers
  const int fr = lane & 15, fq = lane >> 4;
  const int b = blockIdx.x;
  const uint8_t* uimg = a.u8 + (long)b * G::S * G::S * 3;

  // raw padded rows [lo, lo+cnt) (image row = padded row - 3) -> raw ring, by the helpers
  auto load_rows = [&](int lo, int cnt) __attribute__((always_inline)) {
    for (int i = hw; i < cnt; i += 4) {
      const int r = lo + i, iy = r - 3;
      if (iy < 0 || iy >= G::S) continue;
      const uint8_t* src = uimg + (long)iy * UB;
      char* dst = u8ring + (r % kRolesRawRing) * UBS + kU8Front;
      if constexpr (V & 1) {
        static_assert(UB % 16 == 0 && UB / 16 <= 64 && UBS % 16 == 0 && kU8Front % 16 == 0, "16-B raw rows");
        if (lane < UB / 16) dma16(src + lane * 16, dst);
      } else {
        for (int c0 = 0; c0 < UB / 4; c0 += 64)
          if (c0 + lane < UB / 4) dma4(src + (c0 + lane) * 4, dst + c0 * 4);
      }
    }
  };
  // raw rows [lo, lo+cnt) -> paired bf16 rows (stem_conv_pool_kernel's
  // convert_rows, over nthr threads)
  auto convert_rows = [&](int lo, int cnt, int t0, int nthr) __attribute__((always_inline)) {
    if constexpr (DK) {
      // item = (row, group g): padded pixels 8g .. 8g+7 (image columns 8g-3 ..
      // 8g+4) -> 24 bf16 at byte 48 g of the dense row, three 16-B stores.
      // Items of the inner groups 1 .. NG-2 (every pixel inside the image
      // columns) come first and convert without per-element selects; the 2
      // edge groups of each row (zero padding, per element) last, on the last
      // lanes, so only one helper wave takes that path.
      constexpr int NI = NG - 2;
      const int items = cnt * NG;
      for (int it = t0; it < items; it += nthr) {
        const bool inner = it < cnt * NI;
        const int e = it - cnt * NI;
        const int r = lo + (inner ? it / NI : e >> 1);
        const int g = inner ? 1 + it % NI : ((e & 1) ? NG - 1 : 0);
        if (r < 0) continue;
        const int iy = r - 3;
        const bool row_in = iy >= 0 && iy < G::S;
        const char* srow = u8ring + (r % kRolesRawRing) * UBS + kU8Front;
        const int A = 24 * g - 12;
        uint32_t d[7];
#pragma unroll
        for (int j = 0; j < 7; ++j) d[j] = *(const uint32_t*)(srow + A + 4 * j);
        float v[24];
        if (inner && row_in) {
#pragma unroll
          for (int i = 0; i < 24; ++i) {
            const int idx = 3 + i;
            v[i] = imagenet_norm(i % 3, (float)((d[idx >> 2] >> (8 * (idx & 3))) & 0xffu));
          }
        } else {
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            const int ix = 8 * g - 3 + i;
            const bool in = row_in && ix >= 0 && ix < G::S;
#pragma unroll
            for (int c = 0; c < 3; ++c) {
              const int idx = 3 + 3 * i + c;
              const float cv = (float)((d[idx >> 2] >> (8 * (idx & 3))) & 0xffu);
              v[3 * i + c] = in ? imagenet_norm(c, cv) : 0.f;
            }
          }
        }
        char* drow = ring + row_off(r) + g * 48;
#pragma unroll
        for (int q = 0; q < 3; ++q) *(uint4*)(drow + q * 16) = pack8(v + 8 * q);
      }
      return;
    }
    const int G4 = (G::Wq + 3) / 4;
    const int items = cnt * G4;
    for (int it = t0; it < items; it += nthr) {
      const int r = lo + it / G4;
      const int k = it - (it / G4) * G4;
      if (r < 0) continue;
      const int iy = r - 3;
      const bool row_in = iy >= 0 && iy < G::S;
      const char* srow = u8ring + (r % kRolesRawRing) * UBS + kU8Front;
      const int A = 24 * k - 12;
      uint32_t d[7];
#pragma unroll
      for (int j = 0; j < 7; ++j) d[j] = row_in ? *(const uint32_t*)(srow + A + 4 * j) : 0u;
      float v[32];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int ix = 8 * k - 3 + i;
        const bool in = row_in && ix >= 0 && ix < G::S;
#pragma unroll
        for (int c = 0; c < 3; ++c) {
          const int idx = 3 + 3 * i + c;
          const float cv = (float)((d[idx >> 2] >> (8 * (idx & 3))) & 0xffu);
          const float nv = imagenet_norm(c, cv);
          v[8 * (i >> 1) + 3 * (i & 1) + c] = in ? nv : 0.f;
        }
      }
      char* drow = ring + row_off(r);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        v[8 * q + 6] = v[8 * q + 7] = 0.f;
        if (4 * k + q < G::Wq) *(uint4*)(drow + (4 * k + q) * 16) = pack8(v + 8 * q);
      }
    }
  };

  constexpr int KS = DK ? kKD / 32 : 7;  // K steps a fragment
  bf16x8 wf[4][KS];
  float bs[4];
  if (mfma_wave) {
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
      for (int s = 0; s < KS; ++s)
        wf[n][s] = DK ? *(const bf16x8*)(a.w2 + (n * 16 + fr) * kKD + s * 32 + fq * 8)
                      : *(const bf16x8*)(a.w + (n * 16 + fr) * kK + s * 32 + fq * 8);
#pragma unroll
    for (int n = 0; n < 4; ++n) bs[n] = a.bias[n * 16 + fr];
  }
  // raw ring pads stay zero; prologue: raw rows 0..20 (converted before step
  // 0 and at steps 0, 1), rows 0..4 converted by everyone (step 0 reads
  // paired rows -8..4)
  for (int o = tid * 16; o < kRolesRawRing * UBS; o += 512 * 16) *(uint4*)(u8ring + o) = make_uint4(0, 0, 0, 0);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  if (!mfma_wave) load_rows(0, 21);
  vm_wait<0>();
  __builtin_amdgcn_s_barrier();
  convert_rows(0, 5, tid, 512);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();

  // stamps[(b * (T + 2) + t) * 4 + k]: k = 0 step start / 1 MFMA phase done
  // (wave 0), 2 helper work issued / 3 helper waits done (wave 4)
  unsigned long long* stp = (a.stamps && b < kStemStampWgs && (wave == 0 || wave == 4) && lane == 0)
                                ? a.stamps + (long)b * (T + 2) * 4
                                : nullptr;
  for (int t = 0; t <= T + 1; ++t) {
    if (stp && wave == 0) stp[4 * t] = __builtin_amdgcn_s_memrealtime();
    if (mfma_wave) {
      if (t <= T) {
        const int c0 = 4 * t - 4;
        const int cr = c0 + wave;
        char* hrow = hp + ((cr + kRolesHpRing) % kRolesHpRing) * HPB;
        char* erow = edge + ((cr + kRolesHpRing) % kRolesHpRing) * EPB;  // (EDGE only)
        if (cr < 0) {
          if (wave == 3) {
            for (int o = lane * 16; o < HPB; o += 64 * 16) *(uint4*)(hrow + o) = make_uint4(0, 0, 0, 0);
            if constexpr (EDGE)
              for (int o = lane * 16; o < EPB; o += 64 * 16) *(uint4*)(erow + o) = make_uint4(0, 0, 0, 0);
          }
        } else if constexpr (DK) {
          // per-lane operand addresses of this conv row (stem_dense_cell):
          // slots 0..14 from one base per kernel-row pair plus an immediate,
          // 15..19 one register each; fragment f adds 16 * 12 * f bytes
          // (wave-uniform slot bases as separate values, not an array: a
          // lane-selected index into one would go through scratch)
          const int lane_off = 12 * fr;
          auto cell_off = [&](int j, int c) __attribute__((always_inline)) {
            const StemDenseCell cell = stem_dense_cell(j, c);
            return row_off(2 * cr + cell.dy) + 4 * cell.u;
          };
          int ad[8];
#pragma unroll
          for (int rp = 0; rp < 3; ++rp)
            ad[rp] = lane_off + 4 * (fq >> 1) + ((fq & 1) ? row_off(2 * cr + 2 * rp + 1) : row_off(2 * cr + 2 * rp));
#pragma unroll
          for (int q = 0; q < 5; ++q) {
            const int v0 = cell_off(15 + q, 0), v1 = cell_off(15 + q, 1), v2 = cell_off(15 + q, 2),
                      v3 = cell_off(15 + q, 3);
            ad[3 + q] = lane_off + (fq == 0 ? v0 : fq == 1 ? v1 : fq == 2 ? v2 : v3);
          }
          const uint32_t hbase = lds_addr(hrow) + fq * 2 * kHpCol + (fr >> 3) * 16 + (fr & 7) * 2;
          const uint32_t ebase = lds_addr(erow) + fq * kHpCol + (fr >> 3) * 16 + (fr & 7) * 2;
          uint32_t prevq[2];
          using u32x4 = uint32_t __attribute__((ext_vector_type(4)));
          // opaque bases, so the compiler does not re-derive (and re-merge)
          // the addresses across K steps / fragments
#pragma unroll
          for (int j = 0; j < 8; ++j) asm volatile("" : "+v"(ad[j]));
          auto slot = [&](int j) __attribute__((always_inline)) { return j < 15 ? ad[j / 5] + 8 * (j % 5) : ad[j - 12]; };
          u32x4 xq[KS], nx[KS];
#pragma unroll
          for (int s = 0; s < KS; ++s)
#pragma unroll
            for (int i = 0; i < 4; ++i) xq[s][i] = *(const uint32_t*)(ring + slot(4 * s + i));
          // Software pipeline, one scheduling region per fragment f: the
          // operand loads of f + 1, the MFMAs of f, and the pooling epilogue of
          // f - 1 (its accumulators long complete: no hazard waits, its VALU
          // and LDS stores fill the MFMA issue gaps)
          floatx4 acc[2][4];
#pragma unroll
          for (int f = 0; f <= NF; ++f) {
            if (f + 1 < NF) {
#pragma unroll
              for (int s = 0; s < KS; ++s)
#pragma unroll
                for (int i = 0; i < 4; ++i) nx[s][i] = *(const uint32_t*)(ring + slot(4 * s + i) + (f + 1) * 192);
            }
            if (f < NF) {
#pragma unroll
              for (int n = 0; n < 4; ++n) acc[f & 1][n] = floatx4{bs[n], bs[n], bs[n], bs[n]};
#pragma unroll
              for (int s = 0; s < KS; ++s)
#pragma unroll
                for (int n = 0; n < 4; ++n)
                  acc[f & 1][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, xq[s]),
                                                                          wf[n][s], acc[f & 1][n], 0, 0, 0);
            }
            if (f > 0) {
              if constexpr (EDGE)
                hpool_edge<4>(acc[(f - 1) & 1], hbase, ebase, (f - 1) * 8 * kHpCol, (f - 1) * 4 * kHpCol);
              else
                hpool_packed<4>(acc[(f - 1) & 1], prevq, lane, fq, hbase, f - 1, (f - 1) * 8 * kHpCol);
            }
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int s = 0; s < KS; ++s) xq[s] = nx[s];
          }
        } else {
          const char* rbase = ring + (fr + fq) * 16;
          int rows[7];
#pragma unroll
          for (int s = 0; s < 7; ++s) rows[s] = row_off(2 * cr + s);
          const uint32_t hbase = lds_addr(hrow) + fq * 2 * kHpCol + (fr >> 3) * 16 + (fr & 7) * 2;
          uint32_t prevq[2];  // v3 of the previous fragment's row 3, as bf16 pairs
          bf16x8 xf[7];
#pragma unroll
          for (int s = 0; s < 7; ++s) xf[s] = *(const bf16x8*)(rbase + rows[s]);
#pragma unroll
          for (int f = 0; f < NF; ++f) {
            floatx4 acc[4];  // starting from the bias (hpool_packed)
#pragma unroll
            for (int n = 0; n < 4; ++n) acc[n] = floatx4{bs[n], bs[n], bs[n], bs[n]};
#pragma unroll
            for (int s = 0; s < 7; ++s)
#pragma unroll
              for (int n = 0; n < 4; ++n)
                acc[n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xf[s], wf[n][s], acc[n], 0, 0, 0);
            if (f + 1 < NF) {
#pragma unroll
              for (int s = 0; s < 7; ++s) xf[s] = *(const bf16x8*)(rbase + rows[s] + (f + 1) * 256);
            }
            hpool_packed<4>(acc, prevq, lane, fq, hbase, f, f * 8 * kHpCol);
          }
        }
      }
      if (stp) stp[4 * t + 1] = __builtin_amdgcn_s_memrealtime();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    } else {
      // DMA the raw rows step t+2's conversion reads: this wave's rows
      // 8t+21+hw and 8t+25+hw, DPR instructions each (rows outside the image
      // are not loaded)
      constexpr int DPR = (V & 1) ? 1 : (UB / 4 + 63) / 64;
      int nwait = 0;
      if (t + 2 < T) {
        load_rows(8 * t + 21, 8);
#pragma unroll
        for (int i = 0; i < 2; ++i) nwait += (8 * t + 21 + hw + 4 * i - 3 < G::S) ? DPR : 0;
      }
      if (t >= 2) {  // vertical 3-max of step t-1's conv rows -> pooled rows ph, ph+1
        const int ph = 2 * (t - 2);
        constexpr int per_row = G::PW * 8;
        ushort8 m[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int it = htid + j * 256;
          if (it < 2 * per_row) {
            const int pr = it >= per_row;
            const int rem = it - pr * per_row;
            const int pw = rem >> 3, cg = rem & 7;
            const int r1 = 2 * (ph + pr) - 1;
            const int off = pw * kHpCol + cg * 16;
            const ushort8 v1 = *(const ushort8*)(hp + ((r1 + kRolesHpRing) % kRolesHpRing) * HPB + off);
            const ushort8 v2 = *(const ushort8*)(hp + ((r1 + 1) % kRolesHpRing) * HPB + off);
            const ushort8 v3 = *(const ushort8*)(hp + ((r1 + 2) % kRolesHpRing) * HPB + off);
            m[j] = __builtin_elementwise_max(__builtin_elementwise_max(v1, v2), v3);
            if constexpr (EDGE) {
              // even pooled column 2G: its left conv column 4G - 1 = relu(v3)
              // of group G - 1 (hpool_edge); none left of G = 0 (zero pad)
              if (!(pw & 1) && pw > 0) {
                const int eo = (pw / 2 - 1) * kHpCol + cg * 16;
                const ushort8 e1 = *(const ushort8*)(edge + ((r1 + kRolesHpRing) % kRolesHpRing) * EPB + eo);
                const ushort8 e2 = *(const ushort8*)(edge + ((r1 + 1) % kRolesHpRing) * EPB + eo);
                const ushort8 e3 = *(const ushort8*)(edge + ((r1 + 2) % kRolesHpRing) * EPB + eo);
                m[j] = __builtin_elementwise_max(m[j], __builtin_elementwise_max(__builtin_elementwise_max(e1, e2), e3));
              }
            }
          }
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int it = htid + j * 256;
          if (it < 2 * per_row) {
            const int pr = it >= per_row;
            const int rem = it - pr * per_row;
            *(ushort8*)(a.y + (((long)b * G::PH + ph + pr) * G::PW + (rem >> 3)) * 64 + (rem & 7) * 8) = m[j];
          }
          nwait += (64 * hw + 256 * j < 2 * per_row) ? 1 : 0;  // a store instruction of this wave
        }
      }
      if (t < T) convert_rows(8 * t + 5, 8, htid, 256);
      // step t-1's DMAs (converted at t+1) have landed: everything but this
      // step's DMAs and stores (vmcnt retires in issue order)
      if (stp) stp[4 * t + 2] = __builtin_amdgcn_s_memrealtime();
      vm_wait_dyn(nwait);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (stp) stp[4 * t + 3] = __builtin_amdgcn_s_memrealtime();
    }
    __builtin_amdgcn_s_barrier();
  }
}

}  // namespace

int stem_pool_u8_pick_strip(int B, int PH, int num_cus) {
  // one image per workgroup (the role-split kernel: 89 vs 100-104 us at
  // B = 256, profiles/r3_stem_knockouts.txt) once that fills the CUs
  return B >= num_cus ? PH : stem_pool_pick_strip(B, PH, num_cus);
}

int stem_pool_pick_strip(int B, int PH, int num_cus) {
  // Largest even divisor of PH whose grid still gives every CU two
  // workgroups (2 fit per CU: 256 VGPRs, ~80 KB LDS each at 224x224).
  int best = 2;
  for (int s = 2; s <= PH; s += 2) {
    if (PH % s) continue;
    if ((long)B * (PH / s) >= 2L * num_cus) best = s;
  }
  return best;
}

namespace {
int g_stem_dbg = 0;
unsigned long long* g_stem_stamps = nullptr;
constexpr long kStemSplitCus = 256;  // MI355X CUs: the channel split fills them at query batches

void stem_launch(const void* x, const uint8_t* u8, const void* w, const void* w2, const float* bias, void* y, int B,
                 int S, int Wq, int strip, hipStream_t s) {
  if (B <= 0) return;
  const int Ho = S / 2, PH = Ho / 2;
  const int NF = Ho / 16;
  if (S % 32 != 0 || NF < 4 || NF > 8) throw std::invalid_argument("stem_conv_pool: image size must be 128..256, %32");
  if (Wq != stem_row_width(S, 3, 7, 2) / 2) throw std::invalid_argument("stem_conv_pool: bad paired row width");
  if (strip < 2 || strip % 2 || PH % strip) throw std::invalid_argument("stem_conv_pool: bad strip");
  if ((!x && !u8) || !w || !bias || !y || ((uintptr_t)x & 15) || ((uintptr_t)u8 & 3) || ((uintptr_t)w & 15) ||
      ((uintptr_t)y & 15) || ((uintptr_t)w2 & 15))
    throw std::invalid_argument("stem_conv_pool: null / misaligned operand");
  StemArgs a;
  a.x = (const bf16*)x;
  a.u8 = u8;
  a.S = S;
  a.w = (const bf16*)w;
  a.w2 = (const bf16*)w2;
  a.bias = bias;
  a.y = (bf16*)y;
  a.Hp = S + 6;
  a.Wq = Wq;
  a.PH = PH;
  a.PW = PH;
  a.strip = strip;
  // g_stem_dbg (tests): 512 force the role-split kernel, 2048 its 4-B raw-row DMA
  a.stagger = (long)B * (PH / strip) >= 512 ? kStemStagger : 0;
  a.rstagger = kernel_stagger(kStagStem);
  a.stamps = g_stem_stamps;
  const size_t lds = u8 ? (size_t)kRingU8 * Wq * 16 + (size_t)kHp * a.PW * kHpCol + (size_t)kRingU8 * (S * 3 + kU8Pad)
                        : (size_t)kRing * Wq * 16 + (size_t)kHp * a.PW * kHpCol;
  const dim3 grid(B * (PH / strip));
  if (u8 && ((g_stem_dbg & 512) || strip == PH)) {
    // one workgroup per image, role-split waves (stem_pool_u8_pick_strip picks
    // strip = PH once the batch gives every CU an image)
    // 16-B raw-row DMA when the images allow it (g_stem_dbg 2048: force the 4-B form)
    const bool d16 = !((uintptr_t)u8 & 15) && !(g_stem_dbg & 2048);
    if (d16 && w2) {  // dense K (the engine packs both weight orders)
      switch (NF) {
#define DMLC_STEM_DENSE_CASE(F) \
  case F: hipLaunchKernelGGL((stem_roles_kernel<F, 3>), dim3(B), dim3(512), (RolesLds<F, true>::bytes), s, a); break;
        DMLC_STEM_DENSE_CASE(4)
        DMLC_STEM_DENSE_CASE(5)
        DMLC_STEM_DENSE_CASE(6)
        DMLC_STEM_DENSE_CASE(7)
        DMLC_STEM_DENSE_CASE(8)
#undef DMLC_STEM_DENSE_CASE
      }
      DMLC_HIP_CHECK(hipGetLastError());
      return;
    }
    switch (NF * 2 + (d16 ? 1 : 0)) {
#define DMLC_STEM_ROLES_CASE(F) \
  case 2 * F: \
    hipLaunchKernelGGL((stem_roles_kernel<F>), dim3(B), dim3(512), (RolesLds<F, false>::bytes), s, a); \
    break; \
  case 2 * F + 1: \
    hipLaunchKernelGGL((stem_roles_kernel<F, 1>), dim3(B), dim3(512), (RolesLds<F, false>::bytes), s, a); \
    break;
      DMLC_STEM_ROLES_CASE(4)
      DMLC_STEM_ROLES_CASE(5)
      DMLC_STEM_ROLES_CASE(6)
      DMLC_STEM_ROLES_CASE(7)
      DMLC_STEM_ROLES_CASE(8)
#undef DMLC_STEM_ROLES_CASE
    }
  } else if (u8) {
    // query batches: split the 64 channels over 2 or 4 workgroups when the
    // strips alone leave most CUs idle (B = 1: 28 strips -> 112 workgroups)
    const long wgs = (long)B * (PH / strip);
    const int cs = wgs * 4 <= kStemSplitCus ? 4 : wgs * 2 <= kStemSplitCus ? 2 : 1;
    const dim3 gs(grid.x, cs);
    switch (NF * 4 + (cs == 4 ? 2 : cs == 2 ? 1 : 0)) {
      case 7 * 4 + 1: hipLaunchKernelGGL((stem_conv_pool_kernel<7, true, 2>), gs, dim3(256), lds, s, a); break;
      case 7 * 4 + 2: hipLaunchKernelGGL((stem_conv_pool_kernel<7, true, 4>), gs, dim3(256), lds, s, a); break;
      default: break;
    }
    if (NF == 7 && cs > 1) {
      DMLC_HIP_CHECK(hipGetLastError());
      return;
    }
    switch (NF) {
#define DMLC_STEM_U8_CASE(F) \
  case F: hipLaunchKernelGGL((stem_conv_pool_kernel<F, true>), grid, dim3(256), lds, s, a); break;
      DMLC_STEM_U8_CASE(4)
      DMLC_STEM_U8_CASE(5)
      DMLC_STEM_U8_CASE(6)
      DMLC_STEM_U8_CASE(7)
      DMLC_STEM_U8_CASE(8)
#undef DMLC_STEM_U8_CASE
    }
  } else {
    switch (NF) {
#define DMLC_STEM_CASE(F) \
  case F: hipLaunchKernelGGL((stem_conv_pool_kernel<F, false>), grid, dim3(256), lds, s, a); break;
      DMLC_STEM_CASE(4)
      DMLC_STEM_CASE(5)
      DMLC_STEM_CASE(6)
      DMLC_STEM_CASE(7)
      DMLC_STEM_CASE(8)
#undef DMLC_STEM_CASE
    }
  }
  DMLC_HIP_CHECK(hipGetLastError());
}
}  // namespace

void stem_conv_pool_set_dbg(int dbg) { g_stem_dbg = dbg; }
void stem_conv_pool_set_stamps(void* p) { g_stem_stamps = (unsigned long long*)p; }

void stem_conv_pool(const void* x, const void* w, const float* bias, void* y, int B, int S, int Wq, int strip,
                    hipStream_t s) {
  if (!x) throw std::invalid_argument("stem_conv_pool: null input");
  stem_launch(x, nullptr, w, nullptr, bias, y, B, S, Wq, strip, s);
}

void stem_conv_pool_u8(const uint8_t* x, const void* w, const float* bias, void* y, int B, int S, int strip,
                       hipStream_t s, const void* w_dense) {
  if (!x) throw std::invalid_argument("stem_conv_pool_u8: null input");
  stem_launch(nullptr, x, w, w_dense, bias, y, B, S, stem_row_width(S, 3, 7, 2) / 2, strip, s);
}

}  // namespace dmlc
