// Big-tile implicit-GEMM convolution: 8-wave 256x256 / 256x128 tiles with an
// XCD-local, K-lockstep split-K schedule (bf16 MFMA).
//
// Same GEMM view and operand layouts as conv_igemm.hip (M = B*Ho*Wo output
// pixels, N = Cout, K = KH*KW*Cin with NHWC activations; weights [Npad, Kpad];
// folded-BN bias + residual + ReLU epilogue), built for the ResNet layers
// whose GEMMs are too small to fill 256 CUs with big tiles (the conv hot path
// of `forward_t`, reference src/services.rs:493):
//
//  * 512-thread workgroups = 8 waves (2 per SIMD), one per CU (128 KB LDS at
//    256x256): 2x the FLOP per staged byte of a 128x128 tile.
//  * Schedule. Tiles are dealt to the 8 XCDs in contiguous ranges (n-fastest
//    tile order, so an XCD's tiles share activation and weight panels in its
//    own L2); each tile's K range is cut into `splits` equal slices and every
//    (slice, tile) unit is one workgroup. All units of an XCD start together
//    and walk K in lockstep, so the XCD's L2 working set is a few K-tiles of
//    panels. (A stream-K order -- equal contiguous ranges of the flattened
//    (tile, K) space -- puts concurrent workgroups at 30 different K offsets:
//    the whole weight matrix becomes live, L2 thrashes and the conv runs at
//    the Infinity-Cache rate, measured 2x slower: profiles/r1_bigtile_conv.log.)
//  * Split-K hand-off: slices s >= 1 store their fp32 partial tile to a slab
//    and raise a flag; slice 0 (the "head") waits for them, adds the slabs in
//    slice order (deterministic) and runs the epilogue. Within an XCD the
//    contributors come first in dispatch order, so a head only ever waits
//    for a workgroup dispatched before it; spins are bounded and a timeout is
//    reported through `err` instead of hanging the GPU.
//  * Hand-off memory protocol (cdna_hip_programming.md Guideline 16, sc1
//    form): write-through sc1 dwordx4 slab stores -> every wave vmcnt(0) ->
//    barrier -> one lane stores the flag (relaxed agent atomic = sc1);
//    consumer: one lane polls relaxed, barrier, sc1 dwordx4 loads. No
//    release/acquire fences (an agent release writes back the whole XCD L2).
//    The consumer resets the flag (each flag has exactly one consumer).
//  * Staging is the LDS-DMA ring of conv_igemm.hip (global_load_lds_dwordx4,
//    zero page for padding taps, XOR-swizzled 128-B rows, swizzle applied on
//    the per-lane source address); the DMA of K-tile t+1 is issued before
//    the MFMAs of K-tile t.
#include "common.h"
#include "kernels.h"

#include <algorithm>
#include <cmath>
#include <cstdlib>

namespace dmlc {

namespace {

typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef const __attribute__((address_space(1))) void* gbl_ptr_t;
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

// 64-B LDS rows (4 chunks of 16 B): physical chunk = chunk ^ (3 * bit 2 of
// the row). With the ds_read_b128 lane groups {0-3,12-15,20-27},
// {4-11,16-19,28-31}, ... (MI355X_MICROARCH.md §LDS) a fragment read (lane
// reads chunk lane>>4 of row base+(lane&15), base % 16 == 0) puts each group
// on 16 distinct 16-B bank slots: conflict-free.
__device__ __forceinline__ int bt_swz(int row, int chunk) { return chunk ^ (3 * ((row >> 2) & 1)); }

// s_waitcnt vmcnt(N) with a compile-time N.
template <int N>
__device__ __forceinline__ void vm_wait() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}

// Buffer descriptor from provably wave-uniform inputs (else hipcc wraps every
// buffer op in a waterfall loop: cdna_hip_programming.md T20).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t bt_rsrc(const float* p, int bytes) {
  const uint64_t u = (uint64_t)p;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)u);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(u >> 32));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), (short)0,
                                           __builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}

constexpr unsigned kSpinLimit = 1u << 21;  // x (poll + s_sleep) ~ 1-2 s: a hang becomes an error
constexpr int kMaxFlags = 4096;
constexpr size_t kHeader = kMaxFlags * sizeof(unsigned) + 256;  // flags, err word, padding
constexpr int kSlabFloats = 256 * 256;

// Units of XCD x: tiles [T*x/8, T*(x+1)/8) x `splits` K slices; local order
// = slices S-1 .. 1 (contributors) first, then the heads (slice 0).
__device__ __forceinline__ bool bt_unit(int bid, int tiles, int splits, int& tile, int& slice) {
  const int x = bid & 7, local = bid >> 3;
  const int t_lo = (int)((long)tiles * x / 8), t_hi = (int)((long)tiles * (x + 1) / 8);
  const int nt = t_hi - t_lo;
  if (nt <= 0 || local >= nt * splits) return false;
  slice = splits - 1 - local / nt;
  tile = t_lo + local % nt;
  return true;
}

// Wait until this wave's DMA of the current sub-tile landed, leaving the
// min(D-1, y) younger sub-tiles (G instructions each) in flight.
template <int D, int G>
__device__ __forceinline__ void wait_younger(int y) {
  if (y >= D - 1) {
    vm_wait<(D - 1) * G>();
    return;
  }
  if constexpr (D >= 4)
    if (y == 2) {
      vm_wait<2 * G>();
      return;
    }
  if constexpr (D >= 3)
    if (y == 1) {
      vm_wait<G>();
      return;
    }
  vm_wait<0>();
}

template <int BM, int BN, int WM, int WN, int NS>
__global__ __launch_bounds__(512, 1) void conv_bt_kernel(ConvArgs a, int k_tiles, int tiles, int splits,
                                                         float* __restrict__ slabs, unsigned* __restrict__ flags,
                                                         unsigned* __restrict__ err) {
  constexpr int BK = 32;    // bf16 per pipeline sub-tile (one 64-B LDS row)
  constexpr int ROWB = 64;
  constexpr int PA = BM / 128, PB = BN / 128;  // rows staged per lane (8 waves x 16 rows per DMA instruction)
  constexpr int G = PA + PB;                   // LDS-DMA instructions per lane per sub-tile
  constexpr int D = NS - 1;                    // prefetch distance (sub-tiles in flight)
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int TM = WTM / 16, TN = WTN / 16;
  constexpr int STAGE_B = (BM + BN) * ROWB;
  constexpr int A_CH = BM * 4;  // uint4 chunks
  constexpr int STAGE_CH = (BM + BN) * 4;
  static_assert(WM * WN == 8, "8 waves per block");
  static_assert(BM % 128 == 0 && BN % 128 == 0 && TM >= 1 && TN >= 1 && BM * BN <= kSlabFloats, "tile");
  static_assert(NS >= 2 && NS <= 6 && D * G < 64, "stages");

  extern __shared__ __attribute__((aligned(16))) uint4 smem[];

  int tile, slice;
  if (!bt_unit(blockIdx.x, tiles, splits, tile, slice)) return;
  tile = __builtin_amdgcn_readfirstlane(tile);  // provably uniform: scalar buffer descriptors, no waterfall loops
  slice = __builtin_amdgcn_readfirstlane(slice);

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave % WM, wn = wave / WM;
  const int fr = lane & 15, fq = lane >> 4;

  const int M = a.B * a.Ho * a.Wo;
  const int n_tiles = a.Npad / BN;
  const int m0 = (tile / n_tiles) * BM, n0 = (tile % n_tiles) * BN;
  // this slice's sub-tiles (slices are cut on 64-deep K-tile boundaries)
  const int k0 = 2 * (k_tiles * slice / splits), k1 = 2 * (k_tiles * (slice + 1) / splits);

  const bf16* __restrict__ x = (const bf16*)a.x;
  const bf16* __restrict__ w = (const bf16*)a.w;
  const bf16* zero = (const bf16*)a.zero;

  // Rows this lane stages: rows p*128 + wave*16 + lane/4 (p < PA), B likewise;
  // the lane writes physical chunk lane&3 of its row (LDS-DMA is lane-linear),
  // so it loads logical chunk bt_swz(row, lane&3) (an involution).
  const int lrow = lane >> 2;
  const int pchunk = lane & 3;
  int hi0[PA], wi0[PA], abase[PA];
  int wboff[PB];
#pragma unroll
  for (int p = 0; p < PA; ++p) {
    const int r = p * 128 + wave * 16 + lrow;
    const int m = m0 + r;
    if (m < M) {
      const int hw = a.Ho * a.Wo;
      const int b = m / hw;
      const int rem = m - b * hw;
      const int ho = rem / a.Wo;
      const int wo = rem - ho * a.Wo;
      hi0[p] = ho * a.stride - a.pad;
      wi0[p] = wo * a.stride - a.pad;
      abase[p] = ((b * a.H + hi0[p]) * a.W + wi0[p]) * a.Cin + bt_swz(r, pchunk) * 8;
    } else {
      hi0[p] = -(1 << 28);
      wi0[p] = 0;
      abase[p] = 0;
    }
  }
#pragma unroll
  for (int p = 0; p < PB; ++p) {
    const int r = p * 128 + wave * 16 + lrow;
    wboff[p] = (n0 + r) * a.Kpad + bt_swz(r, pchunk) * 8;
  }

  // Issue the LDS-DMA of sub-tile t (k = 32t .. 32t+31) into stage `st`.
  const int ctiles = a.Cin / BK;
  auto stage = [&](int t, int st) __attribute__((always_inline)) {
    char* sbase = (char*)smem + st * STAGE_B;
    const int tap = t / ctiles;
    const int c0 = (t - tap * ctiles) * BK;
    const int kh = tap / a.KW;
    const int kw = tap - kh * a.KW;
    const int off = (kh * a.W + kw) * a.Cin + c0;
#pragma unroll
    for (int p = 0; p < PA; ++p) {
      const bool ok = (unsigned)(hi0[p] + kh) < (unsigned)a.H && (unsigned)(wi0[p] + kw) < (unsigned)a.W;
      const bf16* src = ok ? x + abase[p] + off : zero;
      __builtin_amdgcn_global_load_lds((gbl_ptr_t)src, (lds_ptr_t)(sbase + (p * 128 + wave * 16) * ROWB), 16, 0, 0);
    }
    const bf16* wt = w + t * BK;
#pragma unroll
    for (int p = 0; p < PB; ++p)
      __builtin_amdgcn_global_load_lds((gbl_ptr_t)(wt + wboff[p]),
                                       (lds_ptr_t)(sbase + (BM + p * 128 + wave * 16) * ROWB), 16, 0, 0);
  };

  floatx4 acc[TN][TM];
#pragma unroll
  for (int i = 0; i < TN; ++i)
#pragma unroll
    for (int j = 0; j < TM; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

  // Fragment addresses (uint4 units): lane (fr, fq) reads chunk fq of row
  // base+fr; fragment rows start at multiples of 16, so the swizzle term
  // (row>>2)&1 = (fr>>2)&1 is the same for every i/j, which become immediate
  // offsets (16 rows = 64 chunks).
  const int aoff = A_CH + (wn * WTN + fr) * 4 + bt_swz(fr, fq);
  const int boff = (wm * WTM + fr) * 4 + bt_swz(fr, fq);
  auto compute = [&](int st) __attribute__((always_inline)) {
    const uint4* sb = smem + st * STAGE_CH;
    bf16x8 af[TN], bm[TM];
#pragma unroll
    for (int i = 0; i < TN; ++i) af[i] = __builtin_bit_cast(bf16x8, sb[aoff + i * 64]);
#pragma unroll
    for (int j = 0; j < TM; ++j) bm[j] = __builtin_bit_cast(bf16x8, sb[boff + j * 64]);
#pragma unroll
    for (int i = 0; i < TN; ++i)
#pragma unroll
      for (int j = 0; j < TM; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bm[j], acc[i][j], 0, 0, 0);
  };

  // Main loop: NS-stage LDS ring, D = NS-1 sub-tiles in flight. Iteration t:
  // counted wait until this wave's DMA of sub-tile t landed (the younger
  // ones stay in flight), raw barrier (no vmcnt(0) drain: every wave's part
  // of t is visible and every wave finished reading t-1), then the fragment
  // reads of t and its MFMAs, with the G LDS-DMA instructions that refill
  // t-1's stage with t+D spread one per MFMA group: issued in a burst after
  // the barrier they stall every wave at issue and the DMA and the MFMAs
  // serialise (measured: loop = DMA-only + MFMA-only time). Past the end of
  // the slice the refill reads the zero page (harmless: that stage is never
  // read again), so every iteration issues exactly G and the wait count is
  // constant; the epilogue's __syncthreads drains them before LDS is reused.
  static_assert(G <= TN, "at most one DMA per MFMA row group");
  auto issue_one = [&](int g, char* sbase, int off, int kh, int kw, bool valid, const bf16* wt)
      __attribute__((always_inline)) {
    if (g < PA) {
      const bool ok = valid && (unsigned)(hi0[g] + kh) < (unsigned)a.H && (unsigned)(wi0[g] + kw) < (unsigned)a.W;
      const bf16* src = ok ? x + abase[g] + off : zero;
      __builtin_amdgcn_global_load_lds((gbl_ptr_t)src, (lds_ptr_t)(sbase + (g * 128 + wave * 16) * ROWB), 16, 0, 0);
    } else {
      const int p = g - PA;
      const bf16* src = valid ? wt + wboff[p] : zero;
      __builtin_amdgcn_global_load_lds((gbl_ptr_t)src, (lds_ptr_t)(sbase + (BM + p * 128 + wave * 16) * ROWB), 16,
                                       0, 0);
    }
  };
#pragma unroll
  for (int s2 = 0; s2 < D; ++s2) {
    const int tn = k0 + s2;
    const bool valid = tn < k1;
    const int tap = tn / ctiles, c0 = (tn - tap * ctiles) * BK, kh = tap / a.KW, kw = tap - kh * a.KW;
    char* sbase = (char*)smem + s2 * STAGE_B;
#pragma unroll
    for (int g = 0; g < G; ++g) issue_one(g, sbase, (kh * a.W + kw) * a.Cin + c0, kh, kw, valid, w + tn * BK);
  }
  int st = 0;
  for (int t = k0; t < k1; ++t) {
    vm_wait<(D - 1) * G>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    const int tn = t + D;
    const bool valid = tn < k1;
    const int tap = tn / ctiles, c0 = (tn - tap * ctiles) * BK, kh = tap / a.KW, kw = tap - kh * a.KW;
    const int off = (kh * a.W + kw) * a.Cin + c0;
    char* rbase = (char*)smem + (st == 0 ? NS - 1 : st - 1) * STAGE_B;
    const bf16* wt = w + tn * BK;
    const uint4* sb = smem + st * STAGE_CH;
    bf16x8 af[TN], bm[TM];
#pragma unroll
    for (int i = 0; i < TN; ++i) af[i] = __builtin_bit_cast(bf16x8, sb[aoff + i * 64]);
#pragma unroll
    for (int j = 0; j < TM; ++j) bm[j] = __builtin_bit_cast(bf16x8, sb[boff + j * 64]);
#pragma unroll
    for (int i = 0; i < TN; ++i) {
      if (i < G) issue_one(i, rbase, off, kh, kw, valid, wt);
#pragma unroll
      for (int j = 0; j < TM; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bm[j], acc[i][j], 0, 0, 0);
    }
    // pin the order: fragment reads, then (1 DMA, TM MFMAs) x TN
    __builtin_amdgcn_sched_group_barrier(0x100, TN + TM, 0);
#pragma unroll
    for (int i = 0; i < TN; ++i) {
      if (i < G) __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, TM, 0);
    }
    st = st == NS - 1 ? 0 : st + 1;
  }

  const int nslot = splits - 1;
  if (slice == 0 && splits > 1 && tid == 0) {
    for (int s2 = 1; s2 < splits; ++s2) {
      unsigned* f = flags + tile * nslot + s2 - 1;
      unsigned spins = 0;
      while (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u) {
        __builtin_amdgcn_s_sleep(2);
        if (++spins > kSpinLimit) {
          __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
      }
      __hip_atomic_store(f, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }

  // Epilogue through LDS (cdna_hip_programming.md T21): each wave stages 64
  // rows x 64 cols of fp32 in its own 16 KB of the now idle LDS (16-B chunks
  // XOR-swizzled by row: conflict-free b128 writes and reads); then every
  // lane owns 8 consecutive channels of one row: a wave instruction covers 8
  // rows x 64 channels, so slab traffic is 256 contiguous bytes per row and
  // the bf16 output 128. Heads add the slabs (slice order: deterministic),
  // bias and residual, apply ReLU and store 16 B; contributors store fp32
  // (sc1, write-through) and raise their flag.
  static_assert(WTN == 64 && WTM % 64 == 0, "epilogue staging assumes 64-column wave tiles");
  __syncthreads();  // every wave is done reading the operand stages (and the head's flags matched)
  float* wl = (float*)smem + wave * (64 * 64);
  const bf16* __restrict__ res = (const bf16*)a.res;
  const int q = lane & 7, rr = lane >> 3;
  const int cq = wn * WTN + q * 8;  // tile column of this lane's 8 channels
  const int nq = n0 + cq;
  const __amdgpu_buffer_rsrc_t slab_rs =
      bt_rsrc(slabs + (size_t)(tile * nslot + (slice > 0 ? slice - 1 : 0)) * kSlabFloats,
              splits > 1 ? (slice > 0 ? BM * BN * 4 : nslot * kSlabFloats * 4) : 0);
  floatx4 bq0 = {0.f, 0.f, 0.f, 0.f}, bq1 = bq0;
  if (slice == 0 && a.bias && nq < a.N) {
    bq0 = *(const floatx4*)(a.bias + nq);
    bq1 = *(const floatx4*)(a.bias + nq + 4);
  }
#pragma unroll
  for (int h = 0; h < WTM / 64; ++h) {
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      const int row = jj * 16 + fr;
#pragma unroll
      for (int i = 0; i < TN; ++i) {
        const int chunk = (i * 4 + fq) ^ (row & 15);
        *(floatx4*)(wl + row * 64 + chunk * 4) = acc[i][h * 4 + jj];
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int g = 0; g < 8; ++g) {
      const int row = g * 8 + rr;
      floatx4 lo = *(const floatx4*)(wl + row * 64 + ((2 * q) ^ (row & 15)) * 4);
      floatx4 hi = *(const floatx4*)(wl + row * 64 + ((2 * q + 1) ^ (row & 15)) * 4);
      const int rt = wm * WTM + h * 64 + row;  // tile row
      const int soff = (rt * BN + cq) * 4;      // slab byte offset
      if (slice > 0) {
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, lo), slab_rs, soff, 0, 16 /* sc1 */);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, hi), slab_rs, soff + 16, 0, 16);
        continue;
      }
      for (int s2 = 1; s2 < splits; ++s2) {
        const int o2 = soff + (s2 - 1) * kSlabFloats * 4;
        lo += __builtin_bit_cast(floatx4, __builtin_amdgcn_raw_buffer_load_b128(slab_rs, o2, 0, 16 /* sc1 */));
        hi += __builtin_bit_cast(floatx4, __builtin_amdgcn_raw_buffer_load_b128(slab_rs, o2 + 16, 0, 16));
      }
      const int m = m0 + rt;
      if (m >= M || nq >= a.N) continue;
      float v[8] = {lo[0] + bq0[0], lo[1] + bq0[1], lo[2] + bq0[2], lo[3] + bq0[3],
                    hi[0] + bq1[0], hi[1] + bq1[1], hi[2] + bq1[2], hi[3] + bq1[3]};
      const size_t o = (size_t)m * a.ldo + nq;
      if (res) {
        float r[8];
        unpack8(*(const uint4*)(res + o), r);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += r[e];
      }
      const uint4 pv = pack8_relu(v, a.relu);
      *(uint4*)((bf16*)a.y + o) = pv;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // reads done before the next half overwrites
  }
  if (slice > 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains before the signal
    __syncthreads();
    if (tid == 0) __hip_atomic_store(flags + tile * nslot + slice - 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// Persistent variant for narrow-N convs with many tiles (ResNet layer2: N =
// 128, 784 tiles of 256x128 at batch 256): workgroup b walks tiles
// [T*b/G, T*(b+1)/G) (neighbouring tiles share input halo rows in L2/L1).
// BK = 64 (full 128-B lines per row) in an NS-stage ring that streams across
// tile boundaries, so the next tile's first K-tiles load during this tile's
// last MFMAs and its epilogue. The epilogue stages 16 rows x 64 cols of fp32
// per wave and pass through the stage just consumed (the other stages hold
// the next tile's prefetch), 4 passes for a 64-row wave tile.
__device__ __forceinline__ int bp_swz(int row, int chunk) { return chunk ^ ((row >> 1) & 7); }

template <int BM, int BN, int WM, int WN, int NS>
__global__ __launch_bounds__(512, 1) void conv_btp_kernel(ConvArgs a, int k_tiles, int tiles) {
  constexpr int BK = 64, ROWB = 128;
  constexpr int PA = BM / 64, PB = BN / 64;  // rows staged per lane (8 waves x 8 rows per DMA instruction)
  constexpr int G = PA + PB;
  constexpr int D = NS - 1;
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int TM = WTM / 16, TN = WTN / 16;
  constexpr int STAGE_B = (BM + BN) * ROWB;
  constexpr int A_CH = BM * 8;
  constexpr int STAGE_CH = (BM + BN) * 8;
  static_assert(WM * WN == 8 && WTN == 64 && TM >= 1 && D * G < 64, "config");
  static_assert(STAGE_B >= 8 * 16 * 64 * 4, "epilogue pass staging must fit in one stage");

  extern __shared__ __attribute__((aligned(16))) uint4 smem[];

  const int G_ = gridDim.x;
  const int b = blockIdx.x;
  const int t_lo = (int)((long)tiles * b / G_), t_hi = (int)((long)tiles * (b + 1) / G_);
  if (t_lo >= t_hi) return;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave % WM, wn = wave / WM;
  const int fr = lane & 15, fq = lane >> 4;
  const int M = a.B * a.Ho * a.Wo;
  const int n_tiles = a.Npad / BN;

  const bf16* __restrict__ x = (const bf16*)a.x;
  const bf16* __restrict__ w = (const bf16*)a.w;
  const bf16* zero = (const bf16*)a.zero;

  const int lrow = lane >> 3;
  const int pchunk = lane & 7;
  int hi0[PA], wi0[PA], abase[PA];
  int wboff[PB];
  auto setup_rows = [&](int tile) __attribute__((always_inline)) {
    const int m0_ = (tile / n_tiles) * BM, n0_ = (tile % n_tiles) * BN;
#pragma unroll
    for (int p = 0; p < PA; ++p) {
      const int r = p * 64 + wave * 8 + lrow;
      const int m = m0_ + r;
      if (m < M) {
        const int hw = a.Ho * a.Wo;
        const int bb = m / hw;
        const int rem = m - bb * hw;
        const int ho = rem / a.Wo;
        const int wo = rem - ho * a.Wo;
        hi0[p] = ho * a.stride - a.pad;
        wi0[p] = wo * a.stride - a.pad;
        abase[p] = ((bb * a.H + hi0[p]) * a.W + wi0[p]) * a.Cin + bp_swz(r, pchunk) * 8;
      } else {
        hi0[p] = -(1 << 28);
        wi0[p] = 0;
        abase[p] = 0;
      }
    }
#pragma unroll
    for (int p = 0; p < PB; ++p) {
      const int r = p * 64 + wave * 8 + lrow;
      wboff[p] = (n0_ + r) * a.Kpad + bp_swz(r, pchunk) * 8;
    }
  };

  const int ctiles = a.Cin / BK;
  auto stage = [&](int t, int st) __attribute__((always_inline)) {
    char* sbase = (char*)smem + st * STAGE_B;
    const int tap = t / ctiles;
    const int c0 = (t - tap * ctiles) * BK;
    const int kh = tap / a.KW;
    const int kw = tap - kh * a.KW;
    const int off = (kh * a.W + kw) * a.Cin + c0;
#pragma unroll
    for (int p = 0; p < PA; ++p) {
      const bool ok = (unsigned)(hi0[p] + kh) < (unsigned)a.H && (unsigned)(wi0[p] + kw) < (unsigned)a.W;
      const bf16* src = ok ? x + abase[p] + off : zero;
      __builtin_amdgcn_global_load_lds((gbl_ptr_t)src, (lds_ptr_t)(sbase + (p * 64 + wave * 8) * ROWB), 16, 0, 0);
    }
    const bf16* wt = w + t * BK;
#pragma unroll
    for (int p = 0; p < PB; ++p)
      __builtin_amdgcn_global_load_lds((gbl_ptr_t)(wt + wboff[p]),
                                       (lds_ptr_t)(sbase + (BM + p * 64 + wave * 8) * ROWB), 16, 0, 0);
  };

  floatx4 acc[TN][TM];
  const int sw = (fr >> 1) & 7;
  int aoff[2], boff[2];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) {
    aoff[ks] = A_CH + (wn * WTN + fr) * 8 + ((ks * 4 + fq) ^ sw);
    boff[ks] = (wm * WTM + fr) * 8 + ((ks * 4 + fq) ^ sw);
  }
  auto compute = [&](int st) __attribute__((always_inline)) {
    const uint4* sb = smem + st * STAGE_CH;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 af[TN], bm[TM];
#pragma unroll
      for (int i = 0; i < TN; ++i) af[i] = __builtin_bit_cast(bf16x8, sb[aoff[ks] + i * 128]);
#pragma unroll
      for (int j = 0; j < TM; ++j) bm[j] = __builtin_bit_cast(bf16x8, sb[boff[ks] + j * 128]);
#pragma unroll
      for (int i = 0; i < TN; ++i)
#pragma unroll
        for (int j = 0; j < TM; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bm[j], acc[i][j], 0, 0, 0);
    }
  };

  // Flattened (tile, K-tile) stream of this workgroup: item i = (t_lo + i / k_tiles, i % k_tiles).
  const int items = (t_hi - t_lo) * k_tiles;
  int issue_tile = t_lo;  // tile whose row state is loaded
  setup_rows(issue_tile);
  auto issue = [&](int i, int st) __attribute__((always_inline)) {
    const int tt = t_lo + i / k_tiles;
    if (tt != issue_tile) {  // every DMA of the previous tile is issued: its row state can go
      issue_tile = tt;
      setup_rows(tt);
    }
    stage(i - (tt - t_lo) * k_tiles, st);
  };
#pragma unroll
  for (int s2 = 0; s2 < D; ++s2)
    if (s2 < items) issue(s2, s2);

  const bf16* __restrict__ res = (const bf16*)a.res;
  const int q = lane & 7, rr = lane >> 3;
  int st = 0;
  for (int tile = t_lo; tile < t_hi; ++tile) {
#pragma unroll
    for (int i = 0; i < TN; ++i)
#pragma unroll
      for (int j = 0; j < TM; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
    const int base = (tile - t_lo) * k_tiles;
    for (int kk = 0; kk < k_tiles; ++kk) {
      const int i = base + kk;
      wait_younger<D, G>(items - 1 - i);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      if (i + D < items) issue(i + D, st == 0 ? NS - 1 : st - 1);
      compute(st);
      st = st == NS - 1 ? 0 : st + 1;
    }
    // Epilogue through the stage just consumed (the previous value of st):
    // after this barrier no wave reads it, and it is refilled only after the
    // next K-loop barrier, which every wave reaches after its epilogue reads.
    const int est = st == 0 ? NS - 1 : st - 1;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    float* wl = (float*)((char*)smem + est * STAGE_B) + wave * (16 * 64);
    const int m0 = (tile / n_tiles) * BM, n0 = (tile % n_tiles) * BN;
    const int nq = n0 + wn * WTN + q * 8;
    floatx4 bq0 = {0.f, 0.f, 0.f, 0.f}, bq1 = bq0;
    if (a.bias && nq < a.N) {
      bq0 = *(const floatx4*)(a.bias + nq);
      bq1 = *(const floatx4*)(a.bias + nq + 4);
    }
#pragma unroll
    for (int j = 0; j < TM; ++j) {  // pass j: rows j*16 .. j*16+15 of the wave tile
#pragma unroll
      for (int i = 0; i < TN; ++i) *(floatx4*)(wl + fr * 64 + (((i * 4 + fq) ^ fr) * 4)) = acc[i][j];
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int g = 0; g < 2; ++g) {
        const int row = g * 8 + rr;
        const floatx4 lo = *(const floatx4*)(wl + row * 64 + (((2 * q) ^ row) * 4));
        const floatx4 hi = *(const floatx4*)(wl + row * 64 + (((2 * q + 1) ^ row) * 4));
        const int m = m0 + wm * WTM + j * 16 + row;
        if (m >= M || nq >= a.N) continue;
        float v[8] = {lo[0] + bq0[0], lo[1] + bq0[1], lo[2] + bq0[2], lo[3] + bq0[3],
                      hi[0] + bq1[0], hi[1] + bq1[1], hi[2] + bq1[2], hi[3] + bq1[3]};
        const size_t o = (size_t)m * a.ldo + nq;
        if (res) {
          float r[8];
          unpack8(*(const uint4*)(res + o), r);
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] += r[e];
        }
        *(uint4*)((bf16*)a.y + o) = pack8_relu(v, a.relu);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // reads done before the next pass overwrites
    }
  }
}

struct BtCfg {
  int bm, bn, ns;
};
constexpr BtCfg kBtCfgs[2] = {{256, 256, 4}, {256, 128, 5}};

long bt_tiles(const ConvArgs& a, int cfg) {
  const BtCfg c = kBtCfgs[cfg];
  const long M = (long)a.B * a.Ho * a.Wo;
  return ((M + c.bm - 1) / c.bm) * (a.Npad / c.bn);
}

}  // namespace

int conv_bigtile_pick(const ConvArgs& a, int num_cus) {
  if (a.stem || a.in_fp8 || a.out_fp8 || a.out_f32) return -1;
  if (a.Cin % 64 != 0 || a.Kpad / 64 < 16 || a.N % 8 != 0 || a.ldo % 8 != 0) return -1;
  // 256x256 tiles only when they fill the CUs in one round without a K
  // split (ResNet18 layer3 at batch 256: 196 tiles, 69-71 vs 88-92 us per
  // conv). With 2 K slices (layer4.x.conv2: 98 tiles x 2) the split-K
  // hand-off costs more than it saves in the model (107 vs 94 us with the
  // residual epilogue), and the 256x128 configs (narrow N: 85 FLOP per
  // staged byte) measured slower than conv_igemm's 2-workgroup-per-CU tiles
  // (profiles/r1_bigtile_conv.log).
  if (a.Npad % 256 != 0) return -1;
  const long tiles = bt_tiles(a, 0);
  if (tiles <= num_cus && tiles * 4 >= num_cus * 3) return 0;
  return -1;
}

int conv_bigtile_splits(const ConvArgs& a, int cfg, int num_cus) {
  // Per XCD: ceil(S * tiles/8 / (CUs/8)) rounds of K/S K-tiles each, plus a
  // hand-off cost of ~4 K-tiles when S > 1; slices of at least 8 K-tiles.
  const long tiles = bt_tiles(a, cfg);
  const int kt = a.Kpad / 64;
  const double per_xcd = tiles / 8.0, cus = std::max(1, num_cus / 8);
  int best = 1;
  double best_t = 1e30;
  for (int s = 1; s <= 4; ++s) {
    if (s > 1 && (kt / s < 8 || tiles * (s - 1) > kMaxFlags)) break;
    const double t = std::ceil(std::ceil(per_xcd) * s / cus) * ((double)kt / s) + (s > 1 ? 4.0 : 0.0);
    if (t < best_t - 1e-9) {
      best_t = t;
      best = s;
    }
  }
  return best;
}

size_t conv_bigtile_ws_bytes(long max_slabs) { return kHeader + (size_t)max_slabs * kSlabFloats * sizeof(float); }
size_t conv_bigtile_ws_header_bytes() { return kHeader; }
long conv_bigtile_slabs(const ConvArgs& a, int cfg, int splits) { return bt_tiles(a, cfg) * (splits - 1); }

void conv2d_bigtile(const ConvArgs& a, int cfg, int splits, void* ws, size_t ws_bytes, hipStream_t s) {
  if (cfg < 0 || cfg > 1) throw std::invalid_argument("conv2d_bigtile: bad config");
  if (a.stem || a.in_fp8 || a.out_fp8 || a.out_f32) throw std::invalid_argument("conv2d_bigtile: bf16 convs only");
  if (a.Cin % 64 != 0) throw std::invalid_argument("conv2d_bigtile: Cin must be a multiple of 64");
  if (a.Kpad != conv_kpad(a.Cin, a.KH, a.KW, false)) throw std::invalid_argument("conv2d_bigtile: bad Kpad");
  if (a.N % 8 != 0 || a.N > a.Npad || a.ldo < a.N || a.ldo % 8 != 0)
    throw std::invalid_argument("conv2d_bigtile: bad N/ldo (multiples of 8: 16-B output rows)");
  if (a.Ho != conv_out_dim(a.H, a.KH, a.stride, a.pad) || a.Wo != conv_out_dim(a.W, a.KW, a.stride, a.pad))
    throw std::invalid_argument("conv2d_bigtile: bad output dims");
  if (!a.x || !a.w || !a.y || !a.zero) throw std::invalid_argument("conv2d_bigtile: null operand");
  if (((uintptr_t)a.x | (uintptr_t)a.w | (uintptr_t)a.zero | (uintptr_t)ws | (uintptr_t)a.y | (uintptr_t)a.res |
       (uintptr_t)a.bias) & 15)
    throw std::invalid_argument("conv2d_bigtile: operands must be 16-B aligned");
  const BtCfg c = kBtCfgs[cfg];
  if (a.Npad % c.bn != 0) throw std::invalid_argument("conv2d_bigtile: Npad not a multiple of BN");
  const long M = (long)a.B * a.Ho * a.Wo;
  if (M <= 0) return;
  if ((long)a.B * a.H * a.W * a.Cin >= (1L << 31) || M * a.ldo >= (1L << 31) || (long)a.Npad * a.Kpad >= (1L << 31))
    throw std::invalid_argument("conv2d_bigtile: tensor too large for 32-bit offsets");
  const int k_tiles = a.Kpad / 64;
  const long tiles = bt_tiles(a, cfg);
  if (splits < 1 || splits > k_tiles) throw std::invalid_argument("conv2d_bigtile: bad split count");
  if (splits > 1) {
    if (!ws) throw std::invalid_argument("conv2d_bigtile: split-K needs a workspace");
    if (tiles * (splits - 1) > kMaxFlags) throw std::invalid_argument("conv2d_bigtile: too many hand-off flags");
    if (conv_bigtile_ws_bytes(tiles * (splits - 1)) > ws_bytes)
      throw std::invalid_argument("conv2d_bigtile: workspace too small");
  }
  // grid: 8 XCD groups x the largest group's unit count (bt_unit)
  const long per_xcd = (tiles + 7) / 8 * splits;
  const long grid = 8 * per_xcd;
  if (grid >= (1L << 31)) throw std::invalid_argument("conv2d_bigtile: grid too large");
  unsigned* flags = (unsigned*)ws;
  unsigned* err = flags ? flags + kMaxFlags : nullptr;
  float* slabs = ws ? (float*)((char*)ws + kHeader) : nullptr;
  // operand stages (64-B rows), or the epilogue's 8 x 16 KB fp32 staging if larger
  const size_t lds = std::max((size_t)c.ns * (c.bm + c.bn) * 64, (size_t)8 * 64 * 64 * 4);
  const dim3 g((unsigned)grid), b(512);
  if (cfg == 0)
    hipLaunchKernelGGL((conv_bt_kernel<256, 256, 2, 4, 4>), g, b, lds, s, a, k_tiles, (int)tiles, splits, slabs,
                       flags, err);
  else
    hipLaunchKernelGGL((conv_bt_kernel<256, 128, 4, 2, 5>), g, b, lds, s, a, k_tiles, (int)tiles, splits, slabs,
                       flags, err);
  DMLC_HIP_CHECK(hipGetLastError());
}


// Persistent big-tile conv (conv_btp_kernel): 256x128 tiles, BK=64, 3 stages.
bool conv_bigtile_persistent_ok(const ConvArgs& a) {
  return !(a.stem || a.in_fp8 || a.out_fp8 || a.out_f32) && a.Cin % 64 == 0 && a.Npad % 128 == 0 &&
         a.N % 8 == 0 && a.ldo % 8 == 0;
}

int conv_bigtile_persistent_grid(const ConvArgs& a, int num_cus) {
  // equal tile counts per workgroup: G = tiles / ceil(tiles / CUs)
  const long M = (long)a.B * a.Ho * a.Wo;
  const long tiles = ((M + 255) / 256) * (a.Npad / 128);
  const long per = (tiles + num_cus - 1) / num_cus;
  return (int)std::max<long>(1, (tiles + per - 1) / per);
}

void conv2d_bigtile_persistent(const ConvArgs& a, int grid, hipStream_t s) {
  if (!conv_bigtile_persistent_ok(a)) throw std::invalid_argument("conv2d_bigtile_persistent: unsupported conv");
  if (a.Kpad != conv_kpad(a.Cin, a.KH, a.KW, false)) throw std::invalid_argument("conv2d_bigtile_persistent: bad Kpad");
  if (a.N > a.Npad || a.ldo < a.N) throw std::invalid_argument("conv2d_bigtile_persistent: bad N/ldo");
  if (a.Ho != conv_out_dim(a.H, a.KH, a.stride, a.pad) || a.Wo != conv_out_dim(a.W, a.KW, a.stride, a.pad))
    throw std::invalid_argument("conv2d_bigtile_persistent: bad output dims");
  if (!a.x || !a.w || !a.y || !a.zero) throw std::invalid_argument("conv2d_bigtile_persistent: null operand");
  if (((uintptr_t)a.x | (uintptr_t)a.w | (uintptr_t)a.zero | (uintptr_t)a.y | (uintptr_t)a.res |
       (uintptr_t)a.bias) & 15)
    throw std::invalid_argument("conv2d_bigtile_persistent: operands must be 16-B aligned");
  const long M = (long)a.B * a.Ho * a.Wo;
  if (M <= 0) return;
  if ((long)a.B * a.H * a.W * a.Cin >= (1L << 31) || M * a.ldo >= (1L << 31) || (long)a.Npad * a.Kpad >= (1L << 31))
    throw std::invalid_argument("conv2d_bigtile_persistent: tensor too large for 32-bit offsets");
  const long tiles = ((M + 255) / 256) * (a.Npad / 128);
  if (tiles * (a.Kpad / 64) >= (1L << 31)) throw std::invalid_argument("conv2d_bigtile_persistent: too many items");
  if (grid < 1 || grid > 65536) throw std::invalid_argument("conv2d_bigtile_persistent: bad grid");
  const size_t lds = (size_t)3 * (256 + 128) * 128;
  hipLaunchKernelGGL((conv_btp_kernel<256, 128, 4, 2, 3>), dim3(grid), dim3(512), lds, s, a, a.Kpad / 64, (int)tiles);
  DMLC_HIP_CHECK(hipGetLastError());
}

}  // namespace dmlc
