// Fused ResNet50 identity bottleneck on whole-image workgroups: layer3
// (14x14, C = 1024, M = 256: layer3.1 .. 3.5) and layer4 (7x7, C = 2048,
// M = 512: layer4.1, 4.2) of resnet50_fp8:
//   t1 = relu(bn1(conv1x1 C->M (x)))        e4m3 MFMA (16x16x128), t1 bf16 in LDS
//   t2 = relu(bn2(conv3x3 M->M (t1)))       bf16 MFMA, accumulated in VGPRs
//   y  = relu(bn3(conv1x1 M->C (t2)) + x)   bf16 MFMA, y e4m3
// in ONE kernel per block: x is read twice (conv1 operand, then the residual,
// an L2 / MALL hit), y written once; t1 and t2 never reach HBM.
//
// Reference equivalent: torchvision Bottleneck.forward (conv1/bn1/relu,
// conv2/bn2/relu, conv3/bn3, += identity, relu) of tch::vision::resnet50, run
// per query by `forward_t` (src/services.rs:493; BASELINE config 5). Unfused,
// a layer3 block is three launches that write and re-read both 14x14x256 bf16
// intermediates (4 x 25.7 MB at B = 256) and pay three prologues.
//
// One workgroup = one image (1 per CU: ~100 KB of LDS at layer3), 8 waves,
// every wave on every pixel fragment (NPF = ceil(H*H / 16): 13 at layer3, 4 at
// layer4) and its own slice of output channels, so the 4 SIMDs carry equal
// work and each weight byte is read by one wave only:
//  A. conv1: x goes HBM -> LDS in chunks of 256 channels by LDS-DMA, two
//     buffers (chunk i+1 lands while chunk i computes), 16-B chunks XOR-
//     swizzled by pixel; each wave streams its M/8 channels' e4m3 weight rows
//     from L2 a chunk ahead; epilogue alpha/bias/ReLU -> bf16 t1 in LDS (over
//     the x buffers, after a barrier);
//  B. conv2: 3x3 over t1 (padding taps read a zero chunk), weights through a
//     PD-deep register ring in MFMA fragment order; the result stays in
//     VGPRs until every wave is done with t1, then overwrites it as t2;
//  C. conv3: each wave's C/8 output channels in passes of 32 / 64, its
//     residual rows loaded at the start of each pass; 1/s_y folded into the
//     bias and residual scale, one med3 for ReLU + e4m3 saturation.
// Weight rows are read in the perm32 order (row r of N fragment nf of a
// 32-channel group is channel 8 (r >> 2) + 4 nf + (r & 3)), so a lane's
// accumulators are 8 consecutive channels of one pixel: 16-B t1 / t2 LDS
// stores, 8-B e4m3 residual loads and y stores.
#include "common.h"
#include "kernels.h"

namespace dmlc {

namespace {

typedef int v8i __attribute__((ext_vector_type(8)));

template <int N>
__device__ __forceinline__ void vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
}

struct BiArgs {
  const uint8_t* x;    // [B, H, H, C] e4m3 (value = e4m3 * res_scale)
  const uint8_t* w1;   // [M][C] e4m3 (per-row scales folded into a1)
  const float* a1;     // [M] s_x * s_w1[n]
  const float* b1;     // [M]
  const bf16* wf2;     // [M/32][9M/32][2][64][8] fragment order (stream_frag_index, K = 9M)
  const float* b2;     // [M]
  const bf16* w3;      // [C][M] bf16 row-major
  const float* b3;     // [C]
  uint8_t* y;          // [B, H, H, C] e4m3
  float res_scale;     // s_x
  float out_inv_scale; // 1 / s_y
};
// DBG (timing knock-outs, tools/bottleneck_img_bench.py; layer3 only): bit 0
// no conv1 MFMAs, bit 1 no conv2 loop, bit 2 no conv3 loop, bit 3 no residual
// loads / y stores

// A workgroup owns RS output rows (a strip; RS = H: the whole image) of one
// image; t1 is computed for those rows plus the halo rows inside the image.
// Its 8 waves are PG pixel groups x 8/PG channel groups.
template <int H, int C, int M, int RS, int PG, int KC>
struct BiGeom {
  static constexpr int NS = H / RS;                  // strips per image
  static constexpr int TRM = NS == 1 ? H : RS + 2;   // t1 rows (most)
  static constexpr int TPX = TRM * H;                // t1 pixels (most)
  static constexpr int OPX = RS * H;                 // output pixels
  static constexpr int NA = ((TPX + 15) / 16 + PG - 1) / PG;  // conv1 fragments per pixel group
  static constexpr int NB = ((OPX + 15) / 16 + PG - 1) / PG;  // conv2 / conv3 fragments per pixel group
  static constexpr int CGW = 8 / PG;                 // channel groups (waves per pixel group)
  static constexpr int NFW = M / CGW / 16;           // conv1 / conv2 N fragments per wave
  static constexpr int NG = NFW / 2;                 // ... = perm32 groups per wave
  static constexpr int C3W = C / CGW;                // conv3 channels per wave
  static constexpr int NP3 = C3W / (32 * NG);        // conv3 passes of NG groups
  static constexpr int KS1 = C / 128;                // conv1 e4m3 K steps
  static constexpr int KPC = KC / 128;               // ... per staged x chunk
  static constexpr int NCH = C / KC;                 // x chunks
  static constexpr int XCB = TPX * KC;               // bytes per staged x chunk
  // t1 / t2: a zero-haloed grid of (RS + 2) x (H + 2) pixels (output rows r0
  // - 1 .. r0 + RS, columns -1 .. H), PXS bytes per pixel: M * 2 + 16, so
  // consecutive pixels start one 16-B bank slot apart (PXS / 16 = 1 mod 16:
  // conflict-free fragment reads, no XOR) and every tap / channel offset of
  // a conv2 or conv3 read is an immediate on one per-fragment address
  static constexpr int HP = H + 2;
  static constexpr int PXS = M * 2 + 16;
  static constexpr int TB = (RS + 2) * HP * PXS;     // t1 / t2 bytes
  static constexpr int KPT = M / 32;                 // conv2 K steps per tap
  static constexpr int KS2 = 9 * KPT;                // conv2 K steps
  static constexpr int KS3 = M / 32;                 // conv3 K steps
  static constexpr int PD = 4;                       // conv2 / conv3 weight ring depth
  static constexpr size_t LDS = (size_t)(TB > 2 * XCB ? TB : 2 * XCB);
  static_assert(H % RS == 0 && 8 % PG == 0 && NFW % 2 == 0 && NFW >= 2, "shape");
  static_assert(C3W % (32 * NG) == 0 && C % KC == 0 && (KC == 128 || KC == 256), "shape");
  static_assert(KS2 % PD == 0 && KS3 % PD == 0, "weight ring period");
  static_assert(LDS <= 160 * 1024, "LDS budget");
};

// staged x chunk: pixel p's KC / 16 chunks of 16 e4m3 channels; KC = 256:
// chunk c at c ^ (p & 15); KC = 128 (two pixels per 256-B bank row): c ^
// ((p >> 1) & 7). Either way the 16 pixels of a fragment read 16 distinct
// bank slots.
template <int KC>
__device__ __forceinline__ int x_swz(int p) {
  return KC == 256 ? (p & 15) : ((p >> 1) & 7);
}
template <int KC>
__device__ __forceinline__ int x_off(int p, int c) {
  return p * KC + ((c ^ x_swz<KC>(p)) << 4);
}

__device__ __forceinline__ v8i cat8(const uint4& lo, const uint4& hi) {
  return v8i{(int)lo.x, (int)lo.y, (int)lo.z, (int)lo.w, (int)hi.x, (int)hi.y, (int)hi.z, (int)hi.w};
}

// values already within +-448
__device__ __forceinline__ uint32_t f32x4_to_fp8_sat(const float* f) {
  int v = __builtin_amdgcn_cvt_pk_fp8_f32(f[0], f[1], 0, false);
  v = __builtin_amdgcn_cvt_pk_fp8_f32(f[2], f[3], v, true);
  return (uint32_t)v;
}
__device__ __forceinline__ void fp8x4_to_f32(uint32_t u, float* f) {
  e4m3x4_to_f32(u, f);
}

// A global pointer the compiler cannot move loads through: kernel-argument
// pointers are readonly + noalias, so it hoists their loads to the kernel
// start (epilogue constants, residuals, every unrolled step's weights) and
// spills them. Laundered where the loads are meant to issue; the cast keeps
// them global_load (a laundered generic pointer became flat_load).
template <typename T>
__device__ __forceinline__ const __attribute__((address_space(1))) T* gl(const T* p) {
  asm volatile("" : "+s"(p));
  return (const __attribute__((address_space(1))) T*)p;
}

// perm32: A-operand row fr of N fragment nf of 32-channel group gg
__device__ __forceinline__ int perm_ch(int gg, int nf, int fr) { return 32 * gg + 8 * (fr >> 2) + 4 * nf + (fr & 3); }

template <int H, int C, int M, int RS, int PG, int KC, int DBG = 0>
__global__ __launch_bounds__(512, 1) void bottleneck_img_kernel(BiArgs a) {
  using G = BiGeom<H, C, M, RS, PG, KC>;
  constexpr int NA = G::NA, NB = G::NB, NFW = G::NFW, NG = G::NG;
  extern __shared__ __attribute__((aligned(16))) uint4 smem[];
  char* lds = (char*)smem;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fq = lane >> 4;
  const int pg = PG == 1 ? 0 : wave / G::CGW;     // pixel group
  const int cg = PG == 1 ? wave : wave % G::CGW;  // channel group
  const int b = blockIdx.x / G::NS, strip = blockIdx.x % G::NS;
  const int r0 = strip * RS;                                     // first output row
  const int t0 = r0 > 0 ? r0 - 1 : 0;                            // first t1 row
  const int tpx = ((r0 + RS < H ? r0 + RS + 1 : H) - t0) * H;    // t1 pixels of this strip
  constexpr int OPX = G::OPX;
  const uint8_t* xim = a.x + (long)b * H * H * C;
  uint8_t* yim = a.y + (long)b * H * H * C;

  // ======== A. conv1 (e4m3) over staged x chunks (t1 pixels of the strip) ========
  // chunk i -> buffer i & 1. KC = 256: a DMA instruction covers pixels 4j ..
  // 4j+3 (lane -> pixel 4j + (lane >> 4), physical chunk lane & 15); KC = 128:
  // pixels 8j .. 8j+7 (lane >> 3, physical chunk lane & 7)
  constexpr int PPI = 1024 / KC;  // pixels per DMA instruction
  const char* xt = (const char*)xim + (long)t0 * H * C;
  auto dma_x = [&](int i) __attribute__((always_inline)) {
    char* buf = lds + (i & 1) * G::XCB;
    for (int j = wave; j < (tpx + PPI - 1) / PPI; j += 8) {
      const int p = PPI * j + lane / (KC / 16);
      const int pc = lane % (KC / 16);
      if (p < tpx) dma16(xt + (long)p * C + KC * i + 16 * (pc ^ x_swz<KC>(p)), buf + j * 1024);
    }
  };
  // this wave's conv1 / conv2 channels: perm32 groups cg * NG .. + NG - 1.
  // Its e4m3 weight fragment of K step ks, N fragment n: 32 B per lane by
  // two buffer loads (per-lane row offset, K step as the scalar offset). The
  // K steps are unrolled, so the scalar offset goes through an empty asm
  // where the loads issue: the weight pointer is a readonly noalias kernel
  // argument, and the compiler otherwise issued every K step's weights up
  // front and spilled.
  const __amdgpu_buffer_rsrc_t w1rs = wave_rsrc(a.w1, M * C);
  uint32_t w1vo[NFW];
#pragma unroll
  for (int n = 0; n < NFW; ++n) w1vo[n] = (uint32_t)(perm_ch(cg * NG + (n >> 1), n & 1, fr) * C + 32 * fq);
  auto w1frag = [&](int ks, int n) __attribute__((always_inline)) {
    int so = 128 * ks;
    asm volatile("" : "+s"(so));
    const uint4 lo = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(w1rs, w1vo[n], so, 0));
    const uint4 hi = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(w1rs, w1vo[n] + 16, so, 0));
    return cat8(lo, hi);
  };
  floatx4 acc[NA][NFW];
#pragma unroll
  for (int f = 0; f < NA; ++f)
#pragma unroll
    for (int n = 0; n < NFW; ++n) acc[f][n] = floatx4{0.f, 0.f, 0.f, 0.f};
  dma_x(0);
  // weights through a 3-deep ring (K step ks + 2 issued while ks computes;
  // 2-deep when the accumulators leave no room: layer2's 14 fragments)
  constexpr int WR = NA * NFW > 26 ? 2 : 3;
  v8i wq1[WR][NFW];
#pragma unroll
  for (int s = 0; s < WR - 1; ++s)
#pragma unroll
    for (int n = 0; n < NFW; ++n) wq1[s][n] = w1frag(s, n);
#pragma unroll
  for (int ks = 0; ks < G::KS1; ++ks) {
    const int i = ks / G::KPC, kk = ks % G::KPC;
    if (kk == 0) {
      vm_wait<0>();   // chunk i (this wave's DMA) landed (and the weights issued so far)
      lds_barrier();  // every wave's part of chunk i; every wave done with chunk i - 1
      if (i + 1 < G::NCH) dma_x(i + 1);
    }
    if (ks + WR - 1 < G::KS1) {
#pragma unroll
      for (int n = 0; n < NFW; ++n) wq1[(ks + WR - 1) % WR][n] = w1frag(ks + WR - 1, n);
    }
    const char* buf = lds + (i & 1) * G::XCB;
    // fragment f's operand (chunks 8 kk + 2 fq, +1 of the pixel); the next
    // one's read while the current one's MFMAs issue (sched barriers:
    // hoisting every read spilled)
    auto xread = [&](int f) __attribute__((always_inline)) {
      int p = min(16 * (pg * NA + f) + fr, tpx - 1);  // (padding lanes: a real pixel, results unused)
      asm volatile("" : "+v"(p));                     // recomputed per read: hoisted, the addresses stayed live
      return cat8(*(const uint4*)(buf + x_off<KC>(p, 8 * kk + 2 * fq)),
                  *(const uint4*)(buf + x_off<KC>(p, 8 * kk + 2 * fq + 1)));
    };
    // operands XA fragments ahead (see phase B), within the K step
    constexpr int XA = NFW >= 4 ? 2 : (NA >= 3 ? 3 : NA);  // (4 N fragments: 128 MFMA cycles per fragment)
    v8i xr[XA];
#pragma unroll
    for (int f = 0; f < XA; ++f) xr[f] = xread(f);
#pragma unroll
    for (int f = 0; f < NA; ++f) {
      const v8i xv = xr[f % XA];
      if (f + XA < NA) xr[f % XA] = xread(f + XA);
      __builtin_amdgcn_sched_barrier(0);
      if (!(DBG & 1)) {
#pragma unroll
        for (int n = 0; n < NFW; ++n)  // formats 0/0 = e4m3; E8M0 scales 127 = 1.0
          acc[f][n] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(wq1[ks % WR][n], xv, acc[f][n], 0, 0, 0, 127, 0,
                                                                       127);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  // (the stores below are conditional on the pixel: unpinned, the compiler
  // sank whole MFMA chains into that branch, with every operand kept live)
#pragma unroll
  for (int f = 0; f < NA; ++f)
#pragma unroll
    for (int n = 0; n < NFW; ++n) asm volatile("" : "+v"(acc[f][n]));
  lds_barrier();  // every wave done with the x buffers: t1 goes over them
  {
    const auto* a1p = gl(a.a1);
    const auto* b1p = gl(a.b1);
#pragma unroll
    for (int j = 0; j < NG; ++j) {
      const int c0 = 32 * (cg * NG + j) + 8 * fq;  // this lane's 8 channels of group j
      float al[8], bi[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        al[e] = a1p[c0 + e];
        bi[e] = b1p[c0 + e];
      }
#pragma unroll
      for (int f = 0; f < NA; ++f) {
        // (padding pixels: computed, not stored; a `continue` around the
        // whole body made the unrolled loop spill)
        const int p = 16 * (pg * NA + f) + fr;
        float v[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = fmaxf(acc[f][2 * j + (e >> 2)][e & 3] * al[e] + bi[e], 0.f);
        const uint4 pk = pack8(v);
        // t1 pixel p = image row t0 + p / H -> grid row t0 - r0 + 1 + p / H, column p % H + 1
        const int gq = (t0 - r0 + 1 + p / H) * G::HP + p % H + 1;
        if (p < tpx) *(uint4*)(lds + gq * G::PXS + c0 * 2) = pk;
      }
    }
  }
  // the grid's halo (zero padding of conv2): columns 0 and H + 1 of every
  // row, and the rows above / below the image at its top / bottom strip
  {
    constexpr int CPX = G::PXS / 16;  // 16-B chunks per grid pixel
    const bool top = r0 == 0, bot = r0 + RS == H;
    const int nrow = (top ? G::HP : 0) + (bot ? G::HP : 0);
    const int items = (2 * (RS + 2) + nrow) * CPX;
    for (int it = tid; it < items; it += 512) {
      const int px = it / CPX, cc = it - px * CPX;
      int gq;
      if (px < 2 * (RS + 2)) {
        gq = (px >> 1) * G::HP + ((px & 1) ? H + 1 : 0);
      } else {
        const int k = px - 2 * (RS + 2);
        gq = (top && k < G::HP) ? k : (RS + 1) * G::HP + (top ? k - G::HP : k);
      }
      *(uint4*)(lds + gq * G::PXS + cc * 16) = make_uint4(0, 0, 0, 0);
    }
  }
  lds_barrier();

  // ======== B. conv2 (3x3, bf16) over t1 ========
  // output pixel op of the strip = image pixel (r0 + op / H, op % H) = grid
  // pixel (op / H + 1, op % H + 1); gb: byte address of its tap (0, 0) grid
  // pixel plus this lane's 16-B chunk (padding lanes: a real pixel, results
  // unused). A tap adds (kh HP + kw) PXS, a K step within it 64 B.
  int gb[NB];
#pragma unroll
  for (int f = 0; f < NB; ++f) {
    const int op = min(16 * (pg * NB + f) + fr, OPX - 1);
    gb[f] = ((op / H) * G::HP + op % H) * G::PXS + fq * 16;
  }
  floatx4 acc2[NB][NFW];
#pragma unroll
  for (int f = 0; f < NB; ++f)
#pragma unroll
    for (int n = 0; n < NFW; ++n) acc2[f][n] = floatx4{0.f, 0.f, 0.f, 0.f};
  {
    constexpr int PD = G::PD, KPT = G::KPT;
    static_assert(KPT % PD == 0, "weight ring aligned to a tap");
    // fragment-order weights of this wave's groups: byte offset of
    // (group cg * NG + (n >> 1), K step ks, nf = n & 1) = ((g KS2 + ks) 2 + nf) 1 KB
    const __amdgpu_buffer_rsrc_t w2rs = wave_rsrc(a.wf2 + (long)cg * NG * G::KS2 * 1024, NG * G::KS2 * 2048);
    auto w2 = [&](int ks, int n) __attribute__((always_inline)) {
      int so = ks * 2048;
      asm volatile("" : "+s"(so));  // (see w1frag)
      return __builtin_bit_cast(
          bf16x8, __builtin_amdgcn_raw_buffer_load_b128(w2rs, lane * 16 + ((n >> 1) * G::KS2 * 2 + (n & 1)) * 1024, so, 0));
    };
    bf16x8 wq[PD][NFW];
#pragma unroll
    for (int s = 0; s < PD - 1; ++s)
#pragma unroll
      for (int n = 0; n < NFW; ++n) wq[s][n] = w2(s, n);
    // per tap: NB address adds, then KPT K steps whose reads are the tap
    // address + immediates; (K step, fragment) items in order, the operand of
    // item i + XD read while item i's MFMAs issue (a fragment's NFW MFMAs do
    // not cover an LDS read)
    constexpr int XD = 4;
    for (int tap = 0; tap < ((DBG & 2) ? 0 : 9); ++tap) {
      const int toff = ((tap / 3) * G::HP + tap % 3) * G::PXS;
      int tb[NB];
#pragma unroll
      for (int f = 0; f < NB; ++f) tb[f] = gb[f] + toff;
      auto tread = [&](int kc, int f) __attribute__((always_inline)) {
        return *(const bf16x8*)(lds + tb[f] + kc * 64);
      };
      bf16x8 xr[XD];
#pragma unroll
      for (int i = 0; i < XD; ++i) xr[i] = tread(i / NB, i % NB);
#pragma unroll
      for (int kc = 0; kc < KPT; ++kc) {
        const int ks = tap * KPT + kc;
        if (ks + PD - 1 < G::KS2) {
#pragma unroll
          for (int n = 0; n < NFW; ++n) wq[(kc + PD - 1) % PD][n] = w2(ks + PD - 1, n);
        }
#pragma unroll
        for (int f = 0; f < NB; ++f) {
          const int i = kc * NB + f, in = i + XD;  // (compile time)
          const bf16x8 xb = xr[i % XD];
          if (in < KPT * NB) xr[i % XD] = tread(in / NB, in % NB);
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int n = 0; n < NFW; ++n)
            acc2[f][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wq[kc % PD][n], xb, acc2[f][n], 0, 0, 0);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
    }
  }
  // t2 = relu(acc + b2) as bf16, held until every wave is done reading t1
#pragma unroll
  for (int f = 0; f < NB; ++f)
#pragma unroll
    for (int n = 0; n < NFW; ++n) asm volatile("" : "+v"(acc2[f][n]));  // (see phase A)
  uint4 tv[NB][NG];
  {
    const auto* b2p = gl(a.b2);
#pragma unroll
    for (int j = 0; j < NG; ++j) {
      const int c0 = 32 * (cg * NG + j) + 8 * fq;
      float bi[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) bi[e] = b2p[c0 + e];
#pragma unroll
      for (int f = 0; f < NB; ++f) {
        float v[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = fmaxf(acc2[f][2 * j + (e >> 2)][e & 3] + bi[e], 0.f);
        tv[f][j] = pack8(v);
      }
    }
  }
#pragma unroll
  for (int f = 0; f < NB; ++f)
#pragma unroll
    for (int j = 0; j < NG; ++j) asm volatile("" : "+v"(tv[f][j].x), "+v"(tv[f][j].y), "+v"(tv[f][j].z), "+v"(tv[f][j].w));
  lds_barrier();
  // t2 at output pixel op (stride M * 2 per pixel, over t1)
#pragma unroll
  for (int j = 0; j < NG; ++j)
#pragma unroll
    for (int f = 0; f < NB; ++f) {
      const int op = 16 * (pg * NB + f) + fr;
      // t2 at the output pixel's own grid position (its tap (1, 1))
      const int gq = (op / H + 1) * G::HP + op % H + 1;
      if (op < OPX) *(uint4*)(lds + gq * G::PXS + (32 * (cg * NG + j) + 8 * fq) * 2) = tv[f][j];
    }
  lds_barrier();

  // ======== C. conv3 (1x1, bf16) + residual -> e4m3 ========
  {
    constexpr int PD = G::PD;
    const float inv = a.out_inv_scale, rsi = a.res_scale * inv;
    const uint8_t* xo = xim + (long)r0 * H * C;  // the strip's first output pixel
    uint8_t* yo = yim + (long)r0 * H * C;
    const __amdgpu_buffer_rsrc_t w3rs = wave_rsrc(a.w3, C * M * 2);
    for (int pass = 0; pass < G::NP3; ++pass) {
      const int gg0 = cg * (G::C3W / 32) + pass * NG;  // first 32-channel group of the pass
      // residual: 8 e4m3 channels 32 gg + 8 fq .. of each pixel, loaded at
      // the start of the pass (in flight under its MFMAs), or after them
      // when the accumulators leave no room (layer2's 13 fragments: spilled)
      constexpr bool kEarlyRes = NB * NFW <= 24;
      uint2 rv[NB][NG];
      auto load_rv = [&]() __attribute__((always_inline)) {
        const auto* xr = gl(xo);
#pragma unroll
        for (int f = 0; f < NB; ++f)
#pragma unroll
          for (int j = 0; j < NG; ++j) {
            const int op = min(16 * (pg * NB + f) + fr, OPX - 1);
            const uint64_t r =
                *(const __attribute__((address_space(1))) uint64_t*)(xr + (long)op * C + 32 * (gg0 + j) + 8 * fq);
            rv[f][j] = make_uint2((uint32_t)r, (uint32_t)(r >> 32));
          }
      };
      if (DBG & 8) {
#pragma unroll
        for (int f = 0; f < NB; ++f)
#pragma unroll
          for (int j = 0; j < NG; ++j) rv[f][j] = make_uint2(0, 0);
      } else if constexpr (kEarlyRes) {
        load_rv();
      }
      // w3 rows (perm32) of this pass: per-lane row offset, K step as the scalar offset
      uint32_t w3vo[NFW];
#pragma unroll
      for (int n = 0; n < NFW; ++n) w3vo[n] = (uint32_t)((perm_ch(gg0 + (n >> 1), n & 1, fr) * M + 8 * fq) * 2);
      auto w3 = [&](int ks, int n) __attribute__((always_inline)) {
        int so = 64 * ks;
        asm volatile("" : "+s"(so));  // (see w1frag)
        return __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(w3rs, w3vo[n], so, 0));
      };
      floatx4 c3[NB][NFW];
#pragma unroll
      for (int f = 0; f < NB; ++f)
#pragma unroll
        for (int n = 0; n < NFW; ++n) c3[f][n] = floatx4{0.f, 0.f, 0.f, 0.f};
      bf16x8 wq[PD][NFW];
#pragma unroll
      for (int s = 0; s < PD - 1; ++s)
#pragma unroll
        for (int n = 0; n < NFW; ++n) wq[s][n] = w3(s, n);
      auto t2read = [&](int ks, int f) __attribute__((always_inline)) {
        return *(const bf16x8*)(lds + gb[f] + (G::HP + 1) * G::PXS + ks * 64);
      };
      constexpr int XD = 4;  // (see phase B)
      static_assert((PD * NB) % XD == 0, "operand ring aligned to the unrolled block");
      bf16x8 xr[XD];
#pragma unroll
      for (int i = 0; i < XD; ++i) xr[i] = t2read(i / NB, i % NB);
#pragma unroll
      for (int k0 = 0; k0 < ((DBG & 4) ? 0 : G::KS3); k0 += PD) {
#pragma unroll
        for (int s = 0; s < PD; ++s) {
          const int ks = k0 + s;
          if (ks + PD - 1 < G::KS3) {
#pragma unroll
            for (int n = 0; n < NFW; ++n) wq[(s + PD - 1) % PD][n] = w3(ks + PD - 1, n);
          }
#pragma unroll
          for (int f = 0; f < NB; ++f) {
            const int i = s * NB + f, in = i + XD;  // (compile time)
            const bf16x8 xb = xr[i % XD];
            if (k0 + in / NB < G::KS3) xr[i % XD] = t2read(k0 + in / NB, in % NB);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int n = 0; n < NFW; ++n)
              c3[f][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wq[s][n], xb, c3[f][n], 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
          }
        }
      }
#pragma unroll
      for (int f = 0; f < NB; ++f)
#pragma unroll
        for (int n = 0; n < NFW; ++n) asm volatile("" : "+v"(c3[f][n]));  // (see phase A)
      if constexpr (!kEarlyRes) {
        if (!(DBG & 8)) load_rv();
      }
      const auto* b3p = gl(a.b3);
#pragma unroll
      for (int j = 0; j < NG; ++j) {
        const int c0 = 32 * (gg0 + j) + 8 * fq;
        float bs[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) bs[e] = b3p[c0 + e] * inv;
#pragma unroll
        for (int f = 0; f < NB; ++f) {
          const int op = 16 * (pg * NB + f) + fr;
          float r[8], v[8];
          fp8x4_to_f32(rv[f][j].x, r);
          fp8x4_to_f32(rv[f][j].y, r + 4);
#pragma unroll
          for (int e = 0; e < 8; ++e)
            v[e] = __builtin_amdgcn_fmed3f(c3[f][2 * j + (e >> 2)][e & 3] * inv + bs[e] + r[e] * rsi, 0.f, 448.f);
          const uint2 pk = make_uint2(f32x4_to_fp8_sat(v), f32x4_to_fp8_sat(v + 4));
          if (op < OPX && (!(DBG & 8) || pk.x == 0x12345678u)) *(uint2*)(yo + (long)op * C + c0) = pk;
        }
      }
    }
  }
}

}  // namespace

bool bottleneck_img_supported(int H, int W, int C, int M) {
  return H == W && ((H == 28 && C == 512 && M == 128) || (H == 14 && C == 1024 && M == 256) ||
                    (H == 7 && C == 2048 && M == 512));
}

void bottleneck_img(const void* x, const void* w1, const float* a1, const float* b1, const void* wf2, const float* b2,
                    const void* w3, const float* b3, void* y, float res_scale, float out_inv_scale, int B, int H, int C,
                    int M, hipStream_t s, int dbg) {
  if (B <= 0) return;
  if (!bottleneck_img_supported(H, H, C, M)) throw std::invalid_argument("bottleneck_img: unsupported shape");
  if (!x || !w1 || !a1 || !b1 || !wf2 || !b2 || !w3 || !b3 || !y ||
      (((uintptr_t)x | (uintptr_t)w1 | (uintptr_t)wf2 | (uintptr_t)w3 | (uintptr_t)y) & 15))
    throw std::invalid_argument("bottleneck_img: null / misaligned operand");
  if (x == y) throw std::invalid_argument("bottleneck_img: in-place not supported (the residual is re-read)");
  if ((long)B * H * H * C >= (1L << 31)) throw std::invalid_argument("bottleneck_img: tensor too large");
  BiArgs a;
  a.x = (const uint8_t*)x;
  a.w1 = (const uint8_t*)w1;
  a.a1 = a1;
  a.b1 = b1;
  a.wf2 = (const bf16*)wf2;
  a.b2 = b2;
  a.w3 = (const bf16*)w3;
  a.b3 = b3;
  a.y = (uint8_t*)y;
  a.res_scale = res_scale;
  a.out_inv_scale = out_inv_scale;
  // layer2: half-image strips (t1 of 15 rows: 105 KB), 2 pixel groups x 4
  // channel groups, x staged 128 channels at a time; layer3 / layer4: whole
  // images, 8 channel groups, 256 channels at a time
  using G2 = BiGeom<28, 512, 128, 14, 2, 128>;
  using G3 = BiGeom<14, 1024, 256, 14, 1, 256>;
  using G4 = BiGeom<7, 2048, 512, 7, 1, 256>;
  constexpr size_t lds2 = G2::LDS, lds3 = G3::LDS, lds4 = G4::LDS;
  if (H == 28)
    hipLaunchKernelGGL((bottleneck_img_kernel<28, 512, 128, 14, 2, 128>), dim3(B * G2::NS), dim3(512), lds2, s, a);
  else if (H == 14) {
    switch (dbg) {
#define DMLC_BI_DBG(D)                                                                                             \
  case D:                                                                                                          \
    hipLaunchKernelGGL((bottleneck_img_kernel<14, 1024, 256, 14, 1, 256, D>), dim3(B), dim3(512), lds3, s, a); \
    break;
      DMLC_BI_DBG(1) DMLC_BI_DBG(2) DMLC_BI_DBG(4)
#undef DMLC_BI_DBG
      default: hipLaunchKernelGGL((bottleneck_img_kernel<14, 1024, 256, 14, 1, 256>), dim3(B), dim3(512), lds3, s, a);
    }
  }
  else
    hipLaunchKernelGGL((bottleneck_img_kernel<7, 2048, 512, 7, 1, 256>), dim3(B), dim3(512), lds4, s, a);
  DMLC_HIP_CHECK(hipGetLastError());
}

}  // namespace dmlc
