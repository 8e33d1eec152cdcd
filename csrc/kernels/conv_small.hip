// Query-batch 3x3/p1 conv (B <= a few images): ResNet layers 1-4 at the
// serving fleet's batch-1 query shape, with the block's 1x1/s2 downsample
// fused into a stride-2 conv1.
//
// Reference equivalent: every conv/bn/relu (and downsample) of the basic
// blocks of tch::vision::resnet18/34, run for ONE image per query by
// `forward_t` (src/services.rs:421,493). At B = 1 the implicit GEMM has
// M = Ho*Wo = 49..3136 pixels against K = 576..4608, so the throughput kernels
// either leave most CUs idle or split K and pay a second reduction launch per
// conv (conv_igemm + splitk_reduce: 12 + 5 us per conv, profiles/r4_*).
// Here one launch per conv, no split-K workspace, no reduction kernel:
//
//  * grid = (Cout/16 channel tiles, pixel tiles of MF x 16 pixels, B). A
//    channel tile is one 16-row N fragment (nf) of a 32-channel group g of
//    the fragment-order weights (stream_frag_index, perm32 rows), so each
//    lane ends with 4 consecutive output channels 32g + 8fq + 4nf .. +3 of one
//    pixel (8-B stores);
//  * the input rows the pixel tile reads (all columns, all channels) are
//    DMA'd into LDS once (global_load_lds_dwordx4), 16-B chunks XOR-swizzled
//    by pixel so the 16 pixels of a fragment read distinct bank groups;
//    padding taps read a zero chunk (address select, no VALU on the data);
//  * the 4 waves split K (wave w: K steps w, w+4, ...) and load ALL their
//    weight fragments into registers up front (<= 36 x 16 B per lane, issued
//    right after the input DMA: every global load of the kernel is in flight
//    at once, one memory round trip instead of a dependent chain);
//  * stride 2 with DS: the 1x1/s2 downsample reads exactly the centre tap's
//    input (pixel (2oh, 2ow)), so its K steps are the centre-tap K steps of
//    the 3x3 with the downsample's weights: a second accumulator, no loads;
//  * the 4 waves' partial sums meet in LDS; each wave then finishes whole
//    fragments: + bias (+ residual), ReLU, bf16.
#include "common.h"
#include "kernels.h"

#include <algorithm>

namespace dmlc {

namespace {

template <int N>
__device__ __forceinline__ void vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}

struct SmallArgs {
  const bf16* x;      // [B, H, W, CI]
  const bf16* wf;     // [CO/32][9 CI/32][2][64][8] fragment order
  const float* bias;  // [CO]
  const bf16* res;    // [B, Ho, Wo, CO] or null
  bf16* y;            // [B, Ho, Wo, CO]
  const bf16* wdf;    // DS: [CO/32][CI/32][2][64][8]
  const float* bd;    // DS: [CO]
  bf16* yd;           // DS: [B, Ho, Wo, CO]
  int H, W, Ho, Wo, CO;
  int relu;
};

// physical 16-B chunk of logical chunk c of staged pixel q (CH chunks per pixel)
template <int CH>
__device__ __forceinline__ int swz(int q) {
  if constexpr (CH >= 16)
    return q & 15;  // 16 pixels of a fragment: 16 distinct slots mod 256 B
  else
    return (q >> 1) & 7;  // 128-B pixels, two per 256-B bank row
}

template <int MF, bool DS>
constexpr int part_bytes() {
  return 4 * MF * 64 * 16 * (DS ? 2 : 1);
}

template <int CI, int S, int MF, bool DS>
__global__ __launch_bounds__(256, 1) void conv_small_kernel(SmallArgs a) {
  constexpr int CH = CI / 8;       // 16-B chunks per pixel
  constexpr int KPT = CI / 32;     // K steps per tap
  constexpr int KT = 9 * KPT;      // K steps
  constexpr int KW = (KT + 3) / 4; // K steps per wave (at most)
  constexpr int KDW = DS ? (KPT + 3) / 4 : 0;
  constexpr int PART = part_bytes<MF, DS>();
  constexpr int ZOFF = PART;         // 16 zero bytes
  constexpr int ROFF = PART + 16;    // staged input rows
  extern __shared__ __attribute__((aligned(16))) uint4 smem[];
  char* lds = (char*)smem;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fq = lane >> 4;
  const int g = blockIdx.x >> 1, nf = blockIdx.x & 1;
  const int b = blockIdx.z;
  const int H = a.H, W = a.W, Wo = a.Wo;
  const int P = a.Ho * Wo;
  const int p0 = blockIdx.y * (MF * 16);
  const int p1 = min(p0 + MF * 16, P);
  const int oh_lo = p0 / Wo, oh_hi = (p1 - 1) / Wo;
  const int ih_lo = max(0, oh_lo * S - 1), ih_hi = min(H - 1, oh_hi * S + 1);
  const int total = (ih_hi - ih_lo + 1) * W * CH;  // staged chunks

  // ---- input rows ih_lo..ih_hi -> LDS (slot s = q CH + c ^ swz(q))
  {
    const bf16* src0 = a.x + ((long)(b * H + ih_lo) * W) * CI;
    char* reg = lds + ROFF;
    for (int s0 = wave * 64; s0 < total; s0 += 256) {
      const int s = s0 + lane;
      if (s < total) {
        const int q = s / CH, cp = s % CH;
        dma16(src0 + (long)q * CI + (cp ^ swz<CH>(q)) * 8, reg + s0 * 16);
      }
    }
  }
  if (tid == 0) *(uint4*)(lds + ZOFF) = make_uint4(0, 0, 0, 0);

  // ---- this wave's weight fragments: K steps t = wave + 4 j
  const bf16* wb = a.wf + ((long)g * KT * 2 + nf) * 512 + lane * 8;
  bf16x8 wr[KW];
#pragma unroll
  for (int j = 0; j < KW; ++j) {
    const int t = wave + 4 * j;
    if (KT % 4 == 0 || t < KT) wr[j] = *(const bf16x8*)(wb + (long)t * 1024);
  }
  bf16x8 wd[KDW > 0 ? KDW : 1];
  if constexpr (DS) {
    const bf16* wdb = a.wdf + ((long)g * KPT * 2 + nf) * 512 + lane * 8;
#pragma unroll
    for (int j = 0; j < KDW; ++j) {
      const int td = wave + 4 * j;
      if (KPT % 4 == 0 || td < KPT) wd[j] = *(const bf16x8*)(wdb + (long)td * 1024);
    }
  }

  // ---- per-lane pixel geometry: staged pixel of tap (0, 0) and the taps
  // inside the image (bit kh*3 + kw)
  int qb[MF], vm[MF];
#pragma unroll
  for (int f = 0; f < MF; ++f) {
    const int p = p0 + 16 * f + fr;
    const int oh = p / Wo, ow = p - (p / Wo) * Wo;
    const int ih = oh * S - 1, iw = ow * S - 1;
    qb[f] = (ih - ih_lo) * W + iw;
    int m = 0;
#pragma unroll
    for (int kh = 0; kh < 3; ++kh)
#pragma unroll
      for (int kw = 0; kw < 3; ++kw)
        m |= ((unsigned)(ih + kh) < (unsigned)H && (unsigned)(iw + kw) < (unsigned)W) << (kh * 3 + kw);
    vm[f] = p < p1 ? m : 0;
  }

  // the input DMA has landed (only the weight loads, issued after it, may
  // still be in flight: vmcnt retires in order) for every wave
  // (waves with fewer K steps issued fewer loads: wait for the smallest count)
  vm_wait<KT / 4 + (DS ? KPT / 4 : 0)>();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();

  floatx4 acc[MF], accd[MF];
#pragma unroll
  for (int f = 0; f < MF; ++f) {
    acc[f] = floatx4{0.f, 0.f, 0.f, 0.f};
    accd[f] = acc[f];
  }
#pragma unroll
  for (int j = 0; j < KW; ++j) {
    const int t = wave + 4 * j;
    if (KT % 4 != 0 && t >= KT) break;
    const int tap = t / KPT;
    const int c = (t - tap * KPT) * 4 + fq;  // logical chunk
    const int kh = tap / 3, kw = tap - kh * 3;
    const int dq = kh * W + kw;
#pragma unroll
    for (int f = 0; f < MF; ++f) {
      const int q = qb[f] + dq;
      const bool ok = (vm[f] >> tap) & 1;
      const int off = ok ? ROFF + (q * CH + (c ^ swz<CH>(q))) * 16 : ZOFF;
      const bf16x8 xb = *(const bf16x8*)(lds + off);
      acc[f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wr[j], xb, acc[f], 0, 0, 0);
      if constexpr (DS) {
        // centre tap: K step td = t - 4 KPT of the downsample = this wave's j - KPT
        if (j >= KPT && j - KPT < KDW && tap == 4)
          accd[f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wd[std::min(std::max(j - KPT, 0), KDW - 1)], xb, accd[f],
                                                            0, 0, 0);
      }
    }
  }

  // ---- the 4 waves' partial sums meet in LDS: [wave][f][lane] (DS: + MF x 4 x 64)
  floatx4* part = (floatx4*)lds;
#pragma unroll
  for (int f = 0; f < MF; ++f) {
    part[(wave * MF + f) * 64 + lane] = acc[f];
    if constexpr (DS) part[(4 * MF + wave * MF + f) * 64 + lane] = accd[f];
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();

  const int ch = 32 * g + 8 * fq + 4 * nf;  // this lane's 4 output channels
  const floatx4 bs = *(const floatx4*)(a.bias + ch);
  for (int f = wave; f < MF; f += 4) {
    const int p = p0 + 16 * f + fr;
    if (p >= p1) continue;
    floatx4 v = bs;
#pragma unroll
    for (int w = 0; w < 4; ++w) v += part[(w * MF + f) * 64 + lane];
    const long o = ((long)b * P + p) * a.CO + ch;
    if (a.res) {
      const uint2 r = *(const uint2*)(a.res + o);
      v[0] += __uint_as_float(r.x << 16);
      v[1] += __uint_as_float(r.x & 0xffff0000u);
      v[2] += __uint_as_float(r.y << 16);
      v[3] += __uint_as_float(r.y & 0xffff0000u);
    }
    if (a.relu) {
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = fmaxf(v[i], 0.f);
    }
    *(uint2*)(a.y + o) = make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3]));
    if constexpr (DS) {
      floatx4 d = *(const floatx4*)(a.bd + ch);
#pragma unroll
      for (int w = 0; w < 4; ++w) d += part[(4 * MF + w * MF + f) * 64 + lane];
      *(uint2*)(a.yd + o) = make_uint2(pack2(d[0], d[1]), pack2(d[2], d[3]));
    }
  }
}

// staged input rows of the worst pixel tile
int max_rows(int H, int Ho, int Wo, int S, int mf) {
  const int P = Ho * Wo, tp = mf * 16;
  int best = 0;
  for (int p0 = 0; p0 < P; p0 += tp) {
    const int p1 = std::min(p0 + tp, P);
    const int lo = std::max(0, (p0 / Wo) * S - 1), hi = std::min(H - 1, ((p1 - 1) / Wo) * S + 1);
    best = std::max(best, hi - lo + 1);
  }
  return best;
}

size_t lds_bytes(int H, int W, int CI, int Ho, int Wo, int S, int mf, bool ds) {
  return (size_t)4 * mf * 64 * 16 * (ds ? 2 : 1) + 16 + (size_t)max_rows(H, Ho, Wo, S, mf) * W * CI * 2;
}

constexpr size_t kMaxLds = 160 * 1024;

int g_small_mf = 0;  // A/B override (tools/conv_bench.py): 0 = heuristic

template <int CI, int S, int MF, bool DS>
void launch(const SmallArgs& a, int B, size_t lds, hipStream_t s) {
  const dim3 grid(a.CO / 16, (a.Ho * a.Wo + MF * 16 - 1) / (MF * 16), B);
  hipLaunchKernelGGL((conv_small_kernel<CI, S, MF, DS>), grid, dim3(256), lds, s, a);
}

template <int CI, int S, bool DS>
void launch_mf(const SmallArgs& a, int B, int mf, size_t lds, hipStream_t s) {
  switch (mf) {
    case 1: launch<CI, S, 1, DS>(a, B, lds, s); break;
    case 2: launch<CI, S, 2, DS>(a, B, lds, s); break;
    default: launch<CI, S, 4, DS>(a, B, lds, s); break;
  }
}

}  // namespace

void conv_small_set_mf(int mf) { g_small_mf = mf; }

bool conv_small_supported(int H, int W, int CI, int CO, int stride) {
  if (!(CI == 64 || CI == 128 || CI == 256 || CI == 512) || CO % 32 != 0 || CO <= 0) return false;
  if (stride != 1 && stride != 2) return false;
  if (CI == 512 && stride == 2) return false;  // not a ResNet shape (and it spills)
  const int Ho = conv_out_dim(H, 3, stride, 1), Wo = conv_out_dim(W, 3, stride, 1);
  if (Ho <= 0 || Wo <= 0) return false;
  return lds_bytes(H, W, CI, Ho, Wo, stride, 1, stride == 2) <= kMaxLds;
}

int conv_small_pick_mf(int B, int H, int W, int CI, int CO, int stride, int num_cus) {
  const int Ho = conv_out_dim(H, 3, stride, 1), Wo = conv_out_dim(W, 3, stride, 1);
  const int P = Ho * Wo;
  if (g_small_mf == 1 || g_small_mf == 2 || g_small_mf == 4)
    return lds_bytes(H, W, CI, Ho, Wo, stride, g_small_mf, stride == 2) <= kMaxLds ? g_small_mf : 1;
  // the widest pixel tile that still gives ~half the CUs a workgroup (fewer,
  // fatter workgroups re-read the weights less often)
  for (int mf : {4, 2}) {
    const long wgs = (long)(CO / 16) * ((P + mf * 16 - 1) / (mf * 16)) * B;
    if (wgs >= num_cus / 2 && lds_bytes(H, W, CI, Ho, Wo, stride, mf, stride == 2) <= kMaxLds) return mf;
  }
  return 1;
}

void conv_small(const void* x, const void* wf, const float* bias, const void* res, void* y, int B, int H, int W,
                int CI, int CO, int stride, bool relu, int mf, hipStream_t s, const void* wdf, const float* bd,
                void* yd) {
  if (B <= 0) return;
  if (!conv_small_supported(H, W, CI, CO, stride)) throw std::invalid_argument("conv_small: unsupported shape");
  const bool ds = wdf != nullptr;
  if (ds && (stride != 2 || !bd || !yd)) throw std::invalid_argument("conv_small: the downsample needs stride 2, bd, yd");
  if (!x || !wf || !bias || !y) throw std::invalid_argument("conv_small: null operand");
  if (((uintptr_t)x | (uintptr_t)wf | (uintptr_t)y | (uintptr_t)res | (uintptr_t)wdf | (uintptr_t)yd) & 15)
    throw std::invalid_argument("conv_small: operands must be 16-B aligned");
  if (((uintptr_t)bias | (uintptr_t)bd) & 15) throw std::invalid_argument("conv_small: bias must be 16-B aligned");
  if (x == y || (res && res == y)) throw std::invalid_argument("conv_small: in-place not supported");
  if (mf != 1 && mf != 2 && mf != 4) throw std::invalid_argument("conv_small: mf must be 1, 2 or 4");
  const int Ho = conv_out_dim(H, 3, stride, 1), Wo = conv_out_dim(W, 3, stride, 1);
  const size_t lds = lds_bytes(H, W, CI, Ho, Wo, stride, mf, ds);
  if (lds > kMaxLds) throw std::invalid_argument("conv_small: pixel tile too large for LDS");
  if ((long)B * H * W * CI >= (1L << 31) || (long)B * Ho * Wo * CO >= (1L << 31))
    throw std::invalid_argument("conv_small: tensor too large for 32-bit offsets");
  if (B > 65535) throw std::invalid_argument("conv_small: batch too large");
  SmallArgs a;
  a.x = (const bf16*)x;
  a.wf = (const bf16*)wf;
  a.bias = bias;
  a.res = (const bf16*)res;
  a.y = (bf16*)y;
  a.wdf = (const bf16*)wdf;
  a.bd = bd;
  a.yd = (bf16*)yd;
  a.H = H;
  a.W = W;
  a.Ho = Ho;
  a.Wo = Wo;
  a.CO = CO;
  a.relu = relu;
  const int v = (CI == 64 ? 0 : CI == 128 ? 1 : CI == 256 ? 2 : 3) * 3 + (stride == 1 ? 0 : ds ? 2 : 1);
  switch (v) {
    case 0: launch_mf<64, 1, false>(a, B, mf, lds, s); break;
    case 1: launch_mf<64, 2, false>(a, B, mf, lds, s); break;
    case 2: launch_mf<64, 2, true>(a, B, mf, lds, s); break;
    case 3: launch_mf<128, 1, false>(a, B, mf, lds, s); break;
    case 4: launch_mf<128, 2, false>(a, B, mf, lds, s); break;
    case 5: launch_mf<128, 2, true>(a, B, mf, lds, s); break;
    case 6: launch_mf<256, 1, false>(a, B, mf, lds, s); break;
    case 7: launch_mf<256, 2, false>(a, B, mf, lds, s); break;
    case 8: launch_mf<256, 2, true>(a, B, mf, lds, s); break;
    default: launch_mf<512, 1, false>(a, B, mf, lds, s); break;
  }
  DMLC_HIP_CHECK(hipGetLastError());
}

}  // namespace dmlc
