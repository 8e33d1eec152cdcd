// Fused AlexNet stem: u8 image -> ImageNet normalisation -> conv 11x11/s4/p2
// (+bias) -> ReLU -> maxpool 3x3/s2, one workgroup per image, the 55x55x64
// conv output never leaves LDS. [B, 224, 224, 3] u8 in, [B, 27, 27, 64] bf16
// NHWC out.
//
// Reference equivalent: tch::vision::alexnet's features.0 (conv), .1 (relu),
// .2 (maxpool) after imagenet::load_image_and_resize's normalisation, run per
// query by `forward_t` (src/services.rs:492-493). As three kernels
// (preprocess_u8, the packed-RGB implicit GEMM, maxpool2d) the stem took
// 41 + 157 + ~20 us at B = 256 (profiles/r2_alexnet_b256_kernel_stats.txt):
// the implicit GEMM's 11x11 im2col re-reads every input pixel ~30x and its
// 64-wide N tile leaves most of each MFMA tile idle.
//
//  * Paired rows: padded pixel column j (image column j - 2) pairs into 16-B
//    chunks p = (2p, 2p+1) as bf16 [r g b r g b 0 0]. With stride 4, output
//    column ow reads padded columns 4ow .. 4ow+10 = chunks 2ow .. 2ow+5 of
//    each kernel row, so K = 11 rows x 6 chunks x 8 = 528 (+16 zero) = 17
//    MFMA k-steps of 32, and every B operand is one aligned ds_read_b128 from
//    the staged row (no im2col). Weights are zero on the pad slots (e = 6, 7,
//    kw = 11, kh = 11).
//  * Two conv rows per iteration and one barrier (one row per barrier: 87 us
//    at B=256, ~2,000 cycles of phase overhead per row beside ~1,100 of
//    MFMA per SIMD). The raw u8 rows of conv rows r0+8, r0+9 go out by
//    LDS-DMA during iteration r0 and are converted into the paired ring two
//    iterations later (beside the MFMAs of the SIMD's other wave).
//  * 8 waves: wave w = pixel fragment w & 3 (16 output columns) x output
//    channels 32 (w >> 2) .. +31 (two n-blocks), D = W x X with the weight
//    rows permuted (perm32) so a lane ends with 8 consecutive channels of one
//    pixel; all 17 x 2 weight fragments stay in VGPRs.
//  * + bias, ReLU, bf16 -> a 4-slot ring of conv rows [55][64] in LDS (16-B
//    chunks XOR-swizzled by pixel: conflict-free stores and reads); every
//    second conv row the 3x3/s2 max of the three latest rows is stored as one
//    pooled row (post-ReLU values are >= 0: bf16 max = unsigned 16-bit max).
#include "common.h"
#include "kernels.h"

namespace dmlc {

namespace {

typedef unsigned short ushort8 __attribute__((ext_vector_type(8)));

constexpr int kS = 224;         // input image size
constexpr int kHo = 55;         // conv output size
constexpr int kPH = 27;         // pooled output size
constexpr int kC = 64;          // output channels
constexpr int kChunks = 114;    // paired chunks per padded row (228 padded pixels)
constexpr int kRowB = 136 * 16; // staged paired row: chunks >= 114 stay zero (fragment padding reads up to 131)
constexpr int kRing = 32;       // paired rows (power of two): 15 in use + 16 converted ahead
constexpr int kKS = 17;         // K steps of 32 (68 chunks, 66 used)
constexpr int kU8B = kS * 3;    // 672 bytes per raw image row
constexpr int kU8Slot = 704;    // raw ring slot (16-B aligned)
constexpr int kU8Ring = 32;     // raw rows: 8 converting + 16 in flight (DMA two iterations ahead)
constexpr int kConvB = kHo * 128;  // one conv row [55][64] bf16
constexpr int kConvRing = 8;    // conv rows: 3 pooled + 2 written per iteration
constexpr size_t kLds = (size_t)kRing * kRowB + (size_t)kConvRing * kConvB + (size_t)kU8Ring * kU8Slot;

struct AlexStemArgs {
  const uint8_t* x;    // [B, 224, 224, 3]
  const bf16* w;       // [64][544] paired-chunk K order (alex_stem_k)
  const float* bias;   // [64]
  bf16* y;             // [B, 27, 27, 64]
};

__device__ __forceinline__ int perm32(int n) {
  const int nf = n >> 4, r = n & 15;
  return 8 * (r >> 2) + 4 * nf + (r & 3);
}

// conv-ring byte offset of 16-B channel chunk c of pixel px
__device__ __forceinline__ int conv_off(int px, int c) { return px * 128 + ((c ^ (px & 7)) << 4); }

__global__ __launch_bounds__(512, 1) void alex_stem_kernel(AlexStemArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint4 smem[];
  char* ring = (char*)smem;
  char* conv = ring + kRing * kRowB;
  char* raw = conv + kConvRing * kConvB;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fq = lane >> 4;
  const int b = blockIdx.x;
  const uint8_t* img = a.x + (long)b * kS * kU8B;

  // zero the paired ring once: out-of-image rows and the fragment-padding
  // chunks must read as finite zeros (they meet zero weights)
  for (int o = tid * 16; o < kRing * kRowB; o += 512 * 16) *(uint4*)(ring + o) = make_uint4(0, 0, 0, 0);

  // paired chunk p of padded row pr from the raw ring (image row pr - 2,
  // columns 2p-2, 2p-1 = bytes 6p-6 .. 6p-1): the exact values preprocess_u8
  // would produce (imagenet_norm). Branch-free: two dword reads issued
  // together (a byte read per value, each under its own branch and wait,
  // was most of this kernel's time), the bytes picked by shifts, out-of-image
  // values selected to zero.
  auto convert_chunk = [&](int pr, int p) __attribute__((always_inline)) {
    const int iy = pr - 2;
    const bool row_in = iy >= 0 && iy < kS;
    const int pc = p < 1 ? 1 : p > kChunks - 2 ? kChunks - 2 : p;  // in-row address for the edge chunks
    const int start = 6 * pc - 6;                                  // byte offset, even
    const uint32_t* src = (const uint32_t*)(raw + (pr % kU8Ring) * kU8Slot + (start & ~3));
    const uint32_t d0 = src[0], d1 = src[1], d2 = src[2];
    // 64-bit window starting at the first wanted byte
    const uint64_t w = (start & 2) ? ((uint64_t)d2 << 48 | (uint64_t)d1 << 16 | (d0 >> 16))
                                   : ((uint64_t)d1 << 32 | d0);
    float v[8];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int ix = 2 * p - 2 + q;
      const bool in = row_in && ix >= 0 && ix < kS;
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const float raw_v = (float)(uint32_t)((w >> (8 * (3 * q + c))) & 0xffu);
        v[3 * q + c] = in ? imagenet_norm(c, raw_v) : 0.f;
      }
    }
    v[6] = v[7] = 0.f;
    *(uint4*)(ring + (pr & (kRing - 1)) * kRowB + p * 16) = pack8(v);
  };
  // raw image row of padded row pr -> raw ring (LDS-DMA, one wave, 42 lanes)
  auto dma_row = [&](int pr) __attribute__((always_inline)) {
    const int iy = pr - 2;
    if (iy < 0 || iy >= kS) return;
    if (lane < kU8B / 16) dma16(img + (long)iy * kU8B + lane * 16, raw + (pr % kU8Ring) * kU8Slot);
  };
  // (wave-uniform) does dma_row(pr) issue a load
  auto dma_issues = [](int pr) { return pr - 2 >= 0 && pr - 2 < kS; };

  // weights: wave's channel group 32 (w >> 2), n-blocks nf = 0, 1 (rows permuted)
  const int ch0 = 32 * (wave >> 2);
  bf16x8 wr[kKS][2];
#pragma unroll
  for (int nf = 0; nf < 2; ++nf) {
    const bf16* row = a.w + (long)(ch0 + perm32(16 * nf + fr)) * (kKS * 32);
#pragma unroll
    for (int ks = 0; ks < kKS; ++ks) wr[ks][nf] = *(const bf16x8*)(row + ks * 32 + fq * 8);
  }
  float bs[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) bs[e] = a.bias[ch0 + 8 * fq + e];

  // per-lane B-operand constants: chunk c = 4 ks + fq = (kh, cc); kh = 11
  // (the two pad chunks) reads row 10 (finite values x zero weights)
  const int f = wave & 3;
  const int ow = 16 * f + fr;
  int kh_of[kKS], col_of[kKS];
#pragma unroll
  for (int ks = 0; ks < kKS; ++ks) {
    const int c = 4 * ks + fq;
    const int kh = c / 6, cc = c - 6 * (c / 6);
    kh_of[ks] = kh < 11 ? kh : 10;
    col_of[ks] = (2 * ow + cc) * 16;
  }

  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __syncthreads();
  // prologue: raw rows of padded rows 0..22 (conv rows 0..3) by DMA into the
  // raw ring, converted here; then the raw rows of conv rows 4, 5 (padded
  // 23..30) and 6, 7 (31..38), one row per wave, converted at iterations 0
  // and 1 (31..38 reuse the slots of rows 0..6, converted by then)
  for (int pr = wave; pr < 23; pr += 8) dma_row(pr);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int it = tid; it < 23 * kChunks; it += 512) {
    const int pr = it / kChunks, p = it - pr * kChunks;
    convert_chunk(pr, p);
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __syncthreads();
  dma_row(23 + wave);
  dma_row(31 + wave);
  asm volatile("s_waitcnt vmcnt(1)" ::: "memory");  // conv rows 4, 5; 6, 7 may stay in flight
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __syncthreads();

  // iteration i: conv rows r0 = 2i, r0 + 1; pooled row i - 2
  for (int i = 0; i <= (kHo + 1) / 2; ++i) {
    const int r0 = 2 * i;
    // pooled row ph = i - 2 from conv rows 2ph .. 2ph+2 (written before the
    // last barrier; this iteration writes slots r0, r0+1, different ones).
    // First in the iteration: its global store is then older than this
    // iteration's DMA, so the closing vmcnt(1) does not wait for the DMA.
    const int ph = i - 2;
    if (ph >= 0 && ph < kPH && tid < kPH * 8) {
      const int pw = tid >> 3, cg = tid & 7;
      ushort8 m = ushort8{0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
      for (int dy = 0; dy < 3; ++dy) {
        const char* row = conv + ((2 * ph + dy) & (kConvRing - 1)) * kConvB;
#pragma unroll
        for (int dx = 0; dx < 3; ++dx)
          m = __builtin_elementwise_max(m, *(const ushort8*)(row + conv_off(2 * pw + dx, cg)));
      }
      *(ushort8*)(a.y + (((long)b * kPH + ph) * kPH + pw) * kC + cg * 8) = m;
    }
    // raw rows of conv rows r0+8, r0+9 (padded 4r0+39 .. 4r0+46, one per
    // wave; their raw ring slots were converted two iterations ago)
    const int dpr = 4 * r0 + 39 + wave;
    const bool dma_now = r0 + 8 + (wave >> 2) < kHo && dma_issues(dpr);
    if (dma_now) dma_row(dpr);
    // convert conv rows r0+4, r0+5's new rows (padded 4r0+23 .. 4r0+30; raw
    // rows landed before the last barrier); disjoint from the rows read below
    for (int it = tid; it < 8 * kChunks; it += 512) {
      const int q = it / kChunks, p = it - q * kChunks;
      const int pr = 4 * r0 + 23 + q;
      if (r0 + 4 + (q >> 2) < kHo) convert_chunk(pr, p);
    }
    // ---- conv rows r0, r0 + 1: 17 k-steps x 2 n-blocks each
#pragma unroll
    for (int rr = 0; rr < 2; ++rr) {
      const int oh = r0 + rr;
      if (oh < kHo) {
        floatx4 acc[2] = {floatx4{0.f, 0.f, 0.f, 0.f}, floatx4{0.f, 0.f, 0.f, 0.f}};
        const int pr0 = 4 * oh;
        // all 17 B operands issued up front (one read fed only 2 MFMAs)
        bf16x8 xb[kKS];
#pragma unroll
        for (int ks = 0; ks < kKS; ++ks)
          xb[ks] = *(const bf16x8*)(ring + ((pr0 + kh_of[ks]) & (kRing - 1)) * kRowB + col_of[ks]);
#pragma unroll
        for (int ks = 0; ks < kKS; ++ks) {
          acc[0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wr[ks][0], xb[ks], acc[0], 0, 0, 0);
          acc[1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wr[ks][1], xb[ks], acc[1], 0, 0, 0);
        }
        // lane: channels ch0 + 8 fq .. +7 of pixel ow (nf 0: +0..3, nf 1: +4..7)
        if (ow < kHo) {
          float v[8];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            v[e] = acc[0][e] + bs[e];
            v[4 + e] = acc[1][e] + bs[4 + e];
          }
          *(uint4*)(conv + (oh & (kConvRing - 1)) * kConvB + conv_off(ow, ch0 / 8 + fq)) = relu_bf16x8(pack8(v));
        }
      }
    }
    // the next iteration converts conv rows r0+6, r0+7 (DMA'd one iteration
    // ago, or in the prologue): in LDS before the barrier; this iteration's
    // DMA may stay in flight
    if (dma_now)
      asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __syncthreads();
  }
}

}  // namespace

size_t alex_stem_lds_bytes() { return kLds; }

bool alex_stem_supported(int S) { return S == kS; }

// K index of weight (kh, kw, c) in the paired-chunk order (544 per channel).
int alex_stem_k(int kh, int kw, int c) {
  const int cc = kw / 2, q = kw % 2;
  return (kh * 6 + cc) * 8 + q * 3 + c;
}

void alex_stem_u8(const uint8_t* x, const void* w, const float* bias, void* y, int B, hipStream_t s) {
  if (B <= 0) return;
  if (!x || !w || !bias || !y || ((uintptr_t)x & 15) || ((uintptr_t)w & 15) || ((uintptr_t)y & 15))
    throw std::invalid_argument("alex_stem_u8: null / misaligned operand");
  AlexStemArgs a;
  a.x = x;
  a.w = (const bf16*)w;
  a.bias = bias;
  a.y = (bf16*)y;
  hipLaunchKernelGGL(alex_stem_kernel, dim3(B), dim3(512), kLds, s, a);
  DMLC_HIP_CHECK(hipGetLastError());
}

}  // namespace dmlc
