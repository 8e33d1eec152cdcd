// Direct 3x3 / stride 1 / pad 1 convolution on the block-scaled e4m3 MFMA
// (v_mfma_scale_f32_16x16x128_f8f6f4, unit block scales), e4m3 in and out:
// ResNet50's bottleneck 3x3 convs of layer3 (14x14x256) and layer4
// (7x7x512), whose input t1 comes from the reduce 1x1 conv and whose output t2
// feeds the e4m3 expand conv (resnet50_fp8, EngineOptions::fp8_3x3_in).
//
// Reference equivalent: Bottleneck.conv2 + bn2 + relu of tch::vision::resnet50
// (BASELINE config 5: the model zoo path of src/services.rs:513-524, run per
// query by `forward_t` at :493). These convs are ~45% of ResNet50's FLOPs; on
// bf16 MFMA (conv3x3_stream.hip) they ran 51-54 us each at B = 256. Here the
// same structure runs at the e4m3 rate (a 16x16x128 MFMA = 2x the bf16 FLOPs
// per cycle) with half the staged bytes:
//
//  * a workgroup owns IMG whole images (resident in LDS, e4m3: 49 KB for a
//    14x14x256 image) and CO / NSP output channels; 8 waves (2 per SIMD) =
//    WM pixel groups x 8 / WM channel groups of 32 NG channels;
//  * every wave streams the fragment-order e4m3 weights of its channels from
//    L2 into a PD-deep register ring (no LDS stage, no barrier in the K loop);
//    a K-tile is one tap's 128 input channels (one MFMA k-step);
//  * D = W x X: lane (fr, fq) of an X fragment holds 32 consecutive input
//    channels of pixel fr (two 16-B LDS reads). A 16-B chunk pair of a
//    staged pixel sits at pair index m ^ (K & 7) (K = the staged pixel's
//    index, consecutive along a fragment), and lanes with odd fq read their
//    pair's second chunk first (their weight fragments are packed with the
//    same half swap, so the dot product is unchanged): in every 16-lane
//    group of a ds_read_b128 the 8 lanes of one fq read 8 distinct pairs and
//    the two fq take opposite halves, so the reads are bank-conflict free
//    (tests/test_layouts_cpu.py);
//  * epilogue: v = acc * alpha[n] + bias[n] (alpha = the per-channel e4m3
//    weight scale x the input scale; t2's per-channel output scales are
//    folded into both), ReLU, e4m3 (saturated at 448), 8 consecutive
//    channels of a pixel per 8-B store.
#include "common.h"
#include "kernels.h"

namespace dmlc {

namespace {

typedef int v8i __attribute__((ext_vector_type(8)));

struct Stream8Args {
  const uint8_t* x;     // [B, H, W, CI] e4m3
  const uint8_t* wf;    // e4m3 weights in stream8 fragment order (conv3x3_stream8_frag_offset)
  const float* alpha;   // [CO]: dequantisation of acc (input scale x weight scale)
  const float* bias;    // [CO]
  uint8_t* y;           // [B, H, W, CO] e4m3
  const uint8_t* zero;  // >= 16 zero bytes
  int B;
  int relu;
  float out_inv_scale;  // y = e4m3(relu(v) * out_inv_scale)
};

template <int H, int W, int CI, int IMG>
struct Stream8Geom {
  static constexpr int XR = IMG * H;          // staged rows
  static constexpr int PXB = CI;              // bytes per staged pixel
  static constexpr int ROWB = W * PXB;
  static constexpr int ZB = XR * ROWB;        // the zero pixel
  static constexpr int LDS = ZB + PXB;
  static constexpr int CH = XR * W * (CI / 16);  // 16-B chunks staged
};

template <int H, int W, int CI, int CO, int IMG, int NSP, int WM, int NG, int PD>
__global__ __launch_bounds__(512, 1) void conv3x3_stream8_kernel(Stream8Args a) {
  using G = Stream8Geom<H, W, CI, IMG>;
  constexpr int NPIX = IMG * H * W;          // output pixels per workgroup
  constexpr int MFT = (NPIX + 15) / 16;      // pixel fragments (the last one partly padding)
  constexpr int MF = (MFT + WM - 1) / WM;    // per wave
  constexpr int WN = 32 * NG;                // channels per wave
  constexpr int NF = 2 * NG;                 // N fragments per wave
  constexpr int CT = CI / 128;               // K-tiles per tap
  constexpr int KT = 9 * CT;                 // K-tiles
  constexpr int CPX = CI / 16;               // 16-B chunks per pixel
  static_assert(CO == 8 / WM * WN * NSP, "channel split");
  static_assert(CI % 128 == 0 && CPX >= 16, "e4m3 pixels of >= 256 B (whole bank rows)");
  static_assert(CT % PD == 0, "the ring slot of K-tile tap * CT + cc is cc % PD: compile-time register indices");
  static_assert(G::CH % 64 == 0, "whole DMA instructions");
  static_assert(G::LDS <= 160 * 1024, "LDS budget");

  extern __shared__ __attribute__((aligned(16))) uint4 smem[];
  char* xs = (char*)smem;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave % WM, wc = wave / WM;
  const int fr = lane & 15, fq = lane >> 4;
  const int ns = blockIdx.x % NSP, bg = blockIdx.x / NSP;
  const int b = bg * IMG, nimg = min(IMG, a.B - b);
  const int npix = nimg * H * W;
  const int ch0 = ns * (CO / NSP) + wc * WN;
  const uint8_t* img = a.x + (long)b * H * W * CI;

  // ---- stage the images (one flat run of 16-B chunks): logical chunk pair m
  // of staged pixel q (= its row * W + x, the key K) at physical pair
  // m ^ (q & 7), each chunk keeping its half
  const int nchunks = nimg * H * W * CPX;
  for (int k0 = wave * 64; k0 < G::CH; k0 += 512) {
    const int ci = k0 + lane;
    const int q = ci / CPX, pc = ci - q * CPX;  // staged pixel, physical chunk
    const int lc = ((((pc >> 1) ^ (q & 7)) << 1) | (pc & 1));  // logical chunk at physical pc
    const uint8_t* src = ci < nchunks ? img + (long)q * CI + 16 * lc : a.zero;
    dma16(src, xs + k0 * 16);
  }
  if (wave == 0 && lane < CPX) dma16(a.zero, xs + G::ZB);

  // ---- weights: fragment (group j, K-tile t, nf, half h) = 1 KB, lane l's
  // 16 B at l * 16 (conv3x3_stream8_frag_offset); this wave's NG groups are
  // consecutive
  const __amdgpu_buffer_rsrc_t wrs = wave_rsrc(a.wf + (long)(ch0 / 32) * KT * 4 * 1024, NG * KT * 4 * 1024);
  auto wfrag = [&](int t, int nf) __attribute__((always_inline)) {
    const int base = (((nf >> 1) * KT + t) * 2 + (nf & 1)) * 2 * 1024;
    const uint4 lo = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(wrs, lane * 16, base, 0));
    const uint4 hi = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(wrs, lane * 16, base + 1024, 0));
    return v8i{(int)lo.x, (int)lo.y, (int)lo.z, (int)lo.w, (int)hi.x, (int)hi.y, (int)hi.z, (int)hi.w};
  };
  v8i wq[PD][NF];
#pragma unroll
  for (int t = 0; t < PD - 1; ++t)
#pragma unroll
    for (int nf = 0; nf < NF; ++nf) wq[t][nf] = wfrag(t, nf);

  // ---- per-lane pixel constants: xoff = the staged offset of the tap-(1,1)
  // pixel | flags for the image's first / last row and column (their outside
  // taps read the zero pixel)
  int xoff[MF];
#pragma unroll
  for (int f = 0; f < MF; ++f) {
    const int p = min(16 * (wm * MF + f) + fr, npix - 1);
    const int pi = p % (H * W), ii = p / (H * W), prow = pi / W, pcol = pi - prow * W;
    xoff[f] = ((ii * H + prow) * W + pcol) * G::PXB | (prow == 0 ? 1 : 0) | (prow == H - 1 ? 2 : 0) |
              (pcol == 0 ? 4 : 0) | (pcol == W - 1 ? 8 : 0);
    asm volatile("" : "+v"(xoff[f]));
  }
  floatx4 acc[MF][NF];
#pragma unroll
  for (int f = 0; f < MF; ++f)
#pragma unroll
    for (int nf = 0; nf < NF; ++nf) acc[f][nf] = floatx4{0.f, 0.f, 0.f, 0.f};

  // tap (kh, kw): fragment bases xa[f]; lane offsets of the two reads: pair
  // ((fq + 4 cc) ^ (K & 7)) with K = p + ktap (p & 15 == fr for real pixels),
  // first the half fq & 1, then the other
  int xa[MF], tsw0 = 0, tsw1 = 0;
  auto set_tap = [&](int tap) __attribute__((always_inline)) {
    const int kh = tap / 3, kw = tap - kh * 3;
    const int tm = (kh == 0 ? 1 : 0) | (kh == 2 ? 2 : 0) | (kw == 0 ? 4 : 0) | (kw == 2 ? 8 : 0);
    const int toff = ((kh - 1) * W + (kw - 1)) * G::PXB;
#pragma unroll
    for (int f = 0; f < MF; ++f) xa[f] = (xoff[f] & tm) ? G::ZB : (xoff[f] & ~15) + toff;
    const int ktap = (kh - 1) * W + (kw - 1);
    const int u = fq ^ ((fr + ktap) & 7);
    tsw0 = (u << 5) | ((fq & 1) << 4);
    tsw1 = tsw0 ^ 16;
  };
  auto xread = [&](int f, int cc) __attribute__((always_inline)) {
    const uint4 lo = *(const uint4*)(xs + xa[f] + (tsw0 ^ (cc << 7)));
    const uint4 hi = *(const uint4*)(xs + xa[f] + (tsw1 ^ (cc << 7)));
    return v8i{(int)lo.x, (int)lo.y, (int)lo.z, (int)lo.w, (int)hi.x, (int)hi.y, (int)hi.z, (int)hi.w};
  };

  set_tap(0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // own input DMAs (and the first weights)
  __builtin_amdgcn_s_barrier();                     // everyone's
  asm volatile("" ::: "memory");
  v8i xf[MF];
#pragma unroll
  for (int f = 0; f < MF; ++f) xf[f] = xread(f, 0);
  for (int tap = 0; tap < 9; ++tap) {
#pragma unroll
    for (int cc = 0; cc < CT; ++cc) {
      const int t = tap * CT + cc;
      if (t + PD - 1 < KT)
#pragma unroll
        for (int nf = 0; nf < NF; ++nf) wq[(cc + PD - 1) % PD][nf] = wfrag(t + PD - 1, nf);
      if (cc + 1 == CT && tap + 1 < 9) set_tap(tap + 1);
      const int cn = cc + 1 == CT ? 0 : cc + 1;
      __builtin_amdgcn_s_waitcnt(0xC07F);  // the X fragments read during the previous K-tile
#pragma unroll
      for (int f = 0; f < MF; ++f) {
#pragma unroll
        for (int nf = 0; nf < NF; ++nf)
          acc[f][nf] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(wq[cc % PD][nf], xf[f], acc[f][nf], 0, 0, 0,
                                                                         127, 0, 127);
        if (t + 1 < KT) xf[f] = xread(f, cn);
      }
#pragma unroll
      for (int f = 0; f < MF; ++f) {
        __builtin_amdgcn_sched_group_barrier(0x008, NF, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
      }
    }
  }

  // every MFMA done here: pinned, the compiler cannot sink the last K-tile's
  // MFMA chains into the pixel-conditional stores below (their operands then
  // stay live across the whole epilogue and spill)
#pragma unroll
  for (int f = 0; f < MF; ++f)
#pragma unroll
    for (int nf = 0; nf < NF; ++nf) asm volatile("" : "+v"(acc[f][nf]));
  // ---- epilogue: lane holds channels ch0 + 32 j + 8 fq .. +7 of its pixel
  float al[NG][8], bs[NG][8];
#pragma unroll
  for (int j = 0; j < NG; ++j)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      al[j][e] = a.alpha[ch0 + 32 * j + 8 * fq + e];
      bs[j][e] = a.bias[ch0 + 32 * j + 8 * fq + e];
    }
  const float inv = a.out_inv_scale;
  const long base = (long)b * H * W * CO + ch0 + 8 * fq;
#pragma unroll
  for (int f = 0; f < MF; ++f) {
    const int p = 16 * (wm * MF + f) + fr;
    if (p >= npix) continue;
#pragma unroll
    for (int j = 0; j < NG; ++j) {
      float q[8];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        q[e] = acc[f][2 * j][e] * al[j][e] + bs[j][e];
        q[4 + e] = acc[f][2 * j + 1][e] * al[j][4 + e] + bs[j][4 + e];
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) q[e] = __builtin_amdgcn_fmed3f((a.relu ? fmaxf(q[e], 0.f) : q[e]) * inv, -448.f, 448.f);
      int lo = __builtin_amdgcn_cvt_pk_fp8_f32(q[0], q[1], 0, false);
      lo = __builtin_amdgcn_cvt_pk_fp8_f32(q[2], q[3], lo, true);
      int hi = __builtin_amdgcn_cvt_pk_fp8_f32(q[4], q[5], 0, false);
      hi = __builtin_amdgcn_cvt_pk_fp8_f32(q[6], q[7], hi, true);
      *(uint2*)(a.y + base + 32 * j + (long)p * CO) = make_uint2((uint32_t)lo, (uint32_t)hi);
    }
  }
}

template <int H, int W, int CI, int CO, int IMG, int NSP, int WM, int NG, int PD>
void launch8(const Stream8Args& a, hipStream_t s) {
  using G = Stream8Geom<H, W, CI, IMG>;
  const int grid = (a.B + IMG - 1) / IMG * NSP;
  hipLaunchKernelGGL((conv3x3_stream8_kernel<H, W, CI, CO, IMG, NSP, WM, NG, PD>), dim3(grid), dim3(512),
                     (size_t)G::LDS, s, a);
}

int g_stream8_variant = 0;

}  // namespace

void conv3x3_stream8_set_variant(int v) { g_stream8_variant = v; }

bool conv3x3_stream8_supported(int Hin, int Win, int Cin, int Cout) {
  return Cin == Cout && ((Hin == 14 && Win == 14 && Cin == 256) || (Hin == 7 && Win == 7 && Cin == 512));
}

// Byte offset of the 16 weight bytes lane `lane` loads for (32-channel group
// j, K-tile t, N fragment nf, half h): the bytes are W8[32 j + perm32(16 nf +
// (lane & 15))][128 t + 32 fq + 16 (h ^ (fq & 1)) + 0..15], fq = lane >> 4
// (perm32 as in conv3x3_stream.hip: row 16 nf + r of a group holds channel
// 8 (r >> 2) + 4 nf + (r & 3)).
size_t conv3x3_stream8_frag_offset(int j, int t, int nf, int h, int lane, int KT) {
  return (((((size_t)j * KT + t) * 2 + nf) * 2 + h) * 64 + lane) * 16;
}

void conv3x3_stream8(const void* x, const void* wf, const float* alpha, const float* bias, void* y, const void* zero,
                     int B, int Hin, int Win, int Cin, int Cout, bool relu, float out_inv_scale, hipStream_t s) {
  if (B <= 0) return;
  if (!conv3x3_stream8_supported(Hin, Win, Cin, Cout)) throw std::invalid_argument("conv3x3_stream8: unsupported shape");
  if (!x || !wf || !alpha || !bias || !y || !zero || (((uintptr_t)x | (uintptr_t)wf | (uintptr_t)zero) & 15) ||
      ((uintptr_t)y & 7) || !(out_inv_scale > 0.f))
    throw std::invalid_argument("conv3x3_stream8: null / misaligned operand or no output scale");
  if (x == y) throw std::invalid_argument("conv3x3_stream8: in-place not supported");
  Stream8Args a;
  a.x = (const uint8_t*)x;
  a.wf = (const uint8_t*)wf;
  a.alpha = alpha;
  a.bias = bias;
  a.y = (uint8_t*)y;
  a.zero = (const uint8_t*)zero;
  a.B = B;
  a.relu = relu;
  a.out_inv_scale = out_inv_scale;
  const int v = g_stream8_variant;
  if (Cin == 256) {
    // layer3: one image x half the channels per workgroup (2 pixel halves x 4
    // groups of 32; 188 VGPRs). All 256 channels per workgroup (4 groups of
    // 64 per wave) spills at any ring depth.
    launch8<14, 14, 256, 256, 1, 2, 2, 1, 2>(a, s);
  } else {  // layer4: two images x half the channels, 8 groups of 32 (variant bit 2: a 2-deep weight ring)
    if (v & 2)
      launch8<7, 7, 512, 512, 2, 2, 1, 1, 2>(a, s);
    else
      launch8<7, 7, 512, 512, 2, 2, 1, 1, 4>(a, s);
  }
  DMLC_HIP_CHECK(hipGetLastError());
}

}  // namespace dmlc
