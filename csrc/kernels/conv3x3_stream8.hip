// Direct 3x3 / stride 1 / pad 1 convolution on the block-scaled e4m3 MFMA
// (v_mfma_scale_f32_16x16x128_f8f6f4, unit block scales), e4m3 in and out:
// ResNet50's bottleneck 3x3 convs of layer2 (28x28x128), layer3 (14x14x256)
// and layer4 (7x7x512), whose input t1 comes from the reduce 1x1 conv and
// whose output t2 feeds the e4m3 expand conv (resnet50_fp8,
// EngineOptions::fp8_3x3_in).
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
//    (tests/test_layouts_cpu.py). 128-channel pixels (128 B, half a bank
//    row) key the pair by (K >> 1) & 3 instead: K's parity picks the window
//    half, and the 8 lanes of one fq (4 + 4 consecutive K, or 8) cover the 8
//    values of K & 7 once;
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
  int stagger;          // start_stagger (common.h)
};

// Geometry: output H x W, stride S; a workgroup owns HS output rows of one
// image (PARTS = H / HS > 1: stride 2, or two halves at stride 1) or IMG
// whole images.
template <int H, int W, int CI, int HS, int IMG, int S>
struct Stream8Geom {
  static constexpr int PARTS = H / HS;
  static_assert(PARTS == 1 || IMG == 1, "strips: one image");
  static constexpr int HI = S * H, WI = S * W;   // input rows / columns
  // staged rows: whole images, the strip's input rows 2 r0 - 1 .. 2 (r0 +
  // HS - 1) + 1 (stride 2 never reads below the image), or a strip and its
  // halo rows inside the image (stride 1)
  static constexpr int XR = PARTS == 1 ? IMG * HI
                            : S == 1   ? HS + (PARTS > 2 ? 2 : 1)
                                       : (S * (HS - 1) + 3 < HI ? S * (HS - 1) + 3 : HI);
  static constexpr int PXB = CI;                 // bytes per staged pixel
  static constexpr int ROWB = WI * PXB;
  static constexpr int ZB = XR * ROWB;           // the zero pixel
  // (128-B pixels: two zero pixels, the window half a real pixel of the same
  // K parity would use, so border lanes keep their bank slots)
  static constexpr int ZBYTES = PXB >= 256 ? PXB : 256;
  static constexpr int LDS = ZB + ZBYTES;
  static constexpr int CH = XR * WI * (CI / 16);  // 16-B chunks staged (at most)
};

template <int H, int W, int CI, int CO, int HS, int IMG, int NSP, int WM, int NG, int PD, int S>
__global__ __launch_bounds__(512, 1) void conv3x3_stream8_kernel(Stream8Args a) {
  using G = Stream8Geom<H, W, CI, HS, IMG, S>;
  constexpr int PARTS = G::PARTS, HI = G::HI, WI = G::WI;
  constexpr int NPIX = IMG * HS * W;         // output pixels per workgroup
  constexpr int MFT = (NPIX + 15) / 16;      // pixel fragments (the last one partly padding)
  constexpr int MF = (MFT + WM - 1) / WM;    // per wave
  constexpr int WN = 32 * NG;                // channels per wave
  constexpr int NF = 2 * NG;                 // N fragments per wave
  constexpr int CT = CI / 128;               // K-tiles per tap
  constexpr int KT = 9 * CT;                 // K-tiles
  constexpr int CPX = CI / 16;               // 16-B chunks per pixel
  static_assert(CO == 8 / WM * WN * NSP, "channel split");
  static_assert(CI % 128 == 0 && (CPX >= 16 || CPX == 8), "e4m3 pixels of 128 B or >= 256 B (whole bank rows)");
  // ring slot of K-tile t = tap * CT + cc: cc % PD (tap loop rolled), or t % PD
  // (CT = 1: the 9 taps unrolled): compile-time register indices either way
  static_assert(CT == 1 || CT % PD == 0, "weight ring depth");
  static_assert(G::LDS <= 160 * 1024, "LDS budget");
  static_assert(S == 1 || (S == 2 && WI % 2 == 0), "stride");

  extern __shared__ __attribute__((aligned(16))) uint4 smem[];
  char* xs = (char*)smem;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  start_stagger(a.stagger);
  const int wm = wave % WM, wc = wave / WM;
  const int fr = lane & 15, fq = lane >> 4;
  const int ns = blockIdx.x % NSP, rest = blockIdx.x / NSP;
  const int bg = rest / PARTS, part = rest - bg * PARTS;
  const int b = bg * IMG, nimg = min(IMG, a.B - b);
  const int r0 = part * HS;                                  // first output row
  const int rs = PARTS == 1 ? 0 : max(S * r0 - 1, 0);        // first staged input row
  const int nrows = PARTS == 1 ? nimg * HI : min(S * (r0 + HS - 1) + 1, HI - 1) - rs + 1;
  const int npix = IMG == 1 ? NPIX : nimg * HS * W;
  const int ch0 = ns * (CO / NSP) + wc * WN;
  const uint8_t* img = a.x + (long)b * HI * WI * CI;
  // chunk-pair key of staged pixel K (see the header)
  auto pswz = [](int k) __attribute__((always_inline)) { return CPX >= 16 ? (k & 7) : ((k >> 1) & 3); };

  // ---- stage the input rows (one flat run of 16-B chunks; stride 2: each
  // row's even columns first, then its odd ones). The key K of a staged
  // pixel is chosen so that for output pixel p at tap (kh, kw) it is p + a
  // tap constant, consecutive along a fragment even where it wraps a row:
  //   stride 1 (whole images): K = staged row * W + x;
  //   stride 2: K = image * H * W + (((y + 1) >> 1) - r0) * W + ((x + 1) >> 1).
  // Logical chunk pair m of a staged pixel sits at physical pair m ^ (K & 7),
  // each chunk keeping its half.
  for (int k0 = wave * 64; k0 < G::CH; k0 += 512) {
    const int ci = k0 + lane;
    const int i = ci / (WI * CPX), rem = ci - i * (WI * CPX);
    const int q = rem / CPX, pc = rem - q * CPX;  // physical column, chunk
    const int x = S == 1 ? q : (q < WI / 2 ? 2 * q : 2 * (q - WI / 2) + 1);
    int K;
    if constexpr (S == 1) {
      K = i * W + x;
    } else {
      const int ii = PARTS == 1 ? i / HI : 0, y = PARTS == 1 ? i - ii * HI : rs + i;
      K = ii * (H * W) + (((y + 1) >> 1) - r0) * W + ((x + 1) >> 1);
    }
    const int lc = ((((pc >> 1) ^ pswz(K)) << 1) | (pc & 1));  // logical chunk at physical pc
    const uint8_t* src = i < nrows ? img + ((long)(rs + i) * WI + x) * CI + 16 * lc : a.zero;
    if (G::CH % 64 == 0 || ci < G::CH) dma16(src, xs + k0 * 16);
  }
  if (wave == 0 && lane < G::ZBYTES / 16) dma16(a.zero, xs + G::ZB);

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
  // input pixel | flags for the image's first / last row and column (their
  // outside taps read the zero pixel; stride 2 never leaves the image at the
  // bottom or right)
  int xoff[MF];
#pragma unroll
  for (int f = 0; f < MF; ++f) {
    const int p = min(16 * (wm * MF + f) + fr, npix - 1);
    const int pi = p % (HS * W), ii = p / (HS * W), prow = pi / W, pcol = pi - prow * W, r = r0 + prow;
    const int row = ii * HI + S * r - rs;  // (stride 2: even input column 2 pcol sits at slot pcol)
    xoff[f] = (row * WI + pcol) * G::PXB | (r == 0 ? 1 : 0) | (S == 1 && r == H - 1 ? 2 : 0) | (pcol == 0 ? 4 : 0) |
              (S == 1 && pcol == W - 1 ? 8 : 0);
    asm volatile("" : "+v"(xoff[f]));
  }
  floatx4 acc[MF][NF];
#pragma unroll
  for (int f = 0; f < MF; ++f)
#pragma unroll
    for (int nf = 0; nf < NF; ++nf) acc[f][nf] = floatx4{0.f, 0.f, 0.f, 0.f};

  // tap (kh, kw): fragment bases xa[f]; lane offsets of the two reads: pair
  // ((fq + 4 cc) ^ pswz(K)) with K = p + kb + ktap (p & 15 == fr for real
  // pixels; kb: a stride-1 half image's staged rows start r0 - rs rows above
  // its first output row), first the half fq & 1, then the other
  const int kb = S == 1 ? (r0 - rs) * W : 0;
  int xa[MF], tsw0 = 0, tsw1 = 0;
  auto set_tap = [&](int tap) __attribute__((always_inline)) {
    const int kh = tap / 3, kw = tap - kh * 3;
    const int tm = (kh == 0 ? 1 : 0) | (kh == 2 ? 2 : 0) | (kw == 0 ? 4 : 0) | (kw == 2 ? 8 : 0);
    // staged column offset of tap column kw (stride 2: odd columns start at WI / 2)
    const int dq = S == 1 ? kw - 1 : (kw == 0 ? WI / 2 - 1 : kw == 1 ? 0 : WI / 2);
    const int toff = ((kh - 1) * WI + dq) * G::PXB;
    const int ktap = S == 1 ? (kh - 1) * W + (kw - 1) : (kh == 2 ? W : 0) + (kw == 2 ? 1 : 0);
    // 128-B pixels: a real pixel's window half is its staged column's parity,
    // K's parity (stride 2: flipped for kw != 1, the odd columns staged after
    // the even ones); border lanes read the zero pixel in that half, so they
    // keep the bank slots the swizzle gives their K
    const int zh = CPX >= 16 ? 0 : (((fr + kb + ktap) & 1) ^ (S == 2 && kw != 1 ? 1 : 0));
#pragma unroll
    for (int f = 0; f < MF; ++f) xa[f] = (xoff[f] & tm) ? G::ZB + zh * 128 : (xoff[f] & ~15) + toff;
    const int u = fq ^ pswz(fr + kb + ktap);
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
  // K-tile t = tap * CT + cc, its weights in ring slot `slot`
  auto ktile = [&](const int tap, const int cc, const int slot) __attribute__((always_inline)) {
    const int t = tap * CT + cc;
    if (t + PD - 1 < KT)
#pragma unroll
      for (int nf = 0; nf < NF; ++nf) wq[(slot + PD - 1) % PD][nf] = wfrag(t + PD - 1, nf);
    if (cc + 1 == CT && tap + 1 < 9) set_tap(tap + 1);
    const int cn = cc + 1 == CT ? 0 : cc + 1;
    __builtin_amdgcn_s_waitcnt(0xC07F);  // the X fragments read during the previous K-tile
#pragma unroll
    for (int f = 0; f < MF; ++f) {
#pragma unroll
      for (int nf = 0; nf < NF; ++nf)
        acc[f][nf] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(wq[slot][nf], xf[f], acc[f][nf], 0, 0, 0, 127,
                                                                       0, 127);
      if (t + 1 < KT) xf[f] = xread(f, cn);
    }
#pragma unroll
    for (int f = 0; f < MF; ++f) {
      __builtin_amdgcn_sched_group_barrier(0x008, NF, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
    }
  };
  if constexpr (CT == 1) {
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) ktile(tap, 0, tap % PD);
  } else {
    for (int tap = 0; tap < 9; ++tap)
#pragma unroll
      for (int cc = 0; cc < CT; ++cc) ktile(tap, cc, cc % PD);
  }

  // every MFMA done here: pinned, the compiler cannot sink the last K-tile's
  // MFMA chains into the pixel-conditional stores below (their operands then
  // stay live across the whole epilogue and spill)
#pragma unroll
  for (int f = 0; f < MF; ++f)
#pragma unroll
    for (int nf = 0; nf < NF; ++nf) asm volatile("" : "+v"(acc[f][nf]));
  // ---- epilogue: lane holds channels ch0 + 32 j + 8 fq .. +7 of its pixel.
  // The 1 / s_out quantisation scale (> 0) is folded into alpha and the bias,
  // so a value costs half a v_pk_fma_f32 (channel pairs sit in consecutive
  // accumulator registers) and one med3 (ReLU and the +-448 saturation
  // together)
  const float inv = a.out_inv_scale;
  const float lo_clamp = a.relu ? 0.f : -448.f;
  f32x2 al[NG][4], bs[NG][4];
#pragma unroll
  for (int j = 0; j < NG; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int c = ch0 + 32 * j + 8 * fq + 2 * e;
      al[j][e] = f32x2{a.alpha[c], a.alpha[c + 1]} * inv;
      bs[j][e] = f32x2{a.bias[c], a.bias[c + 1]} * inv;
    }
  const long base = ((long)b * H + r0) * W * CO + ch0 + 8 * fq;
#pragma unroll
  for (int f = 0; f < MF; ++f) {
    const int p = 16 * (wm * MF + f) + fr;
    if (p >= npix) continue;
#pragma unroll
    for (int j = 0; j < NG; ++j) {
      float q[8];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const floatx4& ac = acc[f][2 * j + (e >> 1)];
        const f32x2 r = __builtin_elementwise_fma(f32x2{ac[2 * (e & 1)], ac[2 * (e & 1) + 1]}, al[j][e], bs[j][e]);
        q[2 * e] = r.x;
        q[2 * e + 1] = r.y;
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) q[e] = __builtin_amdgcn_fmed3f(q[e], lo_clamp, 448.f);
      int lo = __builtin_amdgcn_cvt_pk_fp8_f32(q[0], q[1], 0, false);
      lo = __builtin_amdgcn_cvt_pk_fp8_f32(q[2], q[3], lo, true);
      int hi = __builtin_amdgcn_cvt_pk_fp8_f32(q[4], q[5], 0, false);
      hi = __builtin_amdgcn_cvt_pk_fp8_f32(q[6], q[7], hi, true);
      *(uint2*)(a.y + base + 32 * j + (long)p * CO) = make_uint2((uint32_t)lo, (uint32_t)hi);
    }
  }
}

template <int H, int W, int CI, int CO, int HS, int IMG, int NSP, int WM, int NG, int PD, int S>
void launch8(const Stream8Args& a, hipStream_t s) {
  using G = Stream8Geom<H, W, CI, HS, IMG, S>;
  const int grid = (a.B + IMG - 1) / IMG * (H / HS) * NSP;
  hipLaunchKernelGGL((conv3x3_stream8_kernel<H, W, CI, CO, HS, IMG, NSP, WM, NG, PD, S>), dim3(grid), dim3(512),
                     (size_t)G::LDS, s, a);
}

int g_stream8_variant = 0;

}  // namespace

void conv3x3_stream8_set_variant(int v) { g_stream8_variant = v; }

bool conv3x3_stream8_supported(int Hin, int Win, int Cin, int Cout, int stride) {
  if (Cin != Cout) return false;
  if (stride == 1)
    return (Hin == 28 && Win == 28 && Cin == 128) || (Hin == 14 && Win == 14 && Cin == 256) ||
           (Hin == 7 && Win == 7 && Cin == 512);
  // ResNet50 layer2.0 / layer3.0 / layer4.0 conv2 (the bottleneck's strided 3x3)
  if (stride == 2)
    return (Hin == 56 && Win == 56 && Cin == 128) || (Hin == 28 && Win == 28 && Cin == 256) ||
           (Hin == 14 && Win == 14 && Cin == 512);
  return false;
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
                     int B, int Hin, int Win, int Cin, int Cout, int stride, bool relu, float out_inv_scale,
                     hipStream_t s) {
  if (B <= 0) return;
  if (!conv3x3_stream8_supported(Hin, Win, Cin, Cout, stride))
    throw std::invalid_argument("conv3x3_stream8: unsupported shape");
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
  a.stagger = kernel_stagger(kStagStream8);
  const int v = g_stream8_variant;
  if (stride == 2 && Cin == 128) {
    // layer2.0.conv2 (56x56x128 -> 28x28): 4 output rows (9 staged rows of
    // 128-B pixels = 63 KB; 104 VGPRs: two workgroups per CU, one's staging
    // under the other's MFMAs) x all 128 channels, 4 pixel quarters x 2 groups
    // of 64. Variant 4: 7-row strips (105 KB, 164 VGPRs, one per CU):
    // 1927 vs 1923 us per resnet50_fp8 b256 forward (profiles/r5_stream8_layer2.txt)
    if (v & 4)
      launch8<28, 28, 128, 128, 7, 1, 1, 4, 2, 2, 2>(a, s);
    else
      launch8<28, 28, 128, 128, 4, 1, 1, 4, 2, 2, 2>(a, s);
  } else if (stride == 2 && Cin == 256) {
    // layer3.0.conv2 (28x28x256 -> 14x14): half an image (7 output rows, 15
    // staged rows = 105 KB) x all 256 channels, 8 groups of 32
    launch8<14, 14, 256, 256, 7, 1, 1, 1, 1, 2, 2>(a, s);
  } else if (stride == 2) {
    // layer4.0.conv2 (14x14x512 -> 7x7): one image (98 KB) x half the channels
    launch8<7, 7, 512, 512, 7, 1, 2, 1, 1, 2, 2>(a, s);
  } else if (Cin == 128) {
    // layer2 (28x28x128): half an image (14 output rows + a halo row, 54 KB)
    // x all 128 channels, 4 pixel quarters x 2 groups of 64 (the whole image,
    // 100 KB, per workgroup would stage it once per channel half)
    // (4-row strips, 108 VGPRs, two workgroups per CU: 1955 vs 1927 us per
    // resnet50_fp8 b256 forward, profiles/r5_stream8_layer2.txt)
    launch8<28, 28, 128, 128, 14, 1, 1, 4, 2, 2, 1>(a, s);
  } else if (Cin == 256) {
    // layer3: one image x half the channels per workgroup (2 pixel halves x 4
    // groups of 32; 188 VGPRs). All 256 channels per workgroup (4 groups of
    // 64 per wave) spills at any ring depth.
    launch8<14, 14, 256, 256, 14, 1, 2, 2, 1, 2, 1>(a, s);
  } else {  // layer4: two images x half the channels, 8 groups of 32
    launch8<7, 7, 512, 512, 7, 2, 2, 1, 1, 4, 1>(a, s);
  }
  DMLC_HIP_CHECK(hipGetLastError());
}

}  // namespace dmlc
