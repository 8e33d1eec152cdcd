// Direct 3x3 / stride 1 / pad 1 convolution for narrow layers (ResNet
// layer1: 56x56x64 -> 64), BN folded, optional residual, ReLU.
//
// Reference equivalent: layer1.{0,1}.conv{1,2} + bn + (residual) + relu of
// tch::vision::resnet18, run per query by `forward_t` at src/services.rs:493.
// As an implicit GEMM (conv_igemm.hip) each 256x64 output tile re-fetches its
// 3x3 input window for every tap: ~9x the input bytes through L2 into LDS
// per conv, which makes these four convs L2-bandwidth bound (~440 TF). Here
// one workgroup walks one image (or a strip of it) top to bottom:
//
//  * The folded weights (64 x 576 bf16 = 72 KB) are resident in LDS for the
//    whole workgroup.
//  * Input rows go HBM -> LDS once, by LDS-DMA into a 10-row ring with zero
//    pad columns (and zero rows above/below the image) supplied from a zero
//    page. A step computes 4 output rows (224 pixels) from 6 ring rows while
//    the 4 rows of the next step are in flight.
//  * 4 waves = 2 pixel halves (7 fragments of 16 pixels) x 2 channel halves
//    (2 fragments of 16 channels); per 32-wide K step a wave reads 2 weight
//    and 7 input fragments (one ds_read_b128 each) for 14 MFMAs. D = W x X,
//    so a lane ends with 4 consecutive channels of one pixel.
//  * Bank conflicts: ds_read_b128 is serviced in four 16-lane groups
//    ({0-3,12-15,20-27}, {4-11,16-19,28-31}, +32), each needing 16 distinct
//    16-B bank groups (MI355X_MICROARCH.md §LDS). Input chunks are XOR-
//    swizzled by (column & 7) and weight chunks by 2*((n >> 3) & 1); both
//    make every group conflict-free (checked exhaustively for all fragments,
//    taps and channel halves; tests/test_layouts_cpu.py).
#include "common.h"
#include "kernels.h"

namespace dmlc {

namespace {

template <int N>
__device__ __forceinline__ void vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}

// weight-chunk swizzle for output channel n (only bit 3 of n matters; the
// wave's channel offsets are multiples of 16)
__device__ __forceinline__ int wswz(int n) { return ((n >> 3) & 1) << 1; }

struct RowConvArgs {
  const bf16* x;      // [B, H, W, C]
  const bf16* w;      // [C, 9*C], k = (kh*3 + kw)*C + c
  const float* bias;  // [C]
  const bf16* res;    // [B, H, W, C] or null
  bf16* y;            // [B, H, W, C]
  const bf16* zero;   // >= 16 zero bytes
  const bf16* wf;     // WR: weights in stream-conv fragment order [C/32][KS][2][64][8] (kernels.h)
  int H, strip;       // strip = output rows per workgroup (multiple of 4)
  int relu;
};

// WR: the weights are not resident in LDS; every wave streams its fragments
// from L2 (fragment order, 1 KB coalesced per fragment) through a PD-deep
// register ring, so the workgroup needs only the input ring (74 KB) and two
// fit per CU (2 waves per SIMD instead of 1).
template <int W, int C, bool WR>
__global__ __launch_bounds__(256, WR ? 2 : 1) void conv3x3_rows_kernel(RowConvArgs a) {
  static_assert(C == 64, "layout below assumes 64 channels (8 chunks per pixel)");
  constexpr int R = 4;                // output rows per step
  constexpr int MF = R * W / 32;      // pixel fragments per wave (2 pixel halves)
  static_assert(R * W % 32 == 0, "pixels per step must split into 2 x 16k");
  constexpr int KS = 9 * C / 32;      // K steps
  constexpr int Q = W + 2;            // staged columns (zero pads at 0 and W+1)
  constexpr int SLOT = Q * C * 2;     // bytes per staged input row
  constexpr int RING = 10;            // 6 rows for a step + 4 in flight
  constexpr int WB = 9 * C * C * 2;   // weight bytes
  constexpr int ROW_CH = Q * C / 8;   // 16-B chunks per staged row

  extern __shared__ __attribute__((aligned(16))) uint4 smem[];
  char* wl = (char*)smem;
  char* ring = wl + (WR ? 0 : WB);
  constexpr int PD = 3;  // register ring depth (divides KS: the ring is periodic across steps)
  static_assert(!WR || KS % PD == 0, "PD | KS");

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave & 1, wn = wave >> 1;
  const int fr = lane & 15, g = lane >> 4;
  const int strips = a.H / a.strip;
  const int b = blockIdx.x / strips;
  const int oh_first = (blockIdx.x - b * strips) * a.strip;
  const int steps = a.strip / R;
  const bf16* img = a.x + (long)b * a.H * W * C;

  // ---- weights -> LDS: chunk i = (ks*C + n)*4 + c' holds w[perm(n)][ks*32 + 8*(c' ^ wswz(n))].
  // perm maps LDS weight row n = 32*wg + 16*nf + r (the MFMA row r of N
  // fragment nf) to output channel 32*wg + 8*(r>>2) + 4*nf + (r&3): the lane
  // with accumulator rows 4g..4g+3 of both fragments then holds the 8
  // consecutive channels 32*wg + 8g .. +7 (16-B output stores and residual
  // loads instead of two 8-B halves).
  auto perm = [](int n) { return (n & ~31) + 8 * ((n & 15) >> 2) + 4 * ((n >> 4) & 1) + (n & 3); };
  for (int j = 0; j < (WR ? 0 : WB / 16 / 256); ++j) {
    const int i = j * 256 + tid;
    const int c2 = i & 3, n = (i >> 2) % C, ks = i / (4 * C);
    const bf16* src = a.w + (long)perm(n) * (9 * C) + ks * 32 + 8 * (c2 ^ wswz(n));
    dma16(src, (wl + (j * 256 + wave * 64) * 16));
  }

  // ---- one input row (r may be -1 or H: zero row) -> ring slot
  // chunk i = q*8 + c' holds x[r][q-1][8*(c' ^ (q & 7))], zeros at q = 0, W+1.
  auto load_row = [&](int r, int part, int nparts) __attribute__((always_inline)) {
    char* dst = ring + ((r + RING) % RING) * SLOT;
    const bool inside = (unsigned)r < (unsigned)a.H;
    for (int c0 = part * 64; c0 < ROW_CH; c0 += nparts * 64) {
      const int i = c0 + lane;
      const int q = i >> 3, c2 = i & 7;
      const bool ok = inside && q >= 1 && q <= W;
      const bf16* src = ok ? img + ((long)r * W + (q - 1)) * C + 8 * (c2 ^ (q & 7)) : a.zero;
      if (i < ROW_CH)
        dma16(src, (dst + c0 * 16));
    }
  };
  // Rows [lo, lo+n) spread over the 4 waves (each row = ROW_CH/64 instructions).
  auto load_rows = [&](int lo, int n) __attribute__((always_inline)) {
    for (int k = 0; k < n; ++k) load_row(lo + k, wave, 4);
  };

  load_rows(oh_first - 1, 6);
  vm_wait<0>();
  __builtin_amdgcn_s_barrier();

  // ---- per-lane constants
  // pixel of fragment f: p = wm*(R*W/2) + 16f + fr within the step's R x W tile
  int prow[MF], colq[MF][3][2];
#pragma unroll
  for (int f = 0; f < MF; ++f) {
    const int p = wm * (R * W / 2) + 16 * f + fr;
    prow[f] = p / W;
    const int col = p % W;
#pragma unroll
    for (int kw = 0; kw < 3; ++kw) {
      const int q = col + kw;  // staged column of input col-1+kw
#pragma unroll
      for (int h = 0; h < 2; ++h) colq[f][kw][h] = q * (C * 2) + (((4 * h + g) ^ (q & 7)) << 4);
    }
  }
  // weight fragment nf of this wave: rows n = wn*32 + 16nf + fr
  const uint32_t wrow = (uint32_t)(wn * 32 + fr) * 64 + ((g ^ wswz(fr)) << 4);
  const char* wbase = wl + wrow;
  // WR: fragment nf of K step ks for this wave's channel group wn
  // (buffer loads: lane offset in a VGPR, the fragment offset a scalar constant)
  const __amdgpu_buffer_rsrc_t wrs = wave_rsrc(a.wf + (long)wn * KS * 2 * 64 * 8, KS * 2 * 1024);
  auto wload = [&](int kf) __attribute__((always_inline)) {
    return __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(wrs, lane * 16, kf * 1024, 0));
  };
  bf16x8 wq[WR ? PD : 1][2];
  if constexpr (WR) {
#pragma unroll
    for (int ks = 0; ks < PD - 1; ++ks)
#pragma unroll
      for (int nf = 0; nf < 2; ++nf) wq[ks][nf] = wload(ks * 2 + nf);
  }
  // this lane's 8 output channels (see perm): bias of channel wn*32 + 8g + 4nf + i
  float bs[2][4];
#pragma unroll
  for (int nf = 0; nf < 2; ++nf)
#pragma unroll
    for (int i = 0; i < 4; ++i) bs[nf][i] = a.bias[wn * 32 + 8 * g + 4 * nf + i];

  for (int s = 0; s < steps; ++s) {
    const int oh0 = oh_first + s * R;
    if (s + 1 < steps) load_rows(oh0 + R + 1, R);  // the next step's new rows: oh0+5 .. oh0+8

    // ring row offsets for (fragment, kh): input row oh0 + prow + kh - 1
    int roff[MF][3];
#pragma unroll
    for (int f = 0; f < MF; ++f)
#pragma unroll
      for (int kh = 0; kh < 3; ++kh) roff[f][kh] = ((oh0 + prow[f] + kh - 1 + RING) % RING) * SLOT;

    // residual of this step's outputs, loaded now so it lands during the MFMAs
    const long base = ((long)b * a.H + oh0) * W * C;
    uint4 rres[MF];
#pragma unroll
    for (int f = 0; f < MF; ++f) {
      const int p = wm * (R * W / 2) + 16 * f + fr;
      rres[f] = a.res ? *(const uint4*)(a.res + base + (long)p * C + wn * 32 + 8 * g) : make_uint4(0, 0, 0, 0);
    }

    floatx4 acc[MF][2];
#pragma unroll
    for (int f = 0; f < MF; ++f)
#pragma unroll
      for (int nf = 0; nf < 2; ++nf) acc[f][nf] = floatx4{0.f, 0.f, 0.f, 0.f};

    // Fragments of K step ks+1 are read before ks's MFMAs issue (sched_barrier
    // pins the order; left alone the scheduler sinks each read next to its
    // first use and every MFMA group waits on LDS latency).
    bf16x8 wc[2], xc[MF], wn2[2], xn[MF];
    auto load_k = [&](int ks, bf16x8* wd, bf16x8* xd) __attribute__((always_inline)) {
      const int tap = ks >> 1, h = ks & 1;
      const int kh = tap / 3, kw = tap % 3;
#pragma unroll
      for (int nf = 0; nf < 2; ++nf)
        if constexpr (!WR) wd[nf] = *(const bf16x8*)(wbase + (ks * C + nf * 16) * 64);
#pragma unroll
      for (int f = 0; f < MF; ++f) xd[f] = *(const bf16x8*)(ring + roff[f][kh] + colq[f][kw][h]);
    };
    load_k(0, wc, xc);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      if (ks + 1 < KS) load_k(ks + 1, wn2, xn);
      if constexpr (WR) {  // K step ks + PD - 1 (wrapping into the next output step's first ones)
        const int kl = (ks + PD - 1) % KS;
#pragma unroll
        for (int nf = 0; nf < 2; ++nf) wq[(ks + PD - 1) % PD][nf] = wload(kl * 2 + nf);
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int f = 0; f < MF; ++f)
#pragma unroll
        for (int nf = 0; nf < 2; ++nf)
          acc[f][nf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(WR ? wq[ks % PD][nf] : wc[nf], xc[f], acc[f][nf], 0,
                                                               0, 0);
      __builtin_amdgcn_sched_barrier(0);
      if (ks + 1 < KS) {
#pragma unroll
        for (int nf = 0; nf < 2; ++nf) wc[nf] = wn2[nf];
#pragma unroll
        for (int f = 0; f < MF; ++f) xc[f] = xn[f];
      }
    }

    // ---- epilogue: lane holds channels wn*32 + 8g .. +7 of pixel (prow, col)
#pragma unroll
    for (int f = 0; f < MF; ++f) {
      const int p = wm * (R * W / 2) + 16 * f + fr;
      const long off = base + (long)p * C + wn * 32 + 8 * g;
      float v[8];
#pragma unroll
      for (int nf = 0; nf < 2; ++nf)
#pragma unroll
        for (int i = 0; i < 4; ++i) v[4 * nf + i] = acc[f][nf][i] + bs[nf][i];
      if (a.res) {
        float r[8];
        unpack8(rres[f], r);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += r[e];
      }
      *(uint4*)(a.y + off) = pack8_relu(v, a.relu);
    }
    // The next step's rows have landed: vmcnt retires in issue order, so the
    // MF younger stores may stay in flight.
    vm_wait<MF>();
    __builtin_amdgcn_s_barrier();
  }
}

}  // namespace

bool conv3x3_rows_supported(int H, int W, int Cin, int Cout) {
  return W == 56 && H % 4 == 0 && Cin == 64 && Cout == 64;
}

int conv3x3_rows_pick_strip(int B, int H, int num_cus) {
  int best = 4;
  for (int s = 4; s <= H; s += 4)
    if (H % s == 0 && (long)B * (H / s) >= num_cus) best = s;
  return best;
}

void conv3x3_rows(const void* x, const void* w, const float* bias, const void* res, void* y, const void* zero,
                  int B, int H, int W, int C, bool relu, int strip, hipStream_t s, const void* wfrag) {
  if (B <= 0) return;
  if (!conv3x3_rows_supported(H, W, C, C)) throw std::invalid_argument("conv3x3_rows: unsupported shape");
  if (strip <= 0 || strip % 4 || H % strip) throw std::invalid_argument("conv3x3_rows: bad strip");
  if (!x || !w || !bias || !y || !zero ||
      (((uintptr_t)x | (uintptr_t)w | (uintptr_t)y | (uintptr_t)zero | (uintptr_t)res) & 15))
    throw std::invalid_argument("conv3x3_rows: null / misaligned operand");
  RowConvArgs a;
  a.x = (const bf16*)x;
  a.w = (const bf16*)w;
  a.bias = bias;
  a.res = (const bf16*)res;
  a.y = (bf16*)y;
  a.zero = (const bf16*)zero;
  a.H = H;
  a.strip = strip;
  a.relu = relu;
  a.wf = (const bf16*)wfrag;
  if (wfrag && ((uintptr_t)wfrag & 15)) throw std::invalid_argument("conv3x3_rows: misaligned wfrag");
  const size_t ring = (size_t)10 * (56 + 2) * 64 * 2;
  if (wfrag)
    hipLaunchKernelGGL((conv3x3_rows_kernel<56, 64, true>), dim3(B * (H / strip)), dim3(256), ring, s, a);
  else
    hipLaunchKernelGGL((conv3x3_rows_kernel<56, 64, false>), dim3(B * (H / strip)), dim3(256),
                       (size_t)9 * 64 * 64 * 2 + ring, s, a);
  DMLC_HIP_CHECK(hipGetLastError());
}

}  // namespace dmlc
