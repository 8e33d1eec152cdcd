// Host-side launch API for the hand-written gfx950 kernels.
//
// Every launcher is asynchronous on the given stream, performs no allocation
// and no synchronisation (so it can be captured into a hipGraph), and checks
// operand geometry on the host before launching (a bad shape throws instead
// of faulting the GPU).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdexcept>
#include <string>

namespace dmlc {

#define DMLC_HIP_CHECK(expr)                                                          \
  do {                                                                                \
    hipError_t _e = (expr);                                                           \
    if (_e != hipSuccess)                                                             \
      throw std::runtime_error(std::string("HIP error ") + hipGetErrorString(_e) +    \
                               " at " + __FILE__ + ":" + std::to_string(__LINE__)); \
  } while (0)

// Implicit-GEMM convolution (also used for fully-connected layers as a 1x1
// conv on a [B,1,1,C] tensor).
//   x    : bf16 NHWC [B, H, W, Cin], Cin % 64 == 0; or, with `stem`, the
//          zero-padded packed RGB image [B, H, W, 3] written by preprocess_u8
//          (H/W = padded rows / row width; Ho/Wo given; pad ignored)
//   w    : bf16 [Npad, Kpad], k = (kh*KW + kw)*Cin + c, zero padded; for the
//          stem k = kh*CPK*8 + kw*3 + c, CPK = ceil(3*KW/8)
//   zero : >= 16 zero bytes (source of the LDS-DMA for padding taps)
//   bias : fp32 [Npad] (BN folded at load time), may be null
//   res  : bf16 [M, ldo] residual added before the activation, may be null
//   y    : bf16 (or fp32 if out_f32) [M, ldo], M = B*Ho*Wo
struct ConvArgs {
  const void* x = nullptr;
  const void* w = nullptr;
  const void* zero = nullptr;
  const float* bias = nullptr;
  const void* res = nullptr;
  void* y = nullptr;
  int B = 0, H = 0, W = 0, Cin = 0;
  int Ho = 0, Wo = 0, KH = 1, KW = 1, stride = 1, pad = 0;
  int N = 0, Npad = 0, Kpad = 0, ldo = 0;
  bool relu = false;
  bool out_f32 = false;
  bool stem = false;
  int split_k = 1;          // >1: fp32 partial sums into `ws`, reduced by a 2nd kernel
  float* ws = nullptr;      // split-K workspace, >= split_k * M * Npad floats
  int tile = -1;            // force a tile config (-1 = heuristic)
  bool persistent = false;  // cap the grid at max_blocks; blocks walk several tiles
  int max_blocks = 0;       // persistent grid size (multiple of 8), e.g. 2 * #CUs
  // fp8 (OCP e4m3) path, 128x128 / 256x64 tiles, no split-K:
  //   in_fp8: x and w are e4m3 bytes (Cin % 128 == 0); acc is scaled by
  //           alpha[n] (= s_in * s_w[n], fp32 [Npad])
  //   out_fp8: y = e4m3(v * out_inv_scale), saturating; res (if any) is e4m3
  //           scaled by res_scale (bf16 otherwise)
  bool in_fp8 = false, out_fp8 = false;
  const float* alpha = nullptr;
  float res_scale = 1.f, out_inv_scale = 1.f;
  // conv1x1 only: a second bf16 input concatenated along K (same pixels,
  // stride 1): K = Cin channels of x, then cin2 channels of x2 (a bottleneck's
  // expand conv with its stride-1 downsample folded in: w = [W3 | Wd])
  const void* x2 = nullptr;
  int cin2 = 0;
};

int conv_out_dim(int in, int k, int stride, int pad);
// K length of the packed weight matrix for a given conv geometry.
int conv_kpad(int Cin, int KH, int KW, bool stem = false);
// Row width (pixels) of the stem's padded packed-RGB image for an SxS input.
int stem_row_width(int S, int pad, int KW, int stride);
int conv_npad(int N);
size_t conv_splitk_ws_elems(const ConvArgs& a);
int conv_pick_split_k(const ConvArgs& a, int num_cus);
void conv2d_igemm(const ConvArgs& a, hipStream_t s);
// The split-K reduction (+ bias, residual, ReLU, bf16 / fp32 out) of `splits`
// fp32 partial slices [splits][M][Npad] in a.ws.
void splitk_reduce(const ConvArgs& a, long M, int splits, hipStream_t s);
// Fully connected layers at M = B <= 256 (fc_gemm.hip): all rows x 128
// columns x one K slice per workgroup, tiles through a 3-slot LDS-DMA ring,
// fp32 partials reduced by splitk_reduce (so a.ws is required even at 1 slice).
bool fc_gemm_supported(const ConvArgs& a);
int fc_gemm_splits(const ConvArgs& a, int num_cus);  // K slices for ~one workgroup per CU
void fc_gemm(const ConvArgs& a, int splits, hipStream_t s);

// Big-tile conv (conv_bigtile.hip): 8-wave 256x256 (cfg 0, Npad % 256 == 0)
// or 256x128 (cfg 1, Npad == 128) tiles, bf16 in/out, no stem/fp8, with an
// XCD-local K-lockstep split-K over `splits` slices. ws (needed when
// splits > 1): conv_bigtile_ws_bytes(slabs) bytes whose first
// conv_bigtile_ws_header_bytes() are zeroed once at allocation (hand-off
// flags, left zeroed by every completed launch, then an error word that a
// timed-out hand-off sets to 1), followed by the fp32 partial-tile slabs.
// Python/tests select config c with tile = kConvBigTile0 + c.
constexpr int kConvBigTile0 = 11;
// Weight-stationary 1x1 conv (conv1x1.hip): stride 1 or 2, no padding, bf16
// or e4m3 in/out (ConvArgs fp8 fields), optional residual of the output's
// dtype; Cin * elem in {128, 256, 512, 1024} bytes, N % 64 == 0, N == Npad,
// B*Ho*Wo % 64 == 0 (% 32 for 1-KB rows). Python/tests select it with
// tile = kConv1x1Tile.
constexpr int kConv1x1Tile = 100;
bool conv1x1_supported(const ConvArgs& a);
void conv1x1(const ConvArgs& a, int num_cus, hipStream_t s);
// ResNet50 e4m3 layer2: an expand conv (e4m3, residual, N = 512) and the next
// bottleneck's reduce conv r (1x1, K = 512 -> 128) on its output, one launch
// (the reduce input never goes back to HBM; conv1x1.hip CH form)
bool conv1x1_chain_supported(const ConvArgs& a, const ConvArgs& r);
// conv1x1.hip's block-loop vmcnt plan for one kernel form (in8 / out8, staged
// row bytes rb, channels per wave nw, residual, stages s, waves wv, chained
// reduce): per-wave operation counts per block (DMA dt, residual rt, stores st
// of which st2 are the chained reduce's) and every wait's threshold.
struct C1Plan {
  int s, dt, rt, st, st2;
  bool pre;  // residual loaded one block ahead
  int n1, n1_first, pro_wait, pro_wait_ch, res_wait;
};
C1Plan conv1x1_plan(bool in8, bool out8, int rb, int nw, bool res, int s, int wv, bool ch);
void conv1x1_chain(const ConvArgs& a, const ConvArgs& r, int num_cus, hipStream_t s);
int conv_bigtile_pick(const ConvArgs& a, int num_cus);  // engine's choice: config, or -1 (old kernel)
int conv_bigtile_splits(const ConvArgs& a, int cfg, int num_cus);
long conv_bigtile_slabs(const ConvArgs& a, int cfg, int splits);
size_t conv_bigtile_ws_bytes(long max_slabs);
size_t conv_bigtile_ws_header_bytes();
void conv2d_bigtile(const ConvArgs& a, int cfg, int splits, void* ws, size_t ws_bytes, hipStream_t s);
// Persistent 256x128 variant (Npad % 128 == 0): `grid` workgroups walk
// contiguous tile ranges with the LDS-DMA ring streaming across tiles.
// Python/tests select it with tile = kConvBigTile0 + 2.
bool conv_bigtile_persistent_ok(const ConvArgs& a);
int conv_bigtile_persistent_grid(const ConvArgs& a, int num_cus);
void conv2d_bigtile_persistent(const ConvArgs& a, int grid, hipStream_t s);

// 3x3/s2-style max pooling, NHWC bf16, C % 8 == 0.
void maxpool2d(const void* x, void* y, int B, int H, int W, int C, int Ho, int Wo, int k,
               int stride, int pad, hipStream_t s);
// Global average pool [B,H,W,C] -> [B,C] bf16, C % 8 == 0; in_fp8: e4m3
// input dequantised by `scale`.
void avgpool_global(const void* x, void* y, int B, int HW, int C, hipStream_t s, bool in_fp8 = false,
                    float scale = 1.f);
// Adaptive average pool to (Ho,Wo), NHWC bf16 (AlexNet avgpool(6,6)).
void avgpool_adaptive(const void* x, void* y, int B, int H, int W, int C, int Ho, int Wo,
                      hipStream_t s);

// u8 HWC images [B,Hin,Win,3] -> bf16 packed RGB [B, S+2*pad, Wr, 3] with
// the SxS image at (pad, pad) and zeros elsewhere (Wr % 8 == 0, >= S+2*pad).
// Aspect-preserving bilinear resize of the short side to S, centre crop,
// /255, ImageNet mean/std. `paired`: each pair of pixels occupies 16 B as
// [r g b r g b 0 0] (layout [B, S+2*pad, Wr/2, 8]; stem_conv_pool's input).
void preprocess_u8(const uint8_t* x, void* y, int B, int Hin, int Win, int S, int pad, int Wr,
                   hipStream_t s, bool paired = false);

// Ragged batch: image b = descs[b] (device memory, u8 HWC at its own size)
// -> out u8 [B, S, S, 3], same resize rule as preprocess_u8, rounded to u8
// (S % 4 == 0).
struct ImageDesc {
  const uint8_t* ptr;
  int h, w;
};
void resize_u8_ragged(const ImageDesc* descs, uint8_t* out, int B, int S, hipStream_t s);

// Fused ResNet stem: conv 7x7/s2/p3 (folded BN) + ReLU + maxpool 3x3/s2/p1.
//   x : paired image [B, S+6, Wq, 8] bf16 (preprocess_u8 pad=3, paired)
//   w : bf16 [64, 224], k = kh*32 + q*8 + e: chunk q covers kw = 2q, 2q+1,
//       e = 3*(kw-2q) + c; e = 6,7 and kw = 7 are zero
//   y : bf16 NHWC [B, S/4, S/4, 64]
// strip = pooled rows per workgroup (even divisor of S/4).
constexpr int kStemPoolK = 224;

// Direct 3x3/s1/p1 conv for narrow layers (ResNet layer1, 56x56x64 -> 64):
// weights resident in LDS, input rows streamed once through an LDS ring.
// Same operand layouts as conv2d_igemm (w [64, 576], bias fp32, optional
// bf16 residual, NHWC in/out).
bool conv3x3_rows_supported(int H, int W, int Cin, int Cout);
int conv3x3_rows_pick_strip(int B, int H, int num_cus);
// wfrag: the weights in fragment order (stream_frag_index, K = 9C) -> the
// register-weight variant (no LDS weights, 2 workgroups per CU; pick the
// strip for 2 x num_cus workgroups)
void conv3x3_rows(const void* x, const void* w, const float* bias, const void* res, void* y, const void* zero,
                  int B, int H, int W, int C, bool relu, int strip, hipStream_t s, const void* wfrag = nullptr);
// A whole 56x56x64 basic block, relu(conv2(relu(conv1(x))) + x), in one
// kernel (conv3x3_block.hip): one workgroup per image, the intermediate kept
// in LDS. wf1/wf2: fragment-order weights (stream_frag_index, K = 576).
bool conv3x3_block_supported(int H, int W, int C);
void conv3x3_block(const void* x, const void* wf1, const float* bias1, const void* wf2, const float* bias2, void* y,
                   const void* zero, int B, hipStream_t s);
// Direct 3x3/s1/p1 conv on 13x13 images, the whole image in LDS
// (conv3x3_13.hip): AlexNet features.6/.8/.10 (192->384, 384->256,
// 256->256). wf: fragment-order weights (stream_frag_index, K = 9 Cin).
bool conv3x3_13_supported(int H, int W, int Cin, int Cout);
// ypool: also fuse the following 3x3/s2 max-pool (13 -> 6), written instead of
// y (256 -> 256 with ReLU only: conv3x3_13_pool_supported).
bool conv3x3_13_pool_supported(int Cin, int Cout);
void conv3x3_13(const void* x, const void* wf, const float* bias, void* y, const void* zero, int B, int Cin, int Cout,
                bool relu, hipStream_t s, void* ypool = nullptr);
// Direct 5x5/s1/p2 conv 27x27x64 -> 192 with the image in LDS
// (conv5x5_27.hip): AlexNet features.3. wf: fragment-order weights
// (stream_frag_index, K = 1600); bias + ReLU.
bool conv5x5_27_supported(int H, int W, int Cin, int Cout, int pad);
// ypool: also fuse the following 3x3/s2 max-pool (27 -> 13), written instead of y.
void conv5x5_27(const void* x, const void* wf, const float* bias, void* y, const void* zero, int B, hipStream_t s,
                void* ypool = nullptr);
// ResNet50 layer1 identity bottleneck (resnet50_fp8 layer1.1 / 1.2) in one
// kernel (bottleneck56.hip): x, y e4m3 [B,56,56,256]; w1 e4m3 [64][256] with
// a1 = s_x * s_w1; wf2 / wf3: fragment-order bf16 weights (stream_frag_index,
// K = 576 / 64); y = relu(conv3(relu(conv2(relu(conv1(x))))) + x) / s_y.
bool bottleneck56_supported(int H, int W, int C, int Cm);
void bottleneck56(const void* x, const void* w1, const float* a1, const float* b1, const void* wf2, const float* b2,
                  const void* wf3, const float* b3, void* y, float res_scale, float out_inv_scale, int B,
                  hipStream_t s);
// ResNet50 layer1.0's reduce 1x1 (64 -> 64) + 3x3 (64 -> 64) as one kernel
// (bottleneck56.hip, t1 in LDS): x bf16 [B,56,56,64], w1 bf16 [64][64] (BN
// folded), b1, wf2 / b2 as above, y = t2 bf16 [B,56,56,64].
void bottleneck56_head(const void* x, const void* w1, const float* b1, const void* wf2, const float* b2, void* y,
                       int B, hipStream_t s);
// ResNet layer2.0's stride-2 3x3 conv 56x56x64 -> 28x28x128 and its 1x1/s2
// downsample in one row-streaming, weight-stationary kernel
// (conv3x3_s2rows.hip): one workgroup per image. wf / wdf: fragment-order
// weights (stream_frag_index, K = 576 / 64); y = relu?(conv3x3 + bias),
// yd = downsample + bd; wdf = bd = yd = null: the conv alone (the downsample
// then runs inside conv2: conv3x3_rows28's xds).
bool conv3x3_s2rows_supported(int Hin, int Win, int Cin, int Cout);
// ResNet50 layer2.0.conv2, 56x56x128 -> 28x28x128 / s2 (conv3x3_s2rows128.hip):
// one weight-stationary workgroup per image; wf in fragment order; y bf16, or
// e4m3 (relu(v) * out_inv_scale) when out_inv_scale > 0.
bool conv3x3_s2rows128_supported(int Hin, int Win, int Cin, int Cout);
void conv3x3_s2rows128(const void* x, const void* wf, const float* bias, void* y, int B, bool relu,
                       float out_inv_scale, hipStream_t s);
void conv3x3_s2rows(const void* x, const void* wf, const float* bias, const void* wdf, const float* bd, void* y,
                    void* yd, const void* zero, int B, bool relu, hipStream_t s);
// Weight-stationary row-streaming 3x3/s1/p1 conv for 28x28x128 -> 128
// (conv3x3_rows28.hip): one workgroup per image, the weights in registers.
// wf: fragment-order weights (stream_frag_index, K = 1152); res optional.
bool conv3x3_rows28_supported(int H, int W, int Cin, int Cout);
// xds / wds / bds (ds_into_conv2): the block's 1x1/s2 downsample of xds [B, 56,
// 56, 64] as 2 more K steps (wds fragment order [4][2][2][64][8], K = 64; bds
// added to bias), instead of a residual read.
void conv3x3_rows28(const void* x, const void* wf, const float* bias, const void* res, void* y, int B, bool relu,
                    hipStream_t s, float out_inv_scale = 0.f, const void* xds = nullptr,
                    const void* wds = nullptr, const float* bds = nullptr);  // > 0: e4m3 y, no residual
// Query-batch 3x3/p1 conv (conv_small.hip) for B <= a few images: one launch
// per conv, no split-K. x [B,H,W,CI] bf16 NHWC (CI in 64..512), wf: fragment-
// order weights (stream_frag_index, K = 9 CI), y = relu?(conv + bias (+ res)).
// Stride 2 with wdf/bd/yd also computes the block's 1x1/s2 downsample
// (fragment-order weights, K = CI) into yd. mf: pixel fragments of 16 per
// workgroup (1, 2 or 4; conv_small_pick_mf).
bool conv_small_supported(int H, int W, int CI, int CO, int stride);
int conv_small_pick_mf(int B, int H, int W, int CI, int CO, int stride, int num_cus);
void conv_small_set_mf(int mf);  // A/B override of the pick (0 = heuristic)
void conv_small(const void* x, const void* wf, const float* bias, const void* res, void* y, int B, int H, int W,
                int CI, int CO, int stride, bool relu, int mf, hipStream_t s, const void* wdf = nullptr,
                const float* bd = nullptr, void* yd = nullptr);
// Direct 3x3/p1 conv with the input image resident in LDS and per-wave weight
// rings (conv3x3_stream.hip): stride 1 on 28x28x128, 14x14x256, 7x7x512;
// stride 2 on 56x56x64 -> 128 and 28x28x128 -> 256. Hin/Win are the input
// dims; same operand layouts as conv2d_igemm.
bool conv3x3_stream_supported(int Hin, int Win, int Cin, int Cout, int stride = 1);
// e4m3 3x3 / p1 conv, stride 1 or 2, on the block-scaled e4m3 MFMA
// (conv3x3_stream8.hip): ResNet50's layer3 / layer4 bottleneck 3x3 convs with
// e4m3 t1 in and e4m3 t2 out. x [B, H, W, C] e4m3; wf: e4m3 weights [CO][9 C] (k = tap * C + c) in
// the order of conv3x3_stream8_frag_offset (KT = 9 C / 128); y = e4m3(
// relu?(acc * alpha + bias) * out_inv_scale) [B, H, W, CO].
bool conv3x3_stream8_supported(int Hin, int Win, int Cin, int Cout, int stride = 1);
size_t conv3x3_stream8_frag_offset(int j, int t, int nf, int h, int lane, int KT);
void conv3x3_stream8(const void* x, const void* wf, const float* alpha, const float* bias, void* y, const void* zero,
                     int B, int Hin, int Win, int Cin, int Cout, int stride, bool relu, float out_inv_scale,
                     hipStream_t s);
void conv3x3_stream8_set_variant(int v);  // test hook (0 = the defaults; 4: 7-row strips at layer2.0.conv2)
// Stride 2 may also compute the block's 1x1/s2 downsample conv (wd [Cout,
// Cin], bias bd, no ReLU) from the same resident input into yd.
void conv3x3_stream(const void* x, const void* w, const float* bias, const void* res, void* y, const void* zero,
                    int B, int Hin, int Win, int Cin, int Cout, int stride, bool relu, hipStream_t s,
                    unsigned long long* stamps = nullptr, const void* wd = nullptr, const float* bd = nullptr,
                    void* yd = nullptr, const void* wfrag = nullptr, const void* wdfrag = nullptr,
                    void* pool = nullptr, bool store_y = true, float out_inv_scale = 0.f);
// out_inv_scale > 0: y is e4m3 (relu(v) * out_inv_scale, saturated), no
// residual / pool / downsample.
// pool (bf16 [B, Cout]): the global average pool of the output, computed in
// the epilogue (whole-image workgroups: the 7x7x512 stride-1 conv); with
// store_y = false the output activation is not written.
bool conv3x3_stream_pool_supported(int Hin, int Win, int Cin, int Cout, int stride);
// wfrag: the same weights in fragment order (stream_weight_frag_layout), used
// by the variants that load weights straight into VGPRs (7x7x512 stride 1)
bool conv3x3_stream_uses_frag(int Hin, int Win, int Cin, int Cout, int stride);
// test / A/B hook (tests/test_kernels_gpu.py, tools/conv_bench.py), 0 = the
// defaults: bit 0 a 2-deep weight ring (14x14x256), bit 1 two channel groups a
// wave (14x14 128 -> 256 / s2), bit 2 32 channels a wave (7x7 256 -> 512 / s2)
void conv3x3_stream_set_variant(int v);
// [Cout, K] row-major bf16 -> fragment order [Cout/32][K/32][2][64][8]:
// dst index of (n, k) for n < Cout, k < K (Cout % 32 == 0, K % 32 == 0)
inline size_t stream_frag_index(int n, int k, int K) {
  const int g = n / 32, r = n % 32;
  // inverse of perm32: channel r of the group sits at tile row 16nf + rr
  const int nf = (r >> 2) & 1, rr = ((r >> 3) << 2) | (r & 3);
  const int t = k / 32, kk = k % 32, lane = (kk / 8) * 16 + rr, e = kk % 8;
  return ((((size_t)g * (K / 32) + t) * 2 + nf) * 64 + lane) * 8 + e;
}
int stem_pool_pick_strip(int B, int PH, int num_cus);
// u8 images in: strip = PH (one workgroup per image, role-split waves) when
// B >= num_cus, else stem_pool_pick_strip
int stem_pool_u8_pick_strip(int B, int PH, int num_cus);
void stem_conv_pool(const void* x, const void* w, const float* bias, void* y, int B, int S, int Wq, int strip,
                    hipStream_t s);
// Same stem with the preprocess fused: u8 HWC SxS images [B, S, S, 3] in
// (already at the target size: the identity case of preprocess_u8), the
// paired bf16 rows built in LDS with preprocess_u8's exact arithmetic.
// w_dense (optional, 16-B aligned): the same weights in dense-K order
// [64][kStemDenseK] (stem_dense_k_index); with it the one-image-per-workgroup
// kernel runs 5 K steps a fragment instead of 7 (stem_pool.hip, V & 2).
// test hooks (0 = off): 512 forces the one-image-per-workgroup kernel, 2048
// its 4-B raw-row DMA form
void stem_conv_pool_set_dbg(int dbg);
// measurement hook: per-step phase stamps of the one-image-per-workgroup
// stem's first 16 workgroups into p ([16][PH/2 + 2][4] uint64, 100 MHz:
// step start, MFMA phase done, helper work issued, helper waits done), or
// null (off)
void stem_conv_pool_set_stamps(void* p);
// Workgroup start stagger per kernel family (common.h start_stagger): the
// launchers pass kernel_stagger(k) to their kernels. kernel_stagger_set is the
// A/B hook (tools/engine_ab.py); n < 0 restores the default.
enum StaggerKernel { kStagStream = 0, kStagBlock, kStagRows28, kStagS2rows, kStagStem, kStagStream8, kStagConv1x1,
                     kStagBottleneck, kStagCount };
int kernel_stagger(int k);
void kernel_stagger_set(int k, int n);
// The process's compute-lane count (bench.py, dmlc-node --lanes): one lane
// staggers the stream convs (stagger.hip), more lanes use the defaults.
void kernel_stagger_for_lanes(int lanes);
void stem_conv_pool_u8(const uint8_t* x, const void* w, const float* bias, void* y, int B, int S, int strip,
                       hipStream_t s, const void* w_dense = nullptr);
constexpr int kStemDenseK = 160;
// Dense-K stem operand map. A kernel row's window is 22 bf16 (7 px x rgb + 1
// zero-weight slot) = 11 dwords u; K index k = 32 s + 8 fq + 2 i + h is
// element h of the dword that lane group fq reads in dword slot j = 4 s + i
// (K step s). Each slot pairs, in each 32-lane half (fq 0/1, fq 2/3), the same
// dword u of an even and an odd kernel row, which the kernel places 16 banks
// apart (stem_pool.hip): 18 of the 20 ds_read_b32 slots are bank-conflict
// free (the 7th row has no odd partner; 3 of its dwords take the zero-weight
// pad slots' partners, the other 8 pair up in slots 18 and 19). Slots 0..14:
// row pair (2 (j / 5), 2 (j / 5) + 1), dwords 2 (j % 5) + (fq >> 1); 15..19:
// the u = 10 dwords of rows 0..5, then row 6 (against row 5 under zero
// weights for u = 0..2).
struct StemDenseCell {
  int dy, u;
  bool pad;  // zero weights (reads a real dword)
};
constexpr StemDenseCell stem_dense_cell(int j, int fq) {
  if (j < 15) return {2 * (j / 5) + (fq & 1), 2 * (j % 5) + (fq >> 1), false};
  const int hp = 2 * (j - 15) + (fq >> 1), m = fq & 1;
  if (hp < 3) return {2 * hp + m, 10, false};
  if (hp < 6) return {m ? 5 : 6, hp - 3, m == 1};
  return {6, 3 + 2 * (hp - 6) + m, false};
}
// the K index of tap (dy, dx, c) (element 3 dx + c of kernel row dy's window)
inline int stem_dense_k_index(int dy, int dx, int c) {
  const int e = 3 * dx + c, u = e / 2, h = e % 2;
  for (int j = 0; j < 20; ++j)
    for (int fq = 0; fq < 4; ++fq) {
      const StemDenseCell cell = stem_dense_cell(j, fq);
      if (!cell.pad && cell.dy == dy && cell.u == u) return 32 * (j / 4) + 8 * fq + 2 * (j % 4) + h;
    }
  return -1;
}
// AlexNet features.0-2 fused (alex_stem.hip): u8 [B, 224, 224, 3] ->
// normalise -> conv 11x11/s4/p2 + bias -> ReLU -> maxpool 3x3/s2 ->
// [B, 27, 27, 64] bf16. w: [64][544] bf16 in alex_stem_k order.
bool alex_stem_supported(int S);
int alex_stem_k(int kh, int kw, int c);
constexpr int kAlexStemK = 544;
void alex_stem_u8(const uint8_t* x, const void* w, const float* bias, void* y, int B, hipStream_t s);

// One wave of v_mfma_scale_f32_16x16x128_f8f6f4 (fp8 e4m3, unit scales) on
// raw per-lane registers: a, b = int32 [64 lanes][8], d = f32 [64 lanes][4].
void mfma_fp8_probe(const void* a, const void* b, float* d, hipStream_t s);

// Fused ResNet head (head.hip): global avgpool of bf16 x [B, HW, C] + fc
// (w bf16 [Npad, ldw], bias fp32) -> fp32 logits [B, N] + softmax top-1.
// ws: head_ws_bytes(max_batch) bytes, zeroed once at allocation.
bool head_supported(int C, int N, int ldw, int Npad);
int head_splits(int B, int N, int num_cus);
// class splits of head_pooled (16 images per workgroup) when not overridden
int head_pooled_splits(int B, int N, int num_cus);
size_t head_ws_bytes(int max_batch);
void head_fused(const void* x, const void* w, const float* bias, int B, int HW, int C, int N, int ldw, int Npad,
                float* logits, int32_t* idx, float* prob, void* ws, size_t ws_bytes, int num_cus, hipStream_t s,
                bool in_fp8 = false, float scale = 1.f);  // in_fp8: x is e4m3 dequantised by scale (C >= 2048)
// Same head on an already pooled bf16 [B, C] input (the last conv's fused
// avgpool): fc + bias + softmax + top-1, 16 images per workgroup.
void head_pooled(const void* pooled, const void* w, const float* bias, int B, int C, int N, int ldw, int Npad,
                 float* logits, int32_t* idx, float* prob, void* ws, size_t ws_bytes, int num_cus, hipStream_t s,
                 int ns_override = 0, int ko = 0);

// Fully-connected layer at small batch (fc_small.hip): y[b][n] = act(x[b] .
// w[n] + bias[n]) for B <= 16 as a weight-streaming MFMA GEMV; x bf16
// [B, ldx], w bf16 [Npad, ldw], y bf16 / fp32 [B, ldo].
bool fc_small_supported(int B, int K, int ldx, int ldw);
void fc_small(const void* x, int ldx, const void* w, int ldw, const float* bias, void* y, int ldo, bool out_f32,
              int B, int K, int N, int Npad, bool relu, hipStream_t s);

// Row-wise softmax + top-1 over fp32 logits [B, ld] (first N columns).
void softmax_top1(const float* logits, int B, int N, int ld, int32_t* idx, float* prob,
                  hipStream_t s);

}  // namespace dmlc
