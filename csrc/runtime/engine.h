// GPU inference engine: model graph + HBM-resident folded weights + static
// activation arena + hipGraph replay of the whole forward.
//
// Reference counterpart: the member-side model objects built at start-up and
// executed per query (src/services.rs:475-497, 513-524): `resnet18` / `alexnet`
// from tch::vision on the CPU with batch 1. Here the forward is batched, runs
// on the hand-written CDNA4 kernels in csrc/kernels, and the whole launch
// sequence for a given (batch, buffers) is captured once into a hipGraph.
#pragma once
#include <hip/hip_runtime.h>

#include <map>
#include <memory>
#include <string>
#include <tuple>
#include <vector>

#include "../kernels/kernels.h"
#include "weights.h"

namespace dmlc {

enum class OpType { Preprocess, Conv, StemPool, MaxPool, AvgPoolGlobal, AvgPoolAdaptive, SoftmaxTop1 };

struct ActShape {
  int H = 0, W = 0, C = 0;
  bool f32 = false;
  bool fp8 = false;   // OCP e4m3 with a per-tensor scale (resnet50_fp8)
  float scale = 1.f;  // value = e4m3 * scale (calibrated)
  // per-channel e4m3 scales (fp8_3x3_out's t2): value[c] = e4m3 * cscale[c],
  // folded into the producing conv's weights / bias (1 / cscale) and the
  // consuming conv's weights (cscale along K); `scale` is then 1
  std::vector<float> cscale;
  size_t elems_per_image() const { return (size_t)H * W * C; }
  size_t elem_bytes() const { return f32 ? 4 : fp8 ? 1 : 2; }
};

struct ConvLayer {
  std::string name;  // weight prefix (e.g. "layer1.0.conv1")
  std::string bn;    // BN prefix or "" (conv bias used instead)
  int cin = 0, cin_eff = 0, cout = 0, kh = 1, kw = 1, stride = 1, pad = 0;
  bool relu = false;
  bool fc = false;        // linear layer (weight [N,K]) run as a 1x1 conv
  bool pair = false;      // stem conv on the preprocess packed-RGB image (8 (kw,c) values / 16 B)
  bool stem_pool = false; // fused ResNet stem (conv+maxpool) on the paired image, K = 224
  bool alex_stem = false; // AlexNet features.0: also packed for alex_stem.hip (u8 -> conv+relu+pool) at wf_off
  int fc_hwc[3] = {0, 0, 0};  // for fc after a spatial tensor: (H,W,C) of the flatten
  int npad = 0, kpad = 0;
  size_t w_off = 0, b_off = 0;  // offsets (bytes) into the weight arena
  int in_act = -1;              // activation the conv reads
  int out_act = -1;             // activation the conv writes
  bool fp8 = false;             // e4m3 weights (input activation is e4m3)
  size_t a_off = 0;             // fp8: alpha[n] = s_in * s_w[n] (fp32 [npad])
  size_t wf_off = 0;            // weights in stream-conv fragment order (0 = none)
  size_t wf_bytes = 0;          // ... and the size of that region
  // bottleneck expand conv with its stride-1 downsample folded in (conv1x1 x2):
  // [cout][kpad + ds kpad] bf16 = [W3 | Wd] and bias b3 + bd (0 = none)
  int cat_ds = -1;              // convs_ index of that downsample
  size_t cat_off = 0, cat_b_off = 0;
};

struct Op {
  OpType type;
  int in = -1, out = -1, res = -1;  // activation ids
  int conv = -1;
  int k = 0, stride = 0, pad = 0;  // Preprocess: k = 1 for the paired layout
  std::string name;
  bool side = false;  // may run on the side stream (downsample conv, joined via the residual)
};

// Kernel-path selection. Every field defaults to the fastest measured path;
// the switches exist so tests can compare each fused / specialised path with
// the plain one it replaces (tests/test_engine_gpu.py) and so a path can be
// A/B-timed (profiles/). Python: InferenceEngine(..., options={"fused_block":
// False}); the names are the field names.
constexpr int kSmallConvMaxB = 4;  // largest batch on the query-batch conv path
constexpr int kPoolThenHeadB = 32;  // from this batch on an unfused-pool head pools once, then head_pooled

struct EngineOptions {
  bool persistent = true;        // persistent (grid-stride) implicit-GEMM conv grids
  // query-sized implicit GEMMs (M = B*Ho*Wo <= 1024, e.g. batch 1): 3-stage
  // tiles and enough K slices to put ~half the CUs to work (the 2-stage tile
  // with <= 9 slices ran 12 us per conv at batch 1, latency of one K tile
  // at a time: profiles/r4_resnet18_b256_kernel_stats_baseline.txt)
  bool igemm_small_m = true;
  // query batches (B <= kSmallConvMaxB): every 3x3 conv (+ its block's 1x1/s2
  // downsample) as one conv_small.hip launch, no split-K reduction kernels
  bool small_conv = true;
  bool fused_stem = true;        // conv1 + BN + ReLU + maxpool in one kernel (stem_pool.hip)
  bool fused_preprocess = true;  // SxS u8 images straight into the fused stem (no preprocess pass)
  bool row_conv = true;          // direct row-streaming 3x3 convs (conv3x3_rows.hip) for 56x56x64
  bool rows_wreg = true;         // ... with register-streamed weights, 2 workgroups per CU
  bool fused_block = true;       // a 56x56x64 basic block as one kernel (conv3x3_block.hip), B >= 0.7 x CUs
  // resnet50_fp8 layer1 identity bottlenecks as one kernel (bottleneck56.hip, compute / memory
  // wave roles): 156-177 vs ~245 us per block, +6% img/s (profiles/r3_bottleneck_v3.txt)
  bool fused_bottleneck = true;
  bool ds_into_expand = true;    // ResNet50 layer1.0: the 1x1 downsample computed inside conv3 (one K-concat GEMM)
  // ResNet18 layer2.0: the 1x1/s2 downsample as 2 more K steps of conv2
  // (conv3x3_rows28 DSX) instead of an output of conv3x3_s2rows that conv2
  // reads back as its residual (51 MB written + 51 MB read at B = 256)
  bool ds_into_conv2 = true;
  bool stream_conv = true;       // direct 3x3 convs with the input resident in LDS (conv3x3_stream.hip)
  bool stream_wreg = true;       // ... with register-streamed weights where available
  bool stream_l4s2 = true;       // ... also for 14x14x256 -> 512 / s2 (register weights only)
  bool fuse_ds = true;           // the block's 1x1/s2 downsample inside the stride-2 stream conv1
  // ResNet50 layer2.0.conv2 (56x56x128 -> 128 / s2): one weight-stationary
  // workgroup per image walking its rows (conv3x3_s2rows128.hip), B >= 0.7 x CUs
  bool s2rows128 = true;
  bool s2rows = true;            // ... layer2.0 (56x56x64 -> 128): one weight-stationary kernel per image
                                 // walking its rows (conv3x3_s2rows.hip), B >= 0.7 x CUs
  bool rows28 = true;            // layer2's stride-1 convs the same way (conv3x3_rows28.hip), B >= 0.7 x CUs
  bool stem_roles = true;        // u8 stem: one workgroup per image with MFMA / helper waves once B >= CUs
  bool fc_gemm = true;           // fully connected layers at B <= 256 on fc_gemm.hip (else the implicit GEMM)
  bool stem_dense = true;        // ... with the dense-K weight order (5 K steps a fragment instead of 7)
  bool bigtile = true;           // 8-wave big-tile split-K convs where picked (not on the ResNet18 b256 path)
  bool conv1x1 = true;           // weight-stationary 1x1 convs (conv1x1.hip: ResNet50 bottlenecks)
  // resnet50_fp8 layer2: an expand conv and the next bottleneck's reduce conv
  // on its output in one launch (conv1x1_chain: the reduce reads the output
  // blocks from LDS instead of 102.8 MB back from HBM at B = 256)
  bool chain_1x1 = true;
  bool fused_pool = true;        // the last conv's epilogue computes the global average pool
  bool fused_head = true;        // avgpool + fc + softmax / top-1 in one kernel (head.hip)
  bool direct13 = true;          // AlexNet's 13x13 3x3 convs with the image resident in LDS (conv3x3_13.hip)
  bool direct27 = true;          // AlexNet's 5x5 conv on 27x27x64 the same way (conv5x5_27.hip)
  bool fc_small = true;          // weight-streaming GEMV for fc layers at B <= 16 (fc_small.hip)
  // downsample convs on a side stream: measured slower (the branch slows its
  // sibling conv1 by 10-12 us and adds ~10 us of fork/join gaps per block:
  // profiles/r1_fork_ds_timeline.txt); kept to test the side-stream path
  bool fork_ds = false;
  // resnet50_fp8: every 3x3 conv's input and output in e4m3 on the fp8
  // implicit GEMM (off: slower than the default, where the bottleneck 3x3s of
  // layers 2-4 read and write e4m3 on conv3x3_stream8: fp8_3x3_in / _out below)
  bool fp8_3x3 = false;
  // ResNet50 e4m3: the bottleneck 3x3 convs that run on the row / stream
  // kernels write e4m3 (their bf16 inputs stay), so the expand conv reads e4m3:
  // 120.8k vs 116.0k img/s same box (profiles/r4_r50_fp8_3x3_out_perchannel.txt).
  // Per-channel scales folded into the weights (ActShape::cscale): logits 4.2%
  // vs 3.1% off fp32, top-1 16/16 (one per-tensor scale: 4.5% and 1-2 flips,
  // profiles/r4_r50_fp8_3x3_out_accuracy.txt)
  bool fp8_3x3_out = true;
  // ... and the strided 3x3 convs of layer3.0 / layer4.0 (implicit GEMM with
  // an e4m3 epilogue instead of the bf16 big-tile kernel)
  bool fp8_3x3_out_s2 = false;
  // ResNet50 e4m3: the bottleneck 3x3 convs of layer2 / layer3 / layer4 (and
  // the strided ones of layer2.0 / 3.0 / 4.0) also READ e4m3 (t1 written by
  // the reduce 1x1 with per-channel scales) and run on the e4m3 MFMA
  // (conv3x3_stream8.hip: 2x the bf16 rate; layer2: 142.7 -> 144.3 k img/s
  // from 135.4 k, profiles/r5_stream8_layer2.txt); needs fp8_3x3_out
  bool fp8_3x3_in = true;

  // Set a field by name; false if there is no such option.
  bool set(const std::string& name, bool value);
};

// One region of the packed weight arena (Engine::pack_audit).
struct PackRegion {
  std::string layer, kind;  // kind: w | b | alpha | wf | cat | cat_b
  size_t off = 0, bytes = 0;
};

class Engine {
 public:
  // arch: resnet18 | resnet34 | resnet50 | alexnet | resnet50_fp8 (layers 2-4
  // on the block-scaled e4m3 MFMA: per-channel weight scales, per-tensor
  // activation scales calibrated at load time on a synthetic batch)
  Engine(const std::string& arch, const WeightMap& weights, int device, int num_classes = 1000,
         int image_size = 224, const EngineOptions& options = {});
  // A replica of `src` on `device` (same graph, packing, calibration) whose
  // weight arena is allocated but not filled: copy src.weight_arena() into
  // weight_arena() (an RCCL broadcast across the node's GPUs).
  Engine(const Engine& src, int device);
  // Fill this replica's weight arena from `src` on the same device (a second
  // compute lane of a dp::Worker).
  void copy_weights_from(const Engine& src);
  ~Engine();
  Engine& operator=(const Engine&) = delete;
  // Host-only packing audit (no device is touched): build `arch`'s graph,
  // pack its weights into the host image with every write bounds-checked
  // against the region the layout pass gave it (std::runtime_error on a write
  // outside it), and return the regions. e4m3 activation scales are 1
  // instead of calibrated. *total = the arena size.
  static std::vector<PackRegion> pack_audit(const std::string& arch, const WeightMap& weights,
                                            const EngineOptions& options, size_t* total,
                                            int num_classes = 1000, int image_size = 224);
  void* weight_arena() const { return warena_; }

  const std::string& arch() const { return arch_; }
  int device() const { return device_; }
  int num_classes() const { return num_classes_; }
  int image_size() const { return image_size_; }
  int max_batch() const { return max_batch_; }
  const EngineOptions& options() const { return opt_; }
  hipStream_t stream() const { return stream_; }  // the engine's own (capture) stream
  size_t weight_bytes() const { return weight_bytes_; }
  size_t activation_bytes() const { return act_bytes_; }
  double gflop_per_image() const;

  // Allocate the activation arena for batches up to max_batch.
  void reserve(int max_batch);

  // images: device u8 [B, Hin, Win, 3]. Outputs (device): idx int32 [B],
  // prob f32 [B], optional logits f32 [B, num_classes].
  // Ordered after all prior work on `stream`; later work on `stream` sees
  // the outputs. use_graph: replay a captured hipGraph for this exact
  // (B, pointers) signature (captured on first use).
  void forward(const uint8_t* images, int B, int Hin, int Win, int32_t* idx, float* prob,
               float* logits, hipStream_t stream, bool use_graph);

  // Eager forward with an event pair around every op: (op name, ms).
  std::vector<std::pair<std::string, float>> profile(const uint8_t* images, int B, int Hin,
                                                     int Win, hipStream_t stream);

  // Device pointer to a stored activation of the last forward (debug/tests).
  const void* activation(int id) const { return acts_.at(id); }
  int num_activations() const { return (int)shapes_.size(); }
  ActShape activation_shape(int id) const { return shapes_.at(id); }
  const std::vector<Op>& ops() const { return ops_; }

 private:
  int add_act(ActShape s);
  int op_count_conv() const;
  int conv(int in, const std::string& name, const std::string& bn, int cout, int k, int stride,
           int pad, bool relu, int res = -1);
  int fc(int in, const std::string& name, int cout, bool relu, bool last);
  void build_resnet(const std::vector<int>& blocks, bool bottleneck);
  void build_alexnet();
  struct HostOnly {};
  Engine(HostOnly, const std::string& arch, const WeightMap& weights, int num_classes, int image_size,
         const EngineOptions& options);
  void build_graph(const WeightMap& weights, bool calibrate_on_device);
  void pack_weights(const WeightMap& w);
  std::vector<uint8_t> pack_host(const WeightMap& w, std::vector<PackRegion>* regions);
  void init_device();
  void mark_fp8();
  void calibrate(const WeightMap& w);
  void run_ops(const uint8_t* images, int B, int Hin, int Win, int32_t* idx, float* prob,
               float* logits, hipStream_t s, std::vector<hipEvent_t>* evs, bool trace);
  ConvArgs conv_args(const Op& op, int B, float* logits) const;
  enum class ConvPath { Stream, Rows, Rows28, Direct13, Direct27, OneByOne, BigTile, Igemm, Small, Stream8, Fc };
  ConvPath conv_path(const Op& op, int B) const;
  bool side_safe(int B) const;
  bool head_fusable(size_t oi) const;
  bool pool_fusable(size_t oi, int B) const;
  bool ds_fusable(size_t oi, int B) const;     // ops oi, oi+1 = downsample + stride-2 stream conv1
  bool block_fusable(size_t oi, int B) const;  // ops oi, oi+1 = a layer1 basic block -> conv3x3_block
  bool bottleneck_fusable(size_t oi) const;    // ops oi..oi+2 = a layer1 identity bottleneck -> bottleneck56
  bool bottleneck_head_fusable(size_t oi) const;  // ops oi, oi+1 = layer1.0's reduce + 3x3 -> bottleneck56_head
  bool bottleneck_conv3(const ConvLayer& L) const;  // L is such a block's expand conv (fragment-order weights)
  int ds_expand_op(size_t oi) const;  // ops[oi] = a downsample folded into a later expand conv: that op, or -1
  bool s2rows_ok(const Op& op, const ConvLayer& D, int B) const;  // layer2.0 conv1 + downsample -> conv3x3_s2rows
  bool ds_conv2_ok(size_t oi, int B) const;
  bool chain_ok(size_t oi, int B) const;  // ops[oi] (expand) + ops[oi + 1] (reduce) as one conv1x1_chain  // ... and that downsample as K steps of conv2 (ds_into_conv2)

  std::string arch_;
  int device_ = 0;
  int num_classes_ = 1000;
  int image_size_ = 224;
  int num_cus_ = 256;
  int max_batch_ = 0;
  int stem_pad_ = 0;
  EngineOptions opt_;
  bool fp8_ = false;  // resnet50_fp8

  std::vector<ActShape> shapes_;
  std::vector<bool> chan_act_;  // activations with per-channel e4m3 scales (mark_fp8 -> calibrate)
  std::vector<ConvLayer> convs_;
  std::vector<Op> ops_;
  int logits_act_ = -1;

  void* warena_ = nullptr;
  size_t weight_bytes_ = 0;
  std::vector<void*> acts_;
  size_t act_bytes_ = 0;
  float* ws_ = nullptr;
  void* bt_ws_ = nullptr;  // big-tile conv split-K hand-off flags + partial-tile slabs
  size_t bt_ws_bytes_ = 0;
  void* zero_ = nullptr;  // 16-B zero page: LDS-DMA source for conv padding taps
  size_t ws_elems_ = 0;
  int32_t* dummy_idx_ = nullptr;
  void* head_ws_ = nullptr;  // fused head partials + per-group tickets
  size_t head_ws_bytes_ = 0;


  hipStream_t stream_ = nullptr;
  hipEvent_t ev_out_ = nullptr;  // end of the last forward (on last_stream_)
  hipStream_t last_stream_ = nullptr;  // stream of the last direct graph replay (ev_out_ marks its end)
  bool last_stream_valid_ = false;
  hipStream_t side_ = nullptr;                      // downsample branch
  std::vector<hipEvent_t> fork_evs_, join_evs_;     // per op
  using GraphKey = std::tuple<const void*, int, int, int, void*, void*, void*>;
  std::map<GraphKey, hipGraphExec_t> graphs_;
};

}  // namespace dmlc
