// GPU inference engine implementation (see engine.h).
//
// Model definitions follow the torchvision/tch-rs layer naming that the
// reference's `.ot` checkpoints use (tch::vision::resnet::resnet18 and
// tch::vision::alexnet::alexnet, constructed at src/services.rs:515,521):
// conv1/bn1/layer{1..4}.{i}.{conv,bn}{1,2[,3]}/downsample.{0,1}/fc and
// features.{0,3,6,8,10}/classifier.{1,4,6}.
#include "engine.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <optional>
#include <stdexcept>

#include "trace.h"

namespace dmlc {

namespace {

size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

const HostTensor& need(const WeightMap& w, const std::string& k) {
  auto it = w.find(k);
  if (it == w.end()) throw std::runtime_error("missing weight: " + k);
  return it->second;
}

const HostTensor* maybe(const WeightMap& w, const std::string& k) {
  auto it = w.find(k);
  return it == w.end() ? nullptr : &it->second;
}

uint16_t f2bf_host(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  if ((u & 0x7fffffffu) > 0x7f800000u) return 0x7fc0;  // NaN
  u += 0x7fffu + ((u >> 16) & 1u);                        // round to nearest even
  return (uint16_t)(u >> 16);
}

float bf2f_host(uint16_t b) {
  const uint32_t u = (uint32_t)b << 16;
  float f;
  std::memcpy(&f, &u, 4);
  return f;
}

// float -> OCP e4m3 (bias 7, max 448, no infinities), round to nearest even,
// saturating; exact by search over the 127 non-negative finite codes.
uint8_t f2e4m3_host(float f) {
  static const std::vector<float> table = [] {
    std::vector<float> t(127);
    for (int c = 0; c < 127; ++c) {
      const int e = c >> 3, m = c & 7;
      t[c] = e == 0 ? std::ldexp((float)m / 8.f, -6) : std::ldexp(1.f + (float)m / 8.f, e - 7);
    }
    return t;
  }();
  if (std::isnan(f)) return 0x7f;
  const uint8_t sign = std::signbit(f) ? 0x80 : 0;
  const float a = std::fabs(f);
  if (a >= 448.f) return sign | 0x7e;
  int c = (int)(std::upper_bound(table.begin(), table.end(), a) - table.begin()) - 1;  // table[c] <= a
  if (c < 126) {
    const float lo = table[c], hi = table[c + 1];
    if (a - lo > hi - a || (a - lo == hi - a && (c & 1))) ++c;
  }
  return sign | (uint8_t)c;
}

}  // namespace

bool EngineOptions::set(const std::string& name, bool v) {
  static const std::pair<const char*, bool EngineOptions::*> fields[] = {
      {"persistent", &EngineOptions::persistent},   {"fused_stem", &EngineOptions::fused_stem},
      {"fused_preprocess", &EngineOptions::fused_preprocess}, {"row_conv", &EngineOptions::row_conv},
      {"rows_wreg", &EngineOptions::rows_wreg},     {"fused_block", &EngineOptions::fused_block},
      {"fused_bottleneck", &EngineOptions::fused_bottleneck},
      {"ds_into_expand", &EngineOptions::ds_into_expand}, {"ds_into_conv2", &EngineOptions::ds_into_conv2},
      {"chain_1x1", &EngineOptions::chain_1x1},
      {"fp8_3x3_in", &EngineOptions::fp8_3x3_in},
      {"stream_conv", &EngineOptions::stream_conv}, {"stream_wreg", &EngineOptions::stream_wreg},
      {"stream_l4s2", &EngineOptions::stream_l4s2}, {"fuse_ds", &EngineOptions::fuse_ds},
      {"bigtile", &EngineOptions::bigtile},         {"fused_pool", &EngineOptions::fused_pool},
      {"fused_head", &EngineOptions::fused_head},   {"fc_small", &EngineOptions::fc_small},
      {"direct13", &EngineOptions::direct13},
      {"direct27", &EngineOptions::direct27},
      {"fork_ds", &EngineOptions::fork_ds},         {"fp8_3x3", &EngineOptions::fp8_3x3},
      {"fp8_3x3_out", &EngineOptions::fp8_3x3_out},
      {"fp8_3x3_out_s2", &EngineOptions::fp8_3x3_out_s2},
      {"conv1x1", &EngineOptions::conv1x1},         {"s2rows", &EngineOptions::s2rows},
      {"s2rows128", &EngineOptions::s2rows128},
      {"rows28", &EngineOptions::rows28},           {"stem_roles", &EngineOptions::stem_roles},
      {"stem_dense", &EngineOptions::stem_dense},
      {"fc_gemm", &EngineOptions::fc_gemm},
      {"igemm_small_m", &EngineOptions::igemm_small_m},
      {"small_conv", &EngineOptions::small_conv},
  };
  for (const auto& f : fields)
    if (name == f.first) {
      this->*(f.second) = v;
      return true;
    }
  return false;
}

Engine::Engine(const std::string& arch, const WeightMap& weights, int device, int num_classes,
               int image_size, const EngineOptions& options)
    : arch_(arch), device_(device), num_classes_(num_classes), image_size_(image_size), opt_(options) {
  if (num_classes % 4 != 0) throw std::invalid_argument("num_classes must be a multiple of 4");
  DMLC_HIP_CHECK(hipSetDevice(device_));
  hipDeviceProp_t prop;
  DMLC_HIP_CHECK(hipGetDeviceProperties(&prop, device_));
  num_cus_ = prop.multiProcessorCount;
  build_graph(weights, true);
  pack_weights(weights);
  init_device();
}

Engine::Engine(HostOnly, const std::string& arch, const WeightMap& weights, int num_classes, int image_size,
               const EngineOptions& options)
    : arch_(arch), device_(-1), num_classes_(num_classes), image_size_(image_size), opt_(options) {
  if (num_classes % 4 != 0) throw std::invalid_argument("num_classes must be a multiple of 4");
  build_graph(weights, false);
}

void Engine::build_graph(const WeightMap& weights, bool calibrate_on_device) {
  if (arch_ == "resnet18")
    build_resnet({2, 2, 2, 2}, false);
  else if (arch_ == "resnet34")
    build_resnet({3, 4, 6, 3}, false);
  else if (arch_ == "resnet50")
    build_resnet({3, 4, 6, 3}, true);
  else if (arch_ == "resnet50_fp8") {
    fp8_ = true;
    build_resnet({3, 4, 6, 3}, true);
    mark_fp8();
    if (calibrate_on_device) {
      calibrate(weights);
    } else {  // host-only audit: unit scales, same layout
      for (size_t i = 0; i < shapes_.size(); ++i)
        if (shapes_[i].fp8 && chan_act_[i]) shapes_[i].cscale.assign(shapes_[i].C, 1.f);
    }
  }
  else if (arch_ == "alexnet")
    build_alexnet();
  else
    throw std::invalid_argument("unknown arch: " + arch_);
}

std::vector<PackRegion> Engine::pack_audit(const std::string& arch, const WeightMap& weights,
                                           const EngineOptions& options, size_t* total, int num_classes,
                                           int image_size) {
  Engine e(HostOnly{}, arch, weights, num_classes, image_size, options);
  std::vector<PackRegion> regions;
  const std::vector<uint8_t> host = e.pack_host(weights, &regions);
  if (total) *total = host.size();
  return regions;
}

// Same graph, packing and calibration as `src`, on another device, with an
// uninitialised weight arena: the caller fills it (an RCCL broadcast of the
// source arena, GpuExecutor::ModelSlot). The host packing runs once per model
// instead of once per GPU.
Engine::Engine(const Engine& src, int device)
    : arch_(src.arch_), device_(device), num_classes_(src.num_classes_), image_size_(src.image_size_) {
  DMLC_HIP_CHECK(hipSetDevice(device_));
  hipDeviceProp_t prop;
  DMLC_HIP_CHECK(hipGetDeviceProperties(&prop, device_));
  num_cus_ = prop.multiProcessorCount;
  stem_pad_ = src.stem_pad_;
  opt_ = src.opt_;
  fp8_ = src.fp8_;
  shapes_ = src.shapes_;
  convs_ = src.convs_;
  ops_ = src.ops_;
  logits_act_ = src.logits_act_;
  weight_bytes_ = src.weight_bytes_;
  DMLC_HIP_CHECK(hipMalloc(&warena_, weight_bytes_));
  init_device();
}

void Engine::copy_weights_from(const Engine& src) {
  if (src.device_ != device_ || src.weight_bytes_ != weight_bytes_ || src.arch_ != arch_)
    throw std::invalid_argument("Engine::copy_weights_from: not a same-device replica");
  DMLC_HIP_CHECK(hipSetDevice(device_));
  DMLC_HIP_CHECK(hipMemcpy(warena_, src.warena_, weight_bytes_, hipMemcpyDeviceToDevice));
}

void Engine::init_device() {
  DMLC_HIP_CHECK(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
  DMLC_HIP_CHECK(hipEventCreateWithFlags(&ev_out_, hipEventDisableTiming));
  DMLC_HIP_CHECK(hipStreamCreateWithFlags(&side_, hipStreamNonBlocking));
  fork_evs_.resize(ops_.size());
  join_evs_.resize(ops_.size());
  for (size_t i = 0; i < ops_.size(); ++i) {
    DMLC_HIP_CHECK(hipEventCreateWithFlags(&fork_evs_[i], hipEventDisableTiming));
    DMLC_HIP_CHECK(hipEventCreateWithFlags(&join_evs_[i], hipEventDisableTiming));
  }
  ws_elems_ = (size_t)16 << 20;  // 64 MB split-K workspace
  DMLC_HIP_CHECK(hipMalloc(&ws_, ws_elems_ * sizeof(float)));
  DMLC_HIP_CHECK(hipMalloc(&zero_, 256));
  DMLC_HIP_CHECK(hipMemset(zero_, 0, 256));
}

Engine::~Engine() {
  if (device_ < 0) return;  // host-only (pack_audit): nothing on a device
  hipSetDevice(device_);
  for (auto& kv : graphs_) hipGraphExecDestroy(kv.second);
  if (!acts_.empty() && acts_[0]) hipFree(acts_[0]);
  if (warena_) hipFree(warena_);
  if (ws_) hipFree(ws_);
  if (bt_ws_) hipFree(bt_ws_);
  if (zero_) hipFree(zero_);
  if (dummy_idx_) hipFree(dummy_idx_);
  if (head_ws_) hipFree(head_ws_);
  if (ev_out_) hipEventDestroy(ev_out_);
  for (auto e : fork_evs_) hipEventDestroy(e);
  for (auto e : join_evs_) hipEventDestroy(e);
  if (side_) hipStreamDestroy(side_);
  if (stream_) hipStreamDestroy(stream_);
}

int Engine::add_act(ActShape s) {
  shapes_.push_back(s);
  return (int)shapes_.size() - 1;
}

int Engine::op_count_conv() const { return (int)convs_.size(); }

int Engine::conv(int in, const std::string& name, const std::string& bn, int cout, int k,
                 int stride, int pad, bool relu, int res) {
  const ActShape is = shapes_.at(in);
  ConvLayer L;
  L.name = name;
  L.bn = bn;
  L.pair = (op_count_conv() == 0 && is.C == 3);  // stem reads the packed RGB image
  L.cin_eff = is.C;
  L.cin = is.C;
  L.cout = cout;
  L.kh = L.kw = k;
  L.stride = stride;
  L.pad = pad;
  L.relu = relu;
  convs_.push_back(L);
  ActShape os{conv_out_dim(is.H, k, stride, pad), conv_out_dim(is.W, k, stride, pad), cout, false};
  if (L.pair) {  // stem: padding is in the image; its rows are wider than S + 2p
    os.H = conv_out_dim(image_size_, k, stride, stem_pad_);
    os.W = os.H;
  }
  convs_.back().in_act = in;
  const int out = add_act(os);
  convs_.back().out_act = out;
  Op op{OpType::Conv, in, out, res, (int)convs_.size() - 1, 0, 0, 0, name};
  ops_.push_back(op);
  return out;
}

int Engine::fc(int in, const std::string& name, int cout, bool relu, bool last) {
  const ActShape is = shapes_.at(in);
  ConvLayer L;
  L.name = name;
  L.fc = true;
  L.cin = L.cin_eff = is.H * is.W * is.C;
  if (is.H * is.W > 1) {
    L.fc_hwc[0] = is.H;
    L.fc_hwc[1] = is.W;
    L.fc_hwc[2] = is.C;
  }
  L.cout = cout;
  L.relu = relu;
  convs_.push_back(L);
  const int out = add_act(ActShape{1, 1, cout, last});
  ops_.push_back(Op{OpType::Conv, in, out, -1, (int)convs_.size() - 1, 0, 0, 0, name});
  return out;
}

void Engine::build_resnet(const std::vector<int>& blocks, bool bottleneck) {
  const int S = image_size_;
  stem_pad_ = 3;  // packed RGB image with the 7x7/s2 stem's padding built in
  int x;
  if (opt_.fused_stem && S % 32 == 0 && S >= 128 && S <= 256) {
    // paired image -> one kernel for conv1 + bn1 + relu + maxpool
    const int pairs = stem_row_width(S, 3, 7, 2) / 2;
    x = add_act(ActShape{S + 6, pairs, 8, false});
    ops_.push_back(Op{OpType::Preprocess, -1, x, -1, -1, 1, 0, 3, "preprocess"});
    ConvLayer L;
    L.name = "conv1";
    L.bn = "bn1";
    L.stem_pool = true;
    L.cin = L.cin_eff = 3;
    L.cout = 64;
    L.kh = L.kw = 7;
    L.stride = 2;
    L.pad = 3;
    L.relu = true;
    convs_.push_back(L);
    const int y = add_act(ActShape{S / 4, S / 4, 64, false});
    ops_.push_back(Op{OpType::StemPool, x, y, -1, (int)convs_.size() - 1, 0, 0, 0, "conv1+maxpool"});
    x = y;
  } else {
    x = add_act(ActShape{S + 6, stem_row_width(S, 3, 7, 2), 3, false});
    ops_.push_back(Op{OpType::Preprocess, -1, x, -1, -1, 0, 0, 3, "preprocess"});
    x = conv(x, "conv1", "bn1", 64, 7, 2, 0, true);
    const ActShape s = shapes_[x];
    const int y = add_act(ActShape{conv_out_dim(s.H, 3, 2, 1), conv_out_dim(s.W, 3, 2, 1), s.C, false});
    ops_.push_back(Op{OpType::MaxPool, x, y, -1, -1, 3, 2, 1, "maxpool"});
    x = y;
  }
  int inplanes = 64;
  for (int li = 0; li < 4; ++li) {
    const int planes = 64 << li;
    for (int bi = 0; bi < blocks[li]; ++bi) {
      const int stride = (li > 0 && bi == 0) ? 2 : 1;
      const std::string p = "layer" + std::to_string(li + 1) + "." + std::to_string(bi);
      const int outp = bottleneck ? planes * 4 : planes;
      int identity = x;
      if (stride != 1 || inplanes != outp) {
        identity = conv(x, p + ".downsample.0", p + ".downsample.1", outp, 1, stride, 0, false);
        ops_.back().side = true;
      }
      if (!bottleneck) {
        const int y = conv(x, p + ".conv1", p + ".bn1", planes, 3, stride, 1, true);
        x = conv(y, p + ".conv2", p + ".bn2", planes, 3, 1, 1, true, identity);
      } else {
        int y = conv(x, p + ".conv1", p + ".bn1", planes, 1, 1, 0, true);
        y = conv(y, p + ".conv2", p + ".bn2", planes, 3, stride, 1, true);
        x = conv(y, p + ".conv3", p + ".bn3", outp, 1, 1, 0, true, identity);
      }
      inplanes = outp;
    }
  }
  {
    const ActShape s = shapes_[x];
    const int y = add_act(ActShape{1, 1, s.C, false});
    ops_.push_back(Op{OpType::AvgPoolGlobal, x, y, -1, -1, 0, 0, 0, "avgpool"});
    x = y;
  }
  logits_act_ = fc(x, "fc", num_classes_, false, true);
  ops_.push_back(Op{OpType::SoftmaxTop1, logits_act_, -1, -1, -1, 0, 0, 0, "softmax_top1"});
}

void Engine::build_alexnet() {
  const int S = image_size_;
  stem_pad_ = 2;  // packed RGB image with the 11x11/s4 stem's padding built in
  int x = add_act(ActShape{S + 4, stem_row_width(S, 2, 11, 4), 3, false});
  ops_.push_back(Op{OpType::Preprocess, -1, x, -1, -1, 0, 0, 2, "preprocess"});
  auto pool = [&](int in, const std::string& n) {
    const ActShape s = shapes_[in];
    const int y = add_act(ActShape{conv_out_dim(s.H, 3, 2, 0), conv_out_dim(s.W, 3, 2, 0), s.C, false});
    ops_.push_back(Op{OpType::MaxPool, in, y, -1, -1, 3, 2, 0, n});
    return y;
  };
  x = conv(x, "features.0", "", 64, 11, 4, 0, true);
  // 224x224 u8 batches skip preprocess + features.0 + features.2: one fused
  // kernel (alex_stem.hip) writes features.2's output
  convs_.back().alex_stem = opt_.fused_stem && alex_stem_supported(S);
  x = pool(x, "features.2");
  x = conv(x, "features.3", "", 192, 5, 1, 2, true);
  x = pool(x, "features.5");
  x = conv(x, "features.6", "", 384, 3, 1, 1, true);
  x = conv(x, "features.8", "", 256, 3, 1, 1, true);
  x = conv(x, "features.10", "", 256, 3, 1, 1, true);
  x = pool(x, "features.12");
  {
    const ActShape s = shapes_[x];
    if (!(s.H == 6 && s.W == 6)) {
      const int y = add_act(ActShape{6, 6, s.C, false});
      ops_.push_back(Op{OpType::AvgPoolAdaptive, x, y, -1, -1, 0, 0, 0, "avgpool"});
      x = y;
    }
  }
  x = fc(x, "classifier.1", 4096, true, false);
  x = fc(x, "classifier.4", 4096, true, false);
  logits_act_ = fc(x, "classifier.6", num_classes_, false, true);
  ops_.push_back(Op{OpType::SoftmaxTop1, logits_act_, -1, -1, -1, 0, 0, 0, "softmax_top1"});
}

// resnet50_fp8: conv outputs with a multiple of 128 channels are e4m3: the
// 256..2048-channel block outputs and residual paths (where the bytes are:
// layer1's 56x56x256 tensors dominate the traffic), so every 1x1 expand /
// reduce conv and downsample reads or writes e4m3. The bottleneck 3x3 convs
// of layers 2-4 then read e4m3 too and run on the e4m3 MFMA
// (conv3x3_stream8.hip, fp8_3x3_in: their t1 gets per-channel scales from the
// reduce 1x1) and write e4m3 (fp8_3x3_out), so the expand convs read e4m3.
// (EngineOptions::fp8_3x3 instead marks every 3x3 conv's input and output
// e4m3 for the fp8 implicit GEMM: slower, off.) The stem and layer1's
// 64-channel inner convs stay bf16 (Cin = 64 is below the fp8 kernels'
// 128-channel K-tile).
void Engine::mark_fp8() {
  const bool fp8_3x3 = opt_.fp8_3x3;
  std::vector<bool> near_3x3(shapes_.size(), false);  // read or written by a 3x3 conv
  for (const Op& op : ops_)
    if (op.type == OpType::Conv && !convs_[op.conv].fc && convs_[op.conv].kh == 3) {
      near_3x3[op.in] = true;
      near_3x3[op.out] = true;
    }
  for (const Op& op : ops_)
    if (op.type == OpType::Conv && !convs_[op.conv].fc && shapes_[op.out].C % 128 == 0 &&
        (fp8_3x3 || !near_3x3[op.out]))
      shapes_[op.out].fp8 = true;
  chan_act_.assign(shapes_.size(), false);
  if (opt_.fp8_3x3_out && !fp8_3x3) {
    // outputs of 3x3 convs that no 3x3 conv reads (a bottleneck's t2), where
    // the conv runs on conv3x3_rows28 / conv3x3_stream (e4m3 epilogues)
    std::vector<bool> in_3x3(shapes_.size(), false);
    for (const Op& op : ops_)
      if (op.type == OpType::Conv && !convs_[op.conv].fc && convs_[op.conv].kh == 3) in_3x3[op.in] = true;
    for (const Op& op : ops_) {
      if (op.type != OpType::Conv) continue;
      const ConvLayer& L = convs_[op.conv];
      const ActShape& is = shapes_[op.in];
      if (L.fc || L.kh != 3 || L.kw != 3 || L.pad != 1 || op.res >= 0 || in_3x3[op.out] ||
          shapes_[op.out].C % 128 || shapes_[op.in].fp8)
        continue;
      if (conv3x3_rows28_supported(is.H, is.W, is.C, L.cout) ||
          conv3x3_stream_supported(is.H, is.W, is.C, L.cout, L.stride) || (opt_.fp8_3x3_out_s2 && L.stride == 2)) {
        shapes_[op.out].fp8 = true;
        chan_act_[op.out] = true;
      }
    }
    if (opt_.fp8_3x3_in) {
      // ... and their e4m3 input t1 where the e4m3 3x3 kernel runs the conv:
      // t1 is written by a 1x1 conv and read by nothing else
      for (const Op& op : ops_) {
        if (op.type != OpType::Conv) continue;
        const ConvLayer& L = convs_[op.conv];
        const ActShape& is = shapes_[op.in];
        if (L.fc || L.kh != 3 || L.kw != 3 || L.pad != 1 || op.res >= 0 || is.fp8 || is.f32 ||
            shapes_[op.out].f32 || in_3x3[op.out] || !conv3x3_stream8_supported(is.H, is.W, is.C, L.cout, L.stride))
          continue;
        if (!chan_act_[op.out] && (L.stride == 1 || shapes_[op.out].fp8)) continue;
        int producers = 0, readers = 0;
        bool from_1x1 = false;
        for (const Op& o : ops_) {
          if (o.type == OpType::Conv && o.out == op.in) {
            ++producers;
            const ConvLayer& P = convs_[o.conv];
            from_1x1 = !P.fc && P.kh == 1 && P.kw == 1 && P.stride == 1 && o.res < 0;
          }
          if (o.in == op.in || o.res == op.in) ++readers;
        }
        if (producers != 1 || !from_1x1 || readers != 1) continue;
        shapes_[op.in].fp8 = true;
        chan_act_[op.in] = true;
        // (a strided one's t2: e4m3 out too, per-channel scales, as the stride-1 ones')
        shapes_[op.out].fp8 = true;
        chan_act_[op.out] = true;
      }
    }
  }
  for (const Op& op : ops_) {
    if (op.type != OpType::Conv) continue;
    if (op.res >= 0 && shapes_[op.res].fp8 != shapes_[op.out].fp8)
      throw std::runtime_error("mark_fp8: residual and output dtypes differ at " + op.name);
    if (shapes_[op.in].fp8 && shapes_[op.in].C % 128)
      throw std::runtime_error("mark_fp8: fp8 conv needs Cin % 128 == 0: " + op.name);
  }
}

// Static per-tensor activation scales: run the bf16 model on a synthetic
// calibration batch and take amax/448 of every tensor that is stored as e4m3.
void Engine::calibrate(const WeightMap& w) {
  const int Bc = 8;
  // every activation must be materialised: no path that computes one inside
  // its reader (the layer1.0 downsample inside the expand conv)
  EngineOptions ro;
  ro.ds_into_expand = false;
  ro.fused_bottleneck = false;
  Engine ref(arch_.substr(0, arch_.find("_fp8")), w, device_, num_classes_, image_size_, ro);
  if (ref.num_activations() != num_activations()) throw std::runtime_error("calibrate: graph mismatch");
  ref.reserve(Bc);
  const size_t img_bytes = (size_t)Bc * image_size_ * image_size_ * 3;
  std::vector<uint8_t> host(img_bytes);
  uint32_t st = 12345u;  // fixed-seed xorshift: deterministic scales
  for (auto& v : host) {
    st ^= st << 13;
    st ^= st >> 17;
    st ^= st << 5;
    v = (uint8_t)(st >> 24);
  }
  uint8_t* d_img = nullptr;
  DMLC_HIP_CHECK(hipMalloc(&d_img, img_bytes));
  DMLC_HIP_CHECK(hipMemcpy(d_img, host.data(), img_bytes, hipMemcpyHostToDevice));
  ref.forward(d_img, Bc, image_size_, image_size_, nullptr, nullptr, nullptr, nullptr, false);
  DMLC_HIP_CHECK(hipDeviceSynchronize());
  DMLC_HIP_CHECK(hipFree(d_img));
  for (int i = 0; i < num_activations(); ++i) {
    if (!shapes_[i].fp8) continue;
    const size_t n = shapes_[i].elems_per_image() * Bc;
    std::vector<uint16_t> a(n);
    DMLC_HIP_CHECK(hipMemcpy(a.data(), ref.activation(i), n * 2, hipMemcpyDeviceToHost));
    float amax = 0.f;
    for (uint16_t v : a) amax = std::max(amax, std::fabs(bf2f_host(v)));
    shapes_[i].scale = std::max(amax, 1e-6f) / 448.f;
    if (!chan_act_[i]) continue;
    // per-channel scales (a channel whose calibration values stay tiny gets
    // 1/1000 of the tensor's range instead of an unbounded 1 / scale)
    const int C = shapes_[i].C;
    std::vector<float> cm(C, 0.f);
    for (size_t j = 0; j < n; ++j) cm[j % C] = std::max(cm[j % C], std::fabs(bf2f_host(a[j])));
    shapes_[i].cscale.resize(C);
    for (int c = 0; c < C; ++c) shapes_[i].cscale[c] = std::max(cm[c], std::max(amax, 1e-6f) * 1e-3f) / 448.f;
    shapes_[i].scale = 1.f;
  }
}

namespace {

// A layer's region of the host weight image: every write is bounds-checked
// against the size the layout pass gave it, so a packing order that writes
// past its region fails at load instead of corrupting its neighbours.
struct RegionRef {
  uint8_t* base = nullptr;
  size_t bytes = 0;
  const std::string* layer = nullptr;
  const char* kind = "";
  template <class T>
  T& at(size_t i) const {
    if ((i + 1) * sizeof(T) > bytes)
      throw std::runtime_error("pack_weights: write past the " + std::string(kind) + " region of " + *layer);
    return reinterpret_cast<T*>(base)[i];
  }
  void copy(size_t off, const void* src, size_t n) const {
    if (off + n > bytes)
      throw std::runtime_error("pack_weights: copy past the " + std::string(kind) + " region of " + *layer);
    std::memcpy(base + off, src, n);
  }
};

}  // namespace

void Engine::pack_weights(const WeightMap& w) {
  const std::vector<uint8_t> host = pack_host(w, nullptr);
  DMLC_HIP_CHECK(hipMalloc(&warena_, weight_bytes_));
  DMLC_HIP_CHECK(hipMemcpy(warena_, host.data(), weight_bytes_, hipMemcpyHostToDevice));
}

std::vector<uint8_t> Engine::pack_host(const WeightMap& w, std::vector<PackRegion>* regions) {
  // Layout pass.
  size_t off = 0;
  for (auto& L : convs_) {
    L.npad = conv_npad(L.cout);
    L.kpad = L.stem_pool ? kStemPoolK : conv_kpad(L.cin_eff, L.kh, L.kw, L.pair);
    L.fp8 = L.in_act >= 0 && shapes_[L.in_act].fp8;
    L.w_off = off;
    off = align_up(off + (size_t)L.npad * L.kpad * (L.fp8 ? 1 : 2), 256);
    L.b_off = off;
    off = align_up(off + (size_t)L.npad * 4, 256);
    if (L.fp8) {
      L.a_off = off;
      off = align_up(off + (size_t)L.npad * 4, 256);
    }
    L.wf_off = 0;
    L.wf_bytes = 0;
    // (3x3 convs the register-weight stream conv runs, and the 1x1/s2
    // downsample it fuses next to a stride-2 one)
    // (and every 3x3/p1 conv and 1x1/s2 downsample the query-batch conv can
    // run: conv_small.hip)
    const bool small =
        !L.fp8 && !L.fc && !L.pair && !L.stem_pool && L.in_act >= 0 && L.cout % 32 == 0 &&
        ((L.kh == 3 && L.kw == 3 && L.pad == 1) || (L.kh == 1 && L.kw == 1 && L.stride == 2 && L.pad == 0)) &&
        conv_small_supported(shapes_[L.in_act].H, shapes_[L.in_act].W, shapes_[L.in_act].C, L.cout, L.stride);
    if (small || (!L.fp8 && !L.fc && !L.pair && !L.stem_pool && L.in_act >= 0 && L.cout % 32 == 0 && L.kpad % 32 == 0 &&
        (((L.kh == 3 && L.kw == 3) || (L.kh == 1 && L.kw == 1 && L.stride == 2)) &&
             (conv3x3_stream_uses_frag(shapes_[L.in_act].H, shapes_[L.in_act].W, shapes_[L.in_act].C, L.cout,
                                       L.stride) ||
              (L.stride == 2 &&
               conv3x3_s2rows_supported(shapes_[L.in_act].H, shapes_[L.in_act].W, shapes_[L.in_act].C, L.cout)) ||
              (L.kh == 3 && L.stride == 1 && L.pad == 1 &&
               conv3x3_rows28_supported(shapes_[L.in_act].H, shapes_[L.in_act].W, shapes_[L.in_act].C, L.cout))) ||
         (L.kh == 3 && L.kw == 3 && L.stride == 1 && L.pad == 1 &&
          (conv3x3_rows_supported(shapes_[L.in_act].H, shapes_[L.in_act].W, shapes_[L.in_act].C, L.cout) ||
           conv3x3_13_supported(shapes_[L.in_act].H, shapes_[L.in_act].W, shapes_[L.in_act].C, L.cout)))))) {
      L.wf_off = off;  // fragment-order copy for the register-weight stream conv
      L.wf_bytes = (size_t)L.cout * L.kpad * 2;
      off = align_up(off + L.wf_bytes, 256);
    }
    if (!L.fp8 && !L.fc && L.in_act >= 0 && L.kh == 5 && L.kw == 5 && L.stride == 1 &&
        conv5x5_27_supported(shapes_[L.in_act].H, shapes_[L.in_act].W, shapes_[L.in_act].C, L.cout, L.pad)) {
      L.wf_off = off;  // fragment-order copy for conv5x5_27.hip
      L.wf_bytes = (size_t)L.cout * L.kpad * 2;
      off = align_up(off + L.wf_bytes, 256);
    }
    if (L.fp8 && !L.fc && L.in_act >= 0 && L.kh == 3 && L.kw == 3 && L.pad == 1 && L.kpad == 9 * L.cin &&
        conv3x3_stream8_supported(shapes_[L.in_act].H, shapes_[L.in_act].W, shapes_[L.in_act].C, L.cout,
                                  L.stride)) {
      L.wf_off = off;  // e4m3 fragment-order copy for conv3x3_stream8.hip
      L.wf_bytes = (size_t)L.cout * L.kpad;
      off = align_up(off + L.wf_bytes, 256);
    }
    if (bottleneck_conv3(L)) {  // fragment-order copy for bottleneck56.hip's expand conv
      L.wf_off = off;
      L.wf_bytes = (size_t)L.cout * L.kpad * 2;
      off = align_up(off + L.wf_bytes, 256);
    }
    if (L.stem_pool) {  // dense-K order for the one-image-per-workgroup stem (stem_dense_k_index)
      L.wf_off = off;
      L.wf_bytes = (size_t)L.cout * kStemDenseK * 2;
      off = align_up(off + L.wf_bytes, 256);
    }
    if (L.alex_stem) {  // paired-chunk K order for alex_stem.hip
      L.wf_off = off;
      L.wf_bytes = (size_t)L.cout * kAlexStemK * 2;
      off = align_up(off + L.wf_bytes, 256);
    }
  }
  // bottleneck expand convs that can take their stride-1 downsample as a
  // second K block (conv1x1 with x2): both bf16 in, 1x1, same output
  for (size_t j = 0; j < ops_.size(); ++j) {
    const Op& c3 = ops_[j];
    if (c3.type != OpType::Conv || c3.res < 0) continue;
    ConvLayer& L3 = convs_[c3.conv];
    for (size_t i = 0; i < j; ++i) {
      const Op& d = ops_[i];
      if (d.type != OpType::Conv || d.out != c3.res) continue;
      const ConvLayer& D = convs_[d.conv];
      if (D.fc || L3.fc || D.kh != 1 || D.kw != 1 || D.stride != 1 || D.relu || !L3.relu || L3.kh != 1 ||
          L3.kw != 1 || L3.stride != 1 || D.fp8 || L3.fp8 || shapes_[d.in].fp8 || shapes_[c3.in].fp8 ||
          D.cout != L3.cout || D.npad != L3.npad || shapes_[d.in].H != shapes_[c3.in].H ||
          shapes_[d.in].W != shapes_[c3.in].W || D.kpad != D.cin || L3.kpad != L3.cin)
        continue;
      L3.cat_ds = d.conv;
      L3.cat_off = off;
      off = align_up(off + (size_t)L3.npad * (L3.kpad + D.kpad) * 2, 256);
      L3.cat_b_off = off;
      off = align_up(off + (size_t)L3.npad * 4, 256);
    }
  }
  weight_bytes_ = off;
  std::vector<uint8_t> host(off, 0);
  auto region = [&](const ConvLayer& L, const char* kind, size_t roff, size_t bytes) {
    if (roff + bytes > host.size())
      throw std::runtime_error("pack_weights: " + std::string(kind) + " region of " + L.name + " past the arena");
    if (regions) regions->push_back(PackRegion{L.name, kind, roff, bytes});
    return RegionRef{host.data() + roff, bytes, &L.name, kind};
  };
  for (auto& L : convs_) {
    const HostTensor& W = need(w, L.name + ".weight");
    const HostTensor* cb = maybe(w, L.name + ".bias");
    std::vector<float> scale(L.cout, 1.f), bias(L.cout, 0.f);
    if (cb) {
      if (cb->numel() != L.cout) throw std::runtime_error("bad bias size: " + L.name);
      for (int n = 0; n < L.cout; ++n) bias[n] = cb->data[n];
    }
    if (!L.bn.empty()) {
      const HostTensor& g = need(w, L.bn + ".weight");
      const HostTensor& b = need(w, L.bn + ".bias");
      const HostTensor& m = need(w, L.bn + ".running_mean");
      const HostTensor& v = need(w, L.bn + ".running_var");
      for (int n = 0; n < L.cout; ++n) {
        const double s = (double)g.data[n] / std::sqrt((double)v.data[n] + 1e-5);
        scale[n] = (float)s;
        bias[n] = (float)((double)b.data[n] + ((double)bias[n] - (double)m.data[n]) * s);
      }
    }
    if (L.out_act >= 0 && !shapes_[L.out_act].cscale.empty()) {
      // the conv writes e4m3 with per-channel scales: fold 1 / cscale[n] into
      // its weights and bias (ReLU commutes with a positive scale)
      const std::vector<float>& cs = shapes_[L.out_act].cscale;
      for (int n = 0; n < L.cout; ++n) {
        scale[n] /= cs[n];
        bias[n] /= cs[n];
      }
    }
    const RegionRef rw = region(L, "w", L.w_off, (size_t)L.npad * L.kpad * (L.fp8 ? 1 : 2));
    const RegionRef rb = region(L, "b", L.b_off, (size_t)L.npad * 4);
    const RegionRef rf = L.wf_off ? region(L, "wf", L.wf_off, L.wf_bytes) : RegionRef{};
    std::vector<uint16_t> wbf;
    RegionRef rwbf = rw;  // bf16 weights [npad][kpad]
    if (L.fp8) {  // fold into a bf16 staging copy first, then quantise per row
      wbf.assign((size_t)L.npad * L.kpad, 0);
      rwbf.base = (uint8_t*)wbf.data();
      rwbf.bytes = wbf.size() * 2;
      rwbf.kind = "bf16 staging";
    }
    auto pw = [&](size_t i) -> uint16_t& { return rwbf.at<uint16_t>(i); };
    if (!L.fc) {
      if (W.shape.size() != 4 || W.shape[0] != L.cout || W.shape[1] != L.cin || W.shape[2] != L.kh ||
          W.shape[3] != L.kw)
        throw std::runtime_error("bad conv weight shape: " + L.name);
      for (int n = 0; n < L.cout; ++n)
        for (int c = 0; c < L.cin; ++c)
          for (int i = 0; i < L.kh; ++i)
            for (int j = 0; j < L.kw; ++j) {
              const float v = W.data[(((size_t)n * L.cin + c) * L.kh + i) * L.kw + j] * scale[n];
              size_t k;
              if (L.stem_pool)  // paired stem: chunk (kw/2) of row kh, slot 3*(kw%2) + c
                k = (size_t)i * 32 + (j / 2) * 8 + (j % 2) * 3 + c;
              else if (L.pair)  // stem: k = kh*CPK*8 + kw*3 + c
                k = (size_t)i * ((L.kw * 3 + 7) / 8) * 8 + j * 3 + c;
              else
                k = (size_t)(i * L.kw + j) * L.cin_eff + c;
              pw((size_t)n * L.kpad + k) = f2bf_host(v);
            }
    } else {
      if (W.shape.size() != 2 || W.shape[0] != L.cout || W.shape[1] != L.cin)
        throw std::runtime_error("bad linear weight shape: " + L.name);
      const int H = L.fc_hwc[0], Wd = L.fc_hwc[1], C = L.fc_hwc[2];
      for (int n = 0; n < L.cout; ++n)
        for (int k = 0; k < L.cin; ++k) {
          int dst = k;
          if (H > 0) {  // torch flattens NCHW (c,h,w); our activations are NHWC (h,w,c)
            const int c = k / (H * Wd), hw = k % (H * Wd);
            dst = hw * C + c;
          }
          pw((size_t)n * L.kpad + dst) = f2bf_host(W.data[(size_t)n * L.cin + k] * scale[n]);
        }
    }
    for (int n = 0; n < L.cout; ++n) rb.at<float>(n) = bias[n];
    if (L.stem_pool) {
      for (int n = 0; n < L.cout; ++n)
        for (int c = 0; c < L.cin; ++c)
          for (int i = 0; i < L.kh; ++i)
            for (int j = 0; j < L.kw; ++j)
              rf.at<uint16_t>((size_t)n * kStemDenseK + stem_dense_k_index(i, j, c)) =
                  f2bf_host(W.data[(((size_t)n * L.cin + c) * L.kh + i) * L.kw + j] * scale[n]);
    } else if (L.alex_stem) {
      for (int n = 0; n < L.cout; ++n)
        for (int c = 0; c < L.cin; ++c)
          for (int i = 0; i < L.kh; ++i)
            for (int j = 0; j < L.kw; ++j)
              rf.at<uint16_t>((size_t)n * kAlexStemK + alex_stem_k(i, j, c)) =
                  f2bf_host(W.data[(((size_t)n * L.cin + c) * L.kh + i) * L.kw + j] * scale[n]);
    } else if (L.wf_off && !L.fp8) {  // bf16 fragment order (e4m3 layers: stream8's order, below)
      for (int n = 0; n < L.cout; ++n)
        for (int k = 0; k < L.kpad; ++k) rf.at<uint16_t>(stream_frag_index(n, k, L.kpad)) = pw((size_t)n * L.kpad + k);
    }
    if (L.fp8) {
      // e4m3 weights with a per-output-channel scale; alpha = s_in * s_w[n]
      const RegionRef& q = rw;
      const RegionRef alpha = region(L, "alpha", L.a_off, (size_t)L.npad * 4);
      const float s_in = shapes_[L.in_act].scale;
      // per-channel input scales (fp8_3x3_out): along K (channel k % Cin)
      const std::vector<float>& ics = shapes_[L.in_act].cscale;
      const int cin = shapes_[L.in_act].C;
      auto wv = [&](int n, int k) {
        const float v = bf2f_host(pw((size_t)n * L.kpad + k));
        return ics.empty() ? v : v * ics[k % cin];
      };
      for (int n = 0; n < L.npad; ++n) {
        float amax = 0.f;
        for (int k = 0; k < L.kpad; ++k) amax = std::max(amax, std::fabs(wv(n, k)));
        const float sw = amax > 0.f ? amax / 448.f : 1.f;
        for (int k = 0; k < L.kpad; ++k) q.at<uint8_t>((size_t)n * L.kpad + k) = f2e4m3_host(wv(n, k) / sw);
        alpha.at<float>(n) = s_in * sw;
      }
      if (L.wf_off) {  // conv3x3_stream8's fragment order of the e4m3 weights
        const uint8_t* qb = q.base;
        const int KT = L.kpad / 128;
        for (int j = 0; j < L.cout / 32; ++j)
          for (int t = 0; t < KT; ++t)
            for (int nf = 0; nf < 2; ++nf)
              for (int h = 0; h < 2; ++h)
                for (int ln = 0; ln < 64; ++ln) {
                  const int fq = ln >> 4, r = 16 * nf + (ln & 15);
                  const int n = 32 * j + 8 * ((r & 15) >> 2) + 4 * (r >> 4) + (r & 3);  // perm32
                  const int k0 = 128 * t + 32 * fq + 16 * (h ^ (fq & 1));
                  rf.copy(conv3x3_stream8_frag_offset(j, t, nf, h, ln, KT), qb + (size_t)n * L.kpad + k0, 16);
                }
      }
    }
  }
  for (auto& L : convs_) {  // [W3 | Wd] and b3 + bd from the folded bf16 copies above
    if (L.cat_ds < 0) continue;
    const ConvLayer& D = convs_[L.cat_ds];
    const int K = L.kpad + D.kpad;
    const RegionRef cw = region(L, "cat", L.cat_off, (size_t)L.npad * K * 2);
    const uint16_t* w3 = (const uint16_t*)(host.data() + L.w_off);
    const uint16_t* wd = (const uint16_t*)(host.data() + D.w_off);
    for (int n = 0; n < L.npad; ++n) {
      cw.copy((size_t)n * K * 2, w3 + (size_t)n * L.kpad, (size_t)L.kpad * 2);
      cw.copy(((size_t)n * K + L.kpad) * 2, wd + (size_t)n * D.kpad, (size_t)D.kpad * 2);
    }
    const RegionRef cb = region(L, "cat_b", L.cat_b_off, (size_t)L.npad * 4);
    const float* b3 = (const float*)(host.data() + L.b_off);
    const float* bd = (const float*)(host.data() + D.b_off);
    for (int n = 0; n < L.npad; ++n) cb.at<float>(n) = b3[n] + bd[n];
  }
  return host;
}

void Engine::reserve(int max_batch) {
  if (max_batch <= max_batch_) return;
  DMLC_HIP_CHECK(hipSetDevice(device_));
  DMLC_HIP_CHECK(hipDeviceSynchronize());
  for (auto& kv : graphs_) hipGraphExecDestroy(kv.second);
  graphs_.clear();
  if (!acts_.empty() && acts_[0]) DMLC_HIP_CHECK(hipFree(acts_[0]));
  if (dummy_idx_) DMLC_HIP_CHECK(hipFree(dummy_idx_));
  std::vector<size_t> offs;
  size_t total = 0;
  for (const auto& s : shapes_) {
    offs.push_back(total);
    total = align_up(total + s.elems_per_image() * max_batch * s.elem_bytes(), 256);
  }
  void* base = nullptr;
  DMLC_HIP_CHECK(hipMalloc(&base, total));
  acts_.clear();
  for (size_t o : offs) acts_.push_back((uint8_t*)base + o);
  act_bytes_ = total;
  DMLC_HIP_CHECK(hipMalloc(&dummy_idx_, (size_t)max_batch * 8));
  max_batch_ = max_batch;
  if (head_ws_) DMLC_HIP_CHECK(hipFree(head_ws_));
  head_ws_bytes_ = head_ws_bytes(max_batch);
  DMLC_HIP_CHECK(hipMalloc(&head_ws_, head_ws_bytes_));
  DMLC_HIP_CHECK(hipMemset(head_ws_, 0, head_ws_bytes_));
  // big-tile conv split-K slabs for the largest batch
  long slabs = 0;
  for (const Op& op : ops_) {
    if (op.type != OpType::Conv) continue;
    const ConvArgs a = conv_args(op, max_batch, nullptr);
    const int cfg = opt_.bigtile ? conv_bigtile_pick(a, num_cus_) : -1;
    if (cfg >= 0) slabs = std::max(slabs, conv_bigtile_slabs(a, cfg, conv_bigtile_splits(a, cfg, num_cus_)));
  }
  if (bt_ws_) DMLC_HIP_CHECK(hipFree(bt_ws_));
  bt_ws_bytes_ = conv_bigtile_ws_bytes(slabs);
  DMLC_HIP_CHECK(hipMalloc(&bt_ws_, bt_ws_bytes_));
  DMLC_HIP_CHECK(hipMemset(bt_ws_, 0, conv_bigtile_ws_header_bytes()));
}

double Engine::gflop_per_image() const {
  double f = 0;
  for (const auto& op : ops_) {
    if (op.type != OpType::Conv && op.type != OpType::StemPool) continue;
    const ConvLayer& L = convs_[op.conv];
    ActShape o = shapes_[op.out];
    if (op.type == OpType::StemPool) o.H = o.W = image_size_ / 2;  // the conv's (pre-pool) output
    f += 2.0 * o.H * o.W * L.cout * (double)L.cin * L.kh * L.kw;
  }
  return f * 1e-9;
}

ConvArgs Engine::conv_args(const Op& op, int B, float* logits) const {
  const ConvLayer& L = convs_[op.conv];
  const ActShape& is = shapes_[op.in];
  const ActShape& os = shapes_[op.out];
  ConvArgs a;
  a.x = acts_[op.in];
  a.zero = zero_;
  a.stem = L.pair;
  a.w = (const uint8_t*)warena_ + L.w_off;
  a.bias = (const float*)((const uint8_t*)warena_ + L.b_off);
  a.res = op.res >= 0 ? acts_[op.res] : nullptr;
  a.y = (os.f32 && logits) ? (void*)logits : acts_[op.out];
  a.B = B;
  if (L.fc) {
    a.H = a.W = 1;
    a.Cin = L.cin_eff;
  } else {
    a.H = is.H;
    a.W = is.W;
    a.Cin = is.C;
  }
  a.KH = L.kh;
  a.KW = L.kw;
  a.stride = L.stride;
  a.pad = L.pad;
  a.Ho = os.H;
  a.Wo = os.W;
  a.N = L.cout;
  a.Npad = L.npad;
  a.Kpad = L.kpad;
  a.ldo = L.cout;
  a.relu = L.relu;
  a.out_f32 = os.f32;
  a.in_fp8 = L.fp8;
  a.out_fp8 = os.fp8;
  if (L.fp8) a.alpha = (const float*)((const uint8_t*)warena_ + L.a_off);
  if (op.res >= 0 && shapes_[op.res].fp8) a.res_scale = shapes_[op.res].scale;
  if (os.fp8) a.out_inv_scale = 1.f / os.scale;
  int s = conv_pick_split_k(a, num_cus_);
  const size_t M = (size_t)B * os.H * os.W;
  if (opt_.igemm_small_m && M <= 1024 && !L.pair && !L.fc && !L.fp8 && !os.fp8 && !os.f32 && L.npad % 128 == 0) {
    // 64x256 ns3 for the narrowest outputs, else 128x128 ns3 (conv_igemm.hip tile table)
    a.tile = (M <= 64 && L.npad % 256 == 0) ? 5 : 3;
    const int bm = a.tile == 5 ? 64 : 128, bn = a.tile == 5 ? 256 : 128;
    const int tiles = (int)((M + bm - 1) / bm) * (L.npad / bn);
    const int k_tiles = L.kpad / 64;
    s = std::max(1, std::min({k_tiles / 2, (num_cus_ / 2 + tiles - 1) / tiles, 32}));
  }
  while (s > 1 && (size_t)s * M * L.npad > ws_elems_) --s;
  a.split_k = s;
  a.ws = ws_;
  a.persistent = opt_.persistent;
  a.max_blocks = 2 * num_cus_;
  return a;
}

Engine::ConvPath Engine::conv_path(const Op& op, int B) const {
  const ConvLayer& L = convs_[op.conv];
  const ActShape& is = shapes_[op.in];
  const bool k3b = !L.fc && !L.pair && !L.fp8 && L.kh == 3 && L.kw == 3 && L.pad == 1 && !shapes_[op.out].f32;
  const bool k3 = k3b && !shapes_[op.out].fp8;
  // e4m3 output (fp8_3x3_out): the row / stream kernels' e4m3 epilogue
  const bool k3o8 = k3b && shapes_[op.out].fp8 && opt_.fp8_3x3_out && op.res < 0;
  // the stream conv runs 1-4 workgroups per image (or image pair): only
  // worth it once the batch fills the CUs
  // 14x14x256 -> 7x7x512 / s2 (layer4.0.conv1) runs 2 rounds of single-image
  // workgroups with 49 of 64 fragment rows live: with the LDS weight ring and
  // the fused downsample 67.9 us vs 44.2 + 13.3 us as two implicit GEMMs; with
  // register weights 48.1 vs 13.2 + 46.3 us (profiles/r1_fused_ds.txt)
  const bool l4s2 = L.stride == 2 && is.H < 28 && !(opt_.stream_l4s2 && opt_.stream_wreg);
  const bool l1 = L.stride == 1 && is.C == 64;  // layer1: conv3x3_rows (the stream conv measured slower there)
  // layer2's stride-1 convs: one weight-stationary workgroup per image walking
  // its rows (59-60 us vs 62-66 us for the stream conv at B=256,
  // profiles/r2_rows28.txt), once the batch fills >= ~70% of one round
  const int rounds = (B + num_cus_ - 1) / num_cus_;
  // query batches: one launch per conv, no split-K (conv_small.hip)
  if (opt_.small_conv && k3 && L.wf_off && B <= kSmallConvMaxB &&
      conv_small_supported(is.H, is.W, is.C, L.cout, L.stride) &&
      !(opt_.direct13 && conv3x3_13_supported(is.H, is.W, is.C, L.cout)))  // (AlexNet keeps its fused pools)
    return ConvPath::Small;
  if (opt_.rows28 && (k3 || k3o8) && L.stride == 1 && L.wf_off && 10 * B >= 7 * rounds * num_cus_ &&
      conv3x3_rows28_supported(is.H, is.W, is.C, L.cout))
    return ConvPath::Rows28;
  if (opt_.direct13 && k3 && L.stride == 1 && L.wf_off && conv3x3_13_supported(is.H, is.W, is.C, L.cout))
    return ConvPath::Direct13;
  // e4m3 in and out (fp8_3x3_in): whole images per workgroup, once the batch
  // fills the CUs (query batches: the e4m3 implicit GEMM)
  if (L.fp8 && !L.fc && L.kh == 3 && L.kw == 3 && L.pad == 1 && L.wf_off && op.res < 0 && shapes_[op.out].fp8 &&
      4 * B >= num_cus_ && conv3x3_stream8_supported(is.H, is.W, is.C, L.cout, L.stride))
    return ConvPath::Stream8;
  if (opt_.direct27 && !L.fc && !L.fp8 && L.kh == 5 && L.kw == 5 && L.stride == 1 && L.relu && L.wf_off &&
      L.kpad == 1600 && !shapes_[op.out].f32 && conv5x5_27_supported(is.H, is.W, is.C, L.cout, L.pad))
    return ConvPath::Direct27;
  if (opt_.stream_conv && (k3 || k3o8) && !l4s2 && !l1 && 8 * B >= num_cus_ &&
      conv3x3_stream_supported(is.H, is.W, is.C, L.cout, L.stride))
    return ConvPath::Stream;
  if (opt_.row_conv && k3 && L.stride == 1 && conv3x3_rows_supported(is.H, is.W, is.C, L.cout)) return ConvPath::Rows;
  if (opt_.conv1x1 && !L.fc && L.kh == 1 && L.kw == 1) {
    ConvArgs a = conv_args(op, B, nullptr);
    a.split_k = 1;
    if (conv1x1_supported(a)) return ConvPath::OneByOne;
  }
  if (opt_.fc_gemm && L.fc && !L.fp8) {
    const ConvArgs a = conv_args(op, B, nullptr);
    if (fc_gemm_supported(a) && (size_t)B * L.npad <= ws_elems_) return ConvPath::Fc;
  }
  if (opt_.bigtile && conv_bigtile_pick(conv_args(op, B, nullptr), num_cus_) >= 0) return ConvPath::BigTile;
  return ConvPath::Igemm;
}

bool Engine::head_fusable(size_t oi) const {
  if (!opt_.fused_head || oi + 2 >= ops_.size()) return false;
  const Op& pool = ops_[oi];
  const Op& fc = ops_[oi + 1];
  const Op& sm = ops_[oi + 2];
  if (pool.type != OpType::AvgPoolGlobal || fc.type != OpType::Conv || sm.type != OpType::SoftmaxTop1) return false;
  if (fc.in != pool.out || sm.in != fc.out || !shapes_[fc.out].f32 || shapes_[pool.out].fp8) return false;
  const ConvLayer& L = convs_[fc.conv];
  // (an e4m3 pool input, ResNet50 fp8: pooled from e4m3 in the head, C >= 2048)
  if (shapes_[pool.in].fp8 && shapes_[pool.in].C < 2048) return false;
  return L.fc && !L.fp8 && !L.relu && L.cin == shapes_[pool.in].C && head_supported(L.cin, L.cout, L.kpad, L.npad);
}

// ops[oi] is the last conv (stream path, whole-image workgroups) and
// ops[oi+1] the global average pool, the only reader of its output: the
// conv's epilogue writes the pooled bf16 vectors straight into the pool's
// output activation and skips storing its own.
bool Engine::pool_fusable(size_t oi, int B) const {
  if (!opt_.fused_pool || oi + 1 >= ops_.size()) return false;
  const Op& c = ops_[oi];
  const Op& p = ops_[oi + 1];
  if (c.type != OpType::Conv || p.type != OpType::AvgPoolGlobal || p.in != c.out) return false;
  if (shapes_[p.out].fp8 || shapes_[p.out].f32 || shapes_[p.in].fp8) return false;
  for (size_t j = 0; j < ops_.size(); ++j)
    if (j != oi + 1 && (ops_[j].in == c.out || ops_[j].res == c.out)) return false;
  const ConvLayer& L = convs_[c.conv];
  const ActShape& is = shapes_[c.in];
  return !L.fp8 && !shapes_[c.out].fp8 && conv_path(c, B) == ConvPath::Stream &&
         conv3x3_stream_pool_supported(is.H, is.W, is.C, L.cout, L.stride);
}

// ops[oi] is a block's downsample (1x1/s2, BN, no ReLU) and ops[oi+1] the
// block's 3x3/s2 conv1 on the same input, run by the stream conv.
bool Engine::ds_fusable(size_t oi, int B) const {
  if (oi + 1 >= ops_.size()) return false;
  const Op& d = ops_[oi];
  const Op& c = ops_[oi + 1];
  if (d.type != OpType::Conv || c.type != OpType::Conv || d.in != c.in) return false;
  const ConvLayer& D = convs_[d.conv];
  const ConvLayer& L = convs_[c.conv];
  return !D.fc && !D.fp8 && D.kh == 1 && D.kw == 1 && D.stride == 2 && D.pad == 0 && !D.relu && d.res < 0 &&
         D.cout == L.cout && L.stride == 2 && !shapes_[d.out].fp8 && !shapes_[d.out].f32 &&
         (conv_path(c, B) == ConvPath::Stream || (conv_path(c, B) == ConvPath::Small && D.wf_off));
}

// ops[oi], ops[oi+1] = conv1 (+ReLU) and conv2 (+identity residual, ReLU) of
// a 56x56x64 basic block, both on the register-weight row conv, and conv1's
// output read by nothing else: conv3x3_block runs the pair with the
// intermediate kept in LDS (not written to its activation).
bool Engine::block_fusable(size_t oi, int B) const {
  if (!opt_.fused_block || !opt_.rows_wreg || oi + 1 >= ops_.size()) return false;
  // one workgroup per image walks all 56 rows (~100 us per round of num_cus
  // images at B=256 vs ~2 x 72 us for the two row convs, which split images
  // into strips): only worth it with rounds that are >= ~70% full (B=1: 86 us
  // fused vs ~30 us as strips; profiles/r2_block_kernel_stats.txt)
  const int rounds = (B + num_cus_ - 1) / num_cus_;
  if (10 * B < 7 * rounds * num_cus_) return false;
  const Op& c1 = ops_[oi];
  const Op& c2 = ops_[oi + 1];
  if (c1.type != OpType::Conv || c2.type != OpType::Conv || c2.in != c1.out || c1.res >= 0 || c2.res != c1.in)
    return false;
  if (c1.side || c2.side) return false;
  for (size_t j = 0; j < ops_.size(); ++j)
    if (j != oi + 1 && (ops_[j].in == c1.out || ops_[j].res == c1.out)) return false;
  const ConvLayer& L1 = convs_[c1.conv];
  const ConvLayer& L2 = convs_[c2.conv];
  const ActShape& is = shapes_[c1.in];
  return L1.relu && L2.relu && L1.wf_off && L2.wf_off && conv3x3_block_supported(is.H, is.W, is.C) &&
         L1.cout == is.C && L2.cout == is.C && !shapes_[c1.in].fp8 && !shapes_[c2.out].fp8 &&
         conv_path(c1, B) == ConvPath::Rows && conv_path(c2, B) == ConvPath::Rows;
}

// A resnet50_fp8 layer1 identity bottleneck's expand conv (1x1, 64 -> 256 on
// 56x56, bf16 in, e4m3 out): bottleneck56.hip reads its weights in fragment order.
bool Engine::bottleneck_conv3(const ConvLayer& L) const {
  if (L.fc || L.fp8 || L.pair || L.stem_pool || L.in_act < 0 || L.kh != 1 || L.kw != 1 || L.stride != 1) return false;
  const ActShape& is = shapes_[L.in_act];
  return fp8_ && is.C == 64 && L.cout == 256 && L.kpad == 64 && bottleneck56_supported(is.H, is.W, 256, 64);
}

// ops[oi..oi+2] = conv1 (1x1 256 -> 64, e4m3 in) + conv2 (3x3 64 -> 64) +
// conv3 (1x1 64 -> 256 + the block input as residual, e4m3 out) of a
// resnet50_fp8 layer1 identity block, the intermediates read by nothing else.
bool Engine::bottleneck_fusable(size_t oi) const {
  if (!opt_.fused_bottleneck || !fp8_ || oi + 2 >= ops_.size()) return false;
  const Op& c1 = ops_[oi];
  const Op& c2 = ops_[oi + 1];
  const Op& c3 = ops_[oi + 2];
  if (c1.type != OpType::Conv || c2.type != OpType::Conv || c3.type != OpType::Conv) return false;
  if (c1.side || c2.side || c3.side || c2.in != c1.out || c3.in != c2.out || c1.res >= 0 || c2.res >= 0 ||
      c3.res != c1.in)
    return false;
  const ConvLayer& L1 = convs_[c1.conv];
  const ConvLayer& L2 = convs_[c2.conv];
  const ConvLayer& L3 = convs_[c3.conv];
  const ActShape& xs = shapes_[c1.in];
  if (!xs.fp8 || !shapes_[c3.out].fp8 || shapes_[c1.out].fp8 || shapes_[c2.out].fp8) return false;
  if (!bottleneck56_supported(xs.H, xs.W, xs.C, L1.cout) || !L1.fp8 || L1.kh != 1 || L1.stride != 1 || !L1.relu ||
      L1.kpad != 256 || L1.npad != 64)
    return false;
  if (L2.kh != 3 || L2.kw != 3 || L2.stride != 1 || L2.pad != 1 || !L2.relu || L2.cout != 64 || !L2.wf_off ||
      L2.kpad != 576)
    return false;
  if (!bottleneck_conv3(L3) || !L3.wf_off || !L3.relu) return false;
  for (size_t j = 0; j < ops_.size(); ++j) {
    if (j != oi + 1 && (ops_[j].in == c1.out || ops_[j].res == c1.out)) return false;
    if (j != oi + 2 && (ops_[j].in == c2.out || ops_[j].res == c2.out)) return false;
  }
  return true;
}

bool Engine::bottleneck_head_fusable(size_t oi) const {
  if (!opt_.fused_bottleneck || oi + 1 >= ops_.size()) return false;
  const Op& c1 = ops_[oi];
  const Op& c2 = ops_[oi + 1];
  if (c1.type != OpType::Conv || c2.type != OpType::Conv || c1.side || c2.side || c2.in != c1.out || c1.res >= 0 ||
      c2.res >= 0)
    return false;
  const ConvLayer& L1 = convs_[c1.conv];
  const ConvLayer& L2 = convs_[c2.conv];
  const ActShape& xs = shapes_[c1.in];
  if (xs.fp8 || xs.f32 || shapes_[c1.out].fp8 || shapes_[c2.out].fp8 || shapes_[c2.out].f32) return false;
  if (!bottleneck56_supported(xs.H, xs.W, 256, 64) || xs.C != 64) return false;
  if (L1.fc || L1.fp8 || L1.pair || L1.stem_pool || L1.kh != 1 || L1.kw != 1 || L1.stride != 1 || !L1.relu ||
      L1.cout != 64 || L1.kpad != 64 || L1.npad != 64)
    return false;
  if (L2.fp8 || L2.kh != 3 || L2.kw != 3 || L2.stride != 1 || L2.pad != 1 || !L2.relu || L2.cout != 64 ||
      !L2.wf_off || L2.kpad != 576)
    return false;
  for (size_t j = 0; j < ops_.size(); ++j)
    if (j != oi + 1 && (ops_[j].in == c1.out || ops_[j].res == c1.out)) return false;
  return true;
}

// ops[oi] is a downsample whose only reader is a later expand conv that
// computes it itself (its cat_ds): that op's index, else -1.
int Engine::ds_expand_op(size_t oi) const {
  if (!opt_.ds_into_expand || ops_[oi].type != OpType::Conv) return -1;
  const Op& d = ops_[oi];
  int reader = -1;
  for (size_t j = 0; j < ops_.size(); ++j) {
    if (j == oi) continue;
    if (ops_[j].in == d.out) return -1;
    if (ops_[j].res == d.out) {
      if (reader >= 0) return -1;
      reader = (int)j;
    }
  }
  if (reader < 0) return -1;
  const ConvLayer& L3 = convs_[ops_[reader].conv];
  if (L3.cat_ds != d.conv || !L3.cat_off) return -1;
  ConvArgs a = conv_args(ops_[reader], 1, nullptr);
  a.split_k = 1;
  a.res = nullptr;
  a.x2 = acts_.empty() ? (const void*)16 : acts_[d.in];
  a.cin2 = convs_[d.conv].cin;
  a.Kpad = L3.kpad + convs_[d.conv].kpad;
  return conv1x1_supported(a) ? reader : -1;
}

// The stride-2 conv1 of a block whose downsample it computes (fuse_ds) on
// the 56x56x64 -> 128 shape: conv3x3_s2rows runs one workgroup per image
// (59 us at B=256 vs 72 us for the stream conv's 4 rounds of strips,
// profiles/r2_s2rows.txt); like the fused block only with rounds >= ~70% full.
// ops[oi] = layer2.0.conv1 on conv3x3_s2rows (its downsample = ops[oi - 1]);
// the block's conv2 (ops[oi + 1], on conv3x3_rows28) can compute that
// downsample as 2 more K steps when it is the downsample output's only reader.
bool Engine::ds_conv2_ok(size_t oi, int B) const {
  if (!opt_.ds_into_conv2 || oi < 1 || oi + 1 >= ops_.size()) return false;
  const Op& d = ops_[oi - 1];
  const Op& c2 = ops_[oi + 1];
  if (c2.type != OpType::Conv || c2.res != d.out || c2.in != ops_[oi].out) return false;
  const ConvLayer& L2 = convs_[c2.conv];
  const ConvLayer& D = convs_[d.conv];
  if (!L2.wf_off || !D.wf_off || L2.fp8 || shapes_[c2.out].fp8 || conv_path(c2, B) != ConvPath::Rows28) return false;
  const ActShape& xs = shapes_[d.in];
  if (xs.H != 56 || xs.W != 56 || xs.C != 64 || xs.fp8 || xs.f32 || L2.cout != 128 || D.cout != 128) return false;
  for (size_t j = 0; j < ops_.size(); ++j)
    if (j != oi + 1 && (ops_[j].in == d.out || ops_[j].res == d.out)) return false;
  return true;
}

// ops[oi] is a bottleneck's expand conv (1x1, residual) and ops[oi + 1] the
// next bottleneck's reduce conv on its output, both on conv1x1.hip, in a form
// conv1x1_chain runs as one launch (ResNet50 e4m3 layer2.0-2.2 -> 2.1-2.3).
// The expand output keeps its other reader (the next expand's residual).
bool Engine::chain_ok(size_t oi, int B) const {
  if (!opt_.chain_1x1 || oi + 1 >= ops_.size() || acts_.empty()) return false;
  const Op& e = ops_[oi];
  const Op& r = ops_[oi + 1];
  if (e.type != OpType::Conv || r.type != OpType::Conv || e.res < 0 || r.in != e.out || r.res >= 0 || e.side ||
      r.side)
    return false;
  if (conv_path(e, B) != ConvPath::OneByOne || conv_path(r, B) != ConvPath::OneByOne) return false;
  if (convs_[e.conv].cat_off) return false;  // (an expand with its downsample as a second K block)
  ConvArgs a = conv_args(e, B, nullptr), ra = conv_args(r, B, nullptr);
  a.split_k = ra.split_k = 1;
  return conv1x1_chain_supported(a, ra);
}

bool Engine::s2rows_ok(const Op& op, const ConvLayer& D, int B) const {
  const ConvLayer& L = convs_[op.conv];
  const ActShape& is = shapes_[op.in];
  const int rounds = (B + num_cus_ - 1) / num_cus_;
  return opt_.s2rows && op.res < 0 && L.wf_off && D.wf_off && 10 * B >= 7 * rounds * num_cus_ &&
         conv3x3_s2rows_supported(is.H, is.W, is.C, L.cout);
}

bool Engine::side_safe(int B) const {
  for (const Op& op : ops_)
    if (op.type == OpType::Conv && conv_path(op, B) == ConvPath::BigTile) return false;
  return true;
}

void Engine::run_ops(const uint8_t* images, int B, int Hin, int Win, int32_t* idx, float* prob,
                     float* logits, hipStream_t s, std::vector<hipEvent_t>* evs, bool trace) {
  size_t ei = 0;
  if (evs) DMLC_HIP_CHECK(hipEventRecord((*evs)[ei++], s));
  // per-op event timing keeps every op on one stream
  const bool side_ready = opt_.fork_ds && !evs && side_safe(B);
  std::map<int, hipEvent_t> joined;  // activation -> event its side-stream producer recorded
  int skip = 0;                      // ops already done by a fused kernel
  int skip_ds = -1;                  // downsample op left to the next (stream) conv
  int ds_conv2 = -1;                 // downsample op left to the block's conv2 (ds_into_conv2)
  bool pooled = false;               // the last conv wrote pooled_ (fused avgpool)
  for (size_t oi = 0; oi < ops_.size(); ++oi) {
    const Op& op = ops_[oi];
    if (skip > 0) {
      --skip;
      if (evs) DMLC_HIP_CHECK(hipEventRecord((*evs)[ei++], s));
      continue;
    }
    std::optional<TraceRange> tr;  // per-op host ranges (not inside a graph capture)
    if (trace) tr.emplace(op.name.c_str());
    switch (op.type) {
      case OpType::Preprocess: {
        const bool paired = op.k == 1;
        // AlexNet: 224x224 u8 images -> features.2's output in one kernel
        if (oi + 2 < ops_.size() && ops_[oi + 1].type == OpType::Conv && ops_[oi + 2].type == OpType::MaxPool &&
            convs_[ops_[oi + 1].conv].alex_stem && opt_.fused_preprocess && Hin == image_size_ &&
            Win == image_size_) {
          const ConvLayer& L = convs_[ops_[oi + 1].conv];
          const uint8_t* wa = (const uint8_t*)warena_;
          alex_stem_u8(images, wa + L.wf_off, (const float*)(wa + L.b_off), acts_[ops_[oi + 2].out], B, s);
          skip = 2;
          break;
        }
        // images already SxS feed the fused stem directly (stem_conv_pool_u8)
        if (paired && opt_.fused_preprocess && Hin == image_size_ && Win == image_size_) break;
        const int Wr = paired ? 2 * shapes_[op.out].W : shapes_[op.out].W;
        preprocess_u8(images, acts_[op.out], B, Hin, Win, image_size_, op.pad, Wr, s, paired);
        break;
      }
      case OpType::Conv: {
        const ConvLayer& L = convs_[op.conv];
        const ActShape& is = shapes_[op.in];
        // A downsample conv runs on the side stream, concurrently with its
        // block's conv1 (both read the block input; conv2 joins them through
        // the residual). Never next to a big-tile conv: its split-K slices
        // spin on each other and need their CUs.
        if (ds_expand_op(oi) >= 0) break;  // computed by its expand conv (conv1x1 x2)
        if (opt_.fuse_ds && op.side && ds_fusable(oi, B)) {
          skip_ds = (int)oi;  // computed by the next op (the block's stride-2 conv1)
          break;
        }
        hipStream_t cs = s;
        if (side_ready && op.side) {
          DMLC_HIP_CHECK(hipEventRecord(fork_evs_[oi], s));
          DMLC_HIP_CHECK(hipStreamWaitEvent(side_, fork_evs_[oi], 0));
          cs = side_;
        }
        if (op.res >= 0 && joined.count(op.res)) {
          DMLC_HIP_CHECK(hipStreamWaitEvent(s, joined[op.res], 0));
          joined.erase(op.res);
        }
        if (L.fc && !L.fp8 && !shapes_[op.out].fp8 && opt_.fc_small && fc_small_supported(B, L.cin, L.cin, L.kpad)) {
          // query-sized batches: weight-streaming GEMV (AlexNet classifier)
          const ActShape& os = shapes_[op.out];
          fc_small(acts_[op.in], L.cin, (const uint8_t*)warena_ + L.w_off, L.kpad,
                   (const float*)((const uint8_t*)warena_ + L.b_off),
                   (os.f32 && logits) ? (void*)logits : acts_[op.out], L.cout, os.f32, B, L.cin, L.cout, L.npad,
                   L.relu, cs);
          break;
        }
        if (L.cat_off && op.res >= 0) {
          // expand conv + its stride-1 downsample as one K-concatenated GEMM
          int ds_op = -1;
          for (size_t i = 0; i < oi; ++i)
            if (ops_[i].type == OpType::Conv && ops_[i].conv == L.cat_ds && ds_expand_op(i) == (int)oi) ds_op = (int)i;
          if (ds_op >= 0) {
            if (joined.count(op.res)) joined.erase(op.res);
            ConvArgs a = conv_args(op, B, logits);
            const ConvLayer& D = convs_[L.cat_ds];
            a.split_k = 1;
            a.res = nullptr;
            a.x2 = acts_[ops_[ds_op].in];
            a.cin2 = D.cin;
            a.Kpad = L.kpad + D.kpad;
            a.w = (const uint8_t*)warena_ + L.cat_off;
            a.bias = (const float*)((const uint8_t*)warena_ + L.cat_b_off);
            conv1x1(a, num_cus_, cs);
            break;
          }
        }
        if (cs == s && chain_ok(oi, B)) {
          ConvArgs a = conv_args(op, B, logits), ra = conv_args(ops_[oi + 1], B, logits);
          a.split_k = ra.split_k = 1;
          conv1x1_chain(a, ra, num_cus_, cs);
          skip = 1;
          break;
        }
        if (cs == s && bottleneck_fusable(oi)) {
          const ConvLayer& L2 = convs_[ops_[oi + 1].conv];
          const ConvLayer& L3 = convs_[ops_[oi + 2].conv];
          const uint8_t* wa = (const uint8_t*)warena_;
          bottleneck56(acts_[op.in], wa + L.w_off, (const float*)(wa + L.a_off), (const float*)(wa + L.b_off),
                       wa + L2.wf_off, (const float*)(wa + L2.b_off), wa + L3.wf_off, (const float*)(wa + L3.b_off),
                       acts_[ops_[oi + 2].out], shapes_[op.in].scale, 1.f / shapes_[ops_[oi + 2].out].scale, B, s);
          skip = 2;
          break;
        }
        if (cs == s && bottleneck_head_fusable(oi)) {
          const ConvLayer& L2 = convs_[ops_[oi + 1].conv];
          const uint8_t* wa = (const uint8_t*)warena_;
          bottleneck56_head(acts_[op.in], wa + L.w_off, (const float*)(wa + L.b_off), wa + L2.wf_off,
                            (const float*)(wa + L2.b_off), acts_[ops_[oi + 1].out], B, s);
          skip = 1;
          break;
        }
        if (cs == s && block_fusable(oi, B)) {
          const ConvLayer& L2 = convs_[ops_[oi + 1].conv];
          const uint8_t* wa = (const uint8_t*)warena_;
          conv3x3_block(acts_[op.in], wa + L.wf_off, (const float*)(wa + L.b_off), wa + L2.wf_off,
                        (const float*)(wa + L2.b_off), acts_[ops_[oi + 1].out], zero_, B, s);
          skip = 1;
          break;
        }
        switch (conv_path(op, B)) {
          case ConvPath::Stream: {
            const ConvLayer* D = nullptr;
            int yd = -1;
            if (skip_ds >= 0 && skip_ds + 1 == (int)oi) {
              D = &convs_[ops_[skip_ds].conv];
              yd = ops_[skip_ds].out;
            }
            // the fused avgpool keeps the activation for eager/profile runs
            // (tests read it) and drops it under graph capture
            const bool fpool = cs == s && pool_fusable(oi, B);
            if (D && s2rows_ok(op, *D, B)) {
              const uint8_t* wa = (const uint8_t*)warena_;
              if (ds_conv2_ok(oi, B)) {  // the downsample runs inside conv2
                conv3x3_s2rows(acts_[op.in], wa + L.wf_off, (const float*)(wa + L.b_off), nullptr, nullptr,
                               acts_[op.out], nullptr, zero_, B, L.relu, cs);
                ds_conv2 = skip_ds;
              } else {
                conv3x3_s2rows(acts_[op.in], wa + L.wf_off, (const float*)(wa + L.b_off), wa + D->wf_off,
                               (const float*)(wa + D->b_off), acts_[op.out], acts_[yd], zero_, B, L.relu, cs);
              }
              skip_ds = -1;
              break;
            }
            if (!D && opt_.s2rows128 && op.res < 0 && L.wf_off && L.stride == 2 &&
                10 * B >= 7 * ((B + num_cus_ - 1) / num_cus_) * num_cus_ &&
                conv3x3_s2rows128_supported(is.H, is.W, is.C, L.cout)) {
              const uint8_t* wa = (const uint8_t*)warena_;
              conv3x3_s2rows128(acts_[op.in], wa + L.wf_off, (const float*)(wa + L.b_off), acts_[op.out], B, L.relu,
                                shapes_[op.out].fp8 ? 1.f / shapes_[op.out].scale : 0.f, cs);
              skip_ds = -1;
              break;
            }
            // (wf_off may exist for conv3x3_s2rows alone)
            const bool wreg = L.wf_off && opt_.stream_wreg && (!D || D->wf_off) &&
                              conv3x3_stream_uses_frag(is.H, is.W, is.C, L.cout, L.stride);
            conv3x3_stream(acts_[op.in], (const uint8_t*)warena_ + L.w_off,
                           (const float*)((const uint8_t*)warena_ + L.b_off), op.res >= 0 ? acts_[op.res] : nullptr,
                           acts_[op.out], zero_, B, is.H, is.W, is.C, L.cout, L.stride, L.relu, cs, nullptr,
                           D ? (const uint8_t*)warena_ + D->w_off : nullptr,
                           D ? (const float*)((const uint8_t*)warena_ + D->b_off) : nullptr,
                           D ? acts_[yd] : nullptr, wreg ? (const uint8_t*)warena_ + L.wf_off : nullptr,
                           (wreg && D) ? (const uint8_t*)warena_ + D->wf_off : nullptr,
                           fpool ? acts_[ops_[oi + 1].out] : nullptr, !fpool || trace || evs,
                           shapes_[op.out].fp8 ? 1.f / shapes_[op.out].scale : 0.f);
            pooled = fpool;
            skip_ds = -1;
            break;
          }
          case ConvPath::Direct13: {
            // AlexNet features.10 + features.12: the 3x3/s2 max-pool in the
            // conv's epilogue when the pool is the conv output's only reader
            void* ypool = nullptr;
            if (opt_.fused_pool && cs == s && oi + 1 < ops_.size() && L.relu &&
                conv3x3_13_pool_supported(is.C, L.cout)) {
              const Op& mp = ops_[oi + 1];
              bool only = mp.type == OpType::MaxPool && mp.in == op.out && mp.k == 3 && mp.stride == 2 &&
                          mp.pad == 0 && shapes_[mp.out].H == 6 && shapes_[mp.out].W == 6;
              for (size_t j = 0; only && j < ops_.size(); ++j)
                if (j != oi + 1 && (ops_[j].in == op.out || ops_[j].res == op.out)) only = false;
              if (only) {
                ypool = acts_[mp.out];
                skip = 1;
              }
            }
            conv3x3_13(acts_[op.in], (const uint8_t*)warena_ + L.wf_off,
                       (const float*)((const uint8_t*)warena_ + L.b_off), acts_[op.out], zero_, B, is.C, L.cout,
                       L.relu, cs, ypool);
            break;
          }
          case ConvPath::Direct27: {
            // AlexNet features.3 + features.5: the max-pool in the conv's epilogue
            void* ypool = nullptr;
            if (opt_.fused_pool && cs == s && oi + 1 < ops_.size()) {
              const Op& mp = ops_[oi + 1];
              bool only = mp.type == OpType::MaxPool && mp.in == op.out && mp.k == 3 && mp.stride == 2 &&
                          mp.pad == 0 && shapes_[mp.out].H == 13 && shapes_[mp.out].W == 13;
              for (size_t j = 0; only && j < ops_.size(); ++j)
                if (j != oi + 1 && (ops_[j].in == op.out || ops_[j].res == op.out)) only = false;
              if (only) {
                ypool = acts_[mp.out];
                skip = 1;
              }
            }
            conv5x5_27(acts_[op.in], (const uint8_t*)warena_ + L.wf_off,
                       (const float*)((const uint8_t*)warena_ + L.b_off), acts_[op.out], zero_, B, cs, ypool);
            break;
          }
          case ConvPath::Small: {
            const uint8_t* wa = (const uint8_t*)warena_;
            const ConvLayer* D = nullptr;
            int yd = -1;
            if (skip_ds >= 0 && skip_ds + 1 == (int)oi) {
              D = &convs_[ops_[skip_ds].conv];
              yd = ops_[skip_ds].out;
            }
            conv_small(acts_[op.in], wa + L.wf_off, (const float*)(wa + L.b_off), op.res >= 0 ? acts_[op.res] : nullptr,
                       acts_[op.out], B, is.H, is.W, is.C, L.cout, L.stride, L.relu,
                       conv_small_pick_mf(B, is.H, is.W, is.C, L.cout, L.stride, num_cus_), cs,
                       D ? wa + D->wf_off : nullptr, D ? (const float*)(wa + D->b_off) : nullptr,
                       D ? acts_[yd] : nullptr);
            skip_ds = -1;
            break;
          }
          case ConvPath::Stream8: {
            const uint8_t* wa = (const uint8_t*)warena_;
            conv3x3_stream8(acts_[op.in], wa + L.wf_off, (const float*)(wa + L.a_off), (const float*)(wa + L.b_off),
                            acts_[op.out], zero_, B, is.H, is.W, is.C, L.cout, L.stride, L.relu,
                            1.f / shapes_[op.out].scale, cs);
            break;
          }
          case ConvPath::Rows28:
            if (ds_conv2 >= 0 && op.res == ops_[ds_conv2].out) {
              const ConvLayer& D = convs_[ops_[ds_conv2].conv];
              const uint8_t* wa = (const uint8_t*)warena_;
              conv3x3_rows28(acts_[op.in], wa + L.wf_off, (const float*)(wa + L.b_off), nullptr, acts_[op.out], B,
                             L.relu, cs, 0.f, acts_[ops_[ds_conv2].in], wa + D.wf_off,
                             (const float*)(wa + D.b_off));
              ds_conv2 = -1;
              break;
            }
            conv3x3_rows28(acts_[op.in], (const uint8_t*)warena_ + L.wf_off,
                           (const float*)((const uint8_t*)warena_ + L.b_off), op.res >= 0 ? acts_[op.res] : nullptr,
                           acts_[op.out], B, L.relu, cs, shapes_[op.out].fp8 ? 1.f / shapes_[op.out].scale : 0.f);
            break;
          case ConvPath::Rows:
            conv3x3_rows(acts_[op.in], (const uint8_t*)warena_ + L.w_off,
                         (const float*)((const uint8_t*)warena_ + L.b_off), op.res >= 0 ? acts_[op.res] : nullptr,
                         acts_[op.out], zero_, B, is.H, is.W, is.C, L.relu,
                         conv3x3_rows_pick_strip(B, is.H, (L.wf_off && opt_.rows_wreg) ? 2 * num_cus_ : num_cus_),
                         cs,
                         (L.wf_off && opt_.rows_wreg) ? (const uint8_t*)warena_ + L.wf_off : nullptr);
            break;
          case ConvPath::OneByOne: {
            ConvArgs a = conv_args(op, B, logits);
            a.split_k = 1;
            conv1x1(a, num_cus_, cs);
            break;
          }
          case ConvPath::BigTile: {
            const ConvArgs a = conv_args(op, B, logits);
            const int bt = conv_bigtile_pick(a, num_cus_);
            int splits = conv_bigtile_splits(a, bt, num_cus_);
            if (conv_bigtile_ws_bytes(conv_bigtile_slabs(a, bt, splits)) > bt_ws_bytes_) splits = 1;
            conv2d_bigtile(a, bt, splits, bt_ws_, bt_ws_bytes_, cs);
            break;
          }
          case ConvPath::Igemm: {
            ConvArgs a = conv_args(op, B, logits);
            if (cs != s) a.split_k = 1;  // the split-K workspace belongs to the main stream
            conv2d_igemm(a, cs);
            break;
          }
          case ConvPath::Fc: {
            ConvArgs a = conv_args(op, B, logits);
            if (cs != s) {  // (its partials need the main stream's split-K workspace)
              a.split_k = 1;
              conv2d_igemm(a, cs);
              break;
            }
            int sp = fc_gemm_splits(a, num_cus_);
            while (sp > 1 && ((size_t)sp * B * a.Npad > ws_elems_ || (a.Kpad / 64) % sp)) --sp;
            a.ws = ws_;
            fc_gemm(a, sp, cs);
            break;
          }
        }
        if (cs != s) {
          DMLC_HIP_CHECK(hipEventRecord(join_evs_[oi], side_));
          joined[op.out] = join_evs_[oi];
        }
        break;
      }
      case OpType::StemPool: {
        const ConvLayer& L = convs_[op.conv];
        if (opt_.fused_preprocess && Hin == image_size_ && Win == image_size_) {
          stem_conv_pool_u8(images, (const uint8_t*)warena_ + L.w_off,
                            (const float*)((const uint8_t*)warena_ + L.b_off), acts_[op.out], B, image_size_,
                            opt_.stem_roles ? stem_pool_u8_pick_strip(B, shapes_[op.out].H, num_cus_)
                                            : stem_pool_pick_strip(B, shapes_[op.out].H, num_cus_),
                            s, opt_.stem_dense && L.wf_off ? (const uint8_t*)warena_ + L.wf_off : nullptr);
          break;
        }
        stem_conv_pool(acts_[op.in], (const uint8_t*)warena_ + L.w_off,
                       (const float*)((const uint8_t*)warena_ + L.b_off), acts_[op.out], B, image_size_,
                       shapes_[op.in].W, stem_pool_pick_strip(B, shapes_[op.out].H, num_cus_), s);
        break;
      }
      case OpType::MaxPool: {
        const ActShape& i = shapes_[op.in];
        const ActShape& o = shapes_[op.out];
        maxpool2d(acts_[op.in], acts_[op.out], B, i.H, i.W, i.C, o.H, o.W, op.k, op.stride, op.pad, s);
        break;
      }
      case OpType::AvgPoolGlobal: {
        const ActShape& i = shapes_[op.in];
        if (pooled) {  // pooled by the last conv's epilogue
          if (head_fusable(oi)) {  // fc + softmax/top-1 in one launch
            const ConvLayer& L = convs_[ops_[oi + 1].conv];
            head_pooled(acts_[op.out], (const uint8_t*)warena_ + L.w_off,
                        (const float*)((const uint8_t*)warena_ + L.b_off), B, i.C, L.cout, L.kpad, L.npad,
                        logits ? logits : (float*)acts_[ops_[oi + 1].out], idx ? idx : dummy_idx_,
                        prob ? prob : (float*)(dummy_idx_ + max_batch_), head_ws_, head_ws_bytes_, num_cus_, s);
            skip = 2;
          }
          break;  // else the fc and softmax ops follow
        }
        if (head_fusable(oi) && B >= kPoolThenHeadB) {
          // throughput batches: pool once, then fc + softmax/top-1 on the
          // pooled rows (head_fused pools its images again in every class
          // split: resnet50_fp8 b256 86 us, 8 x 25.7 MB of e4m3 reads)
          const ConvLayer& L = convs_[ops_[oi + 1].conv];
          avgpool_global(acts_[op.in], acts_[op.out], B, i.H * i.W, i.C, s, i.fp8, i.scale);
          head_pooled(acts_[op.out], (const uint8_t*)warena_ + L.w_off,
                      (const float*)((const uint8_t*)warena_ + L.b_off), B, i.C, L.cout, L.kpad, L.npad,
                      logits ? logits : (float*)acts_[ops_[oi + 1].out], idx ? idx : dummy_idx_,
                      prob ? prob : (float*)(dummy_idx_ + max_batch_), head_ws_, head_ws_bytes_, num_cus_, s);
          skip = 2;
          break;
        }
        if (head_fusable(oi)) {  // avgpool + fc + softmax/top-1 in one launch
          const ConvLayer& L = convs_[ops_[oi + 1].conv];
          head_fused(acts_[op.in], (const uint8_t*)warena_ + L.w_off,
                     (const float*)((const uint8_t*)warena_ + L.b_off), B, i.H * i.W, i.C, L.cout, L.kpad, L.npad,
                     logits ? logits : (float*)acts_[ops_[oi + 1].out], idx ? idx : dummy_idx_,
                     prob ? prob : (float*)(dummy_idx_ + max_batch_), head_ws_, head_ws_bytes_, num_cus_, s, i.fp8,
                     i.scale);
          skip = 2;
          break;
        }
        avgpool_global(acts_[op.in], acts_[op.out], B, i.H * i.W, i.C, s, i.fp8, i.scale);
        break;
      }
      case OpType::AvgPoolAdaptive: {
        const ActShape& i = shapes_[op.in];
        const ActShape& o = shapes_[op.out];
        avgpool_adaptive(acts_[op.in], acts_[op.out], B, i.H, i.W, i.C, o.H, o.W, s);
        break;
      }
      case OpType::SoftmaxTop1: {
        const float* lg = logits ? logits : (const float*)acts_[op.in];
        softmax_top1(lg, B, num_classes_, num_classes_, idx ? idx : dummy_idx_,
                     prob ? prob : (float*)(dummy_idx_ + max_batch_), s);
        break;
      }
    }
    if (evs) DMLC_HIP_CHECK(hipEventRecord((*evs)[ei++], s));
  }
}

void Engine::forward(const uint8_t* images, int B, int Hin, int Win, int32_t* idx, float* prob,
                     float* logits, hipStream_t stream, bool use_graph) {
  if (B <= 0) return;
  if (B > max_batch_) throw std::invalid_argument("batch exceeds reserved max_batch");
  if (!images) throw std::invalid_argument("null images");
  DMLC_HIP_CHECK(hipSetDevice(device_));
  // Forwards share the activation arena: one on a different stream than the
  // previous forward is ordered after it (an event, only then).
  if (last_stream_valid_ && stream != last_stream_) DMLC_HIP_CHECK(hipStreamWaitEvent(stream, ev_out_, 0));
  if (use_graph) {
    // Replays go straight onto the caller's stream: no event hop to the
    // engine's stream and back (two cross-stream waits cost ~40 us of idle
    // GPU between back-to-back forwards: profiles/r1_graph_gap.txt). The
    // engine's own stream is only used to capture.
    GraphKey key{images, B, Hin, Win, idx, prob, logits};
    auto it = graphs_.find(key);
    if (it == graphs_.end()) {
      DMLC_HIP_CHECK(hipStreamSynchronize(stream));
      hipGraph_t g;
      DMLC_HIP_CHECK(hipStreamBeginCapture(stream_, hipStreamCaptureModeThreadLocal));
      run_ops(images, B, Hin, Win, idx, prob, logits, stream_, nullptr, false);
      DMLC_HIP_CHECK(hipStreamEndCapture(stream_, &g));
      hipGraphExec_t ex;
      DMLC_HIP_CHECK(hipGraphInstantiate(&ex, g, nullptr, nullptr, 0));
      DMLC_HIP_CHECK(hipGraphDestroy(g));
      it = graphs_.emplace(key, ex).first;
    }
    DMLC_TRACE("engine.forward(graph)");
    DMLC_HIP_CHECK(hipGraphLaunch(it->second, stream));
  } else {  // eager launches straight onto the caller's stream
    DMLC_TRACE("engine.forward");
    run_ops(images, B, Hin, Win, idx, prob, logits, stream, nullptr, true);
  }
  DMLC_HIP_CHECK(hipEventRecord(ev_out_, stream));
  last_stream_ = stream;
  last_stream_valid_ = true;
}

std::vector<std::pair<std::string, float>> Engine::profile(const uint8_t* images, int B, int Hin,
                                                           int Win, hipStream_t stream) {
  if (B > max_batch_) throw std::invalid_argument("batch exceeds reserved max_batch");
  DMLC_HIP_CHECK(hipSetDevice(device_));
  DMLC_HIP_CHECK(hipStreamSynchronize(stream));
  std::vector<hipEvent_t> evs(ops_.size() + 1);
  for (auto& e : evs) DMLC_HIP_CHECK(hipEventCreate(&e));
  run_ops(images, B, Hin, Win, nullptr, nullptr, nullptr, stream_, &evs, true);
  DMLC_HIP_CHECK(hipStreamSynchronize(stream_));
  std::vector<std::pair<std::string, float>> out;
  for (size_t i = 0; i < ops_.size(); ++i) {
    float ms = 0;
    DMLC_HIP_CHECK(hipEventElapsedTime(&ms, evs[i], evs[i + 1]));
    out.emplace_back(ops_[i].name, ms);
  }
  for (auto& e : evs) hipEventDestroy(e);
  return out;
}

}  // namespace dmlc
