// pybind11 module `_C`: the Python face of the native runtime.
//
// Device buffers cross the boundary as raw pointers (ints) plus a raw
// hipStream_t, so this module does not depend on PyTorch's HIP headers; the
// Python wrappers in `dmlc.ops` / `dmlc.runtime` pass `tensor.data_ptr()` and
// `torch.cuda.current_stream().cuda_stream`.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include "../serve/shard.h"
#include <pybind11/stl.h>

#include <map>

#include "../kernels/kernels.h"
#include "../runtime/engine.h"
#include "../runtime/jpeg.h"
#include "../runtime/ot_io.h"

namespace py = pybind11;
using namespace dmlc;

namespace {

template <typename T>
T* P(uintptr_t v) {
  return reinterpret_cast<T*>(v);
}
hipStream_t S(uintptr_t v) { return reinterpret_cast<hipStream_t>(v); }

WeightMap to_weight_map(const py::dict& d) {
  WeightMap w;
  for (auto item : d) {
    auto name = py::cast<std::string>(item.first);
    auto arr = py::array_t<float, py::array::c_style | py::array::forcecast>::ensure(item.second);
    if (!arr) throw std::invalid_argument("weight " + name + " is not convertible to float32");
    HostTensor h;
    for (py::ssize_t i = 0; i < arr.ndim(); ++i) h.shape.push_back(arr.shape(i));
    h.data.assign(arr.data(), arr.data() + arr.size());
    w.emplace(name, std::move(h));
  }
  return w;
}

py::dict from_weight_map(const WeightMap& w) {
  py::dict d;
  for (const auto& kv : w) {
    std::vector<py::ssize_t> shape(kv.second.shape.begin(), kv.second.shape.end());
    py::array_t<float> a(shape);
    std::copy(kv.second.data.begin(), kv.second.data.end(), a.mutable_data());
    d[py::str(kv.first)] = a;
  }
  return d;
}

}  // namespace

void bind_dp(py::module& m);  // py_dp.cpp

// {"fused_block": false, ...} -> EngineOptions (unknown names are errors)
static EngineOptions engine_options(const std::map<std::string, bool>& m) {
  EngineOptions o;
  for (const auto& kv : m)
    if (!o.set(kv.first, kv.second)) throw std::invalid_argument("unknown engine option: " + kv.first);
  return o;
}

PYBIND11_MODULE(_C, m) {
  m.doc() = "dmlc native runtime: CDNA4 HIP kernels, inference engine, .ot I/O";

  // ---------------------------------------------------------------- ops
  m.def("conv_kpad", &conv_kpad, py::arg("Cin"), py::arg("KH"), py::arg("KW"), py::arg("stem") = false);
  m.def("stem_row_width", &stem_row_width);
  m.def("conv_npad", &conv_npad);
  m.def("conv_out_dim", &conv_out_dim);
  m.def(
      "conv2d",
      [](uintptr_t x, uintptr_t w, uintptr_t bias, uintptr_t res, uintptr_t y, int B, int H, int W,
         int Cin, int KH, int KW, int stride, int pad, int N, int Npad, int Kpad, int ldo, bool relu,
         bool out_f32, int split_k, uintptr_t ws, int tile, uintptr_t zero, bool stem, int Ho, int Wo,
         int max_blocks, uintptr_t stream, bool in_fp8, bool out_fp8, uintptr_t alpha, float res_scale,
         float out_inv_scale, uintptr_t bt_ws, size_t bt_ws_bytes, int bt_splits) {
        ConvArgs a;
        a.x = P<void>(x);
        a.zero = P<void>(zero);
        a.stem = stem;
        a.w = P<void>(w);
        a.bias = P<float>(bias);
        a.res = P<void>(res);
        a.y = P<void>(y);
        a.B = B;
        a.H = H;
        a.W = W;
        a.Cin = Cin;
        a.KH = KH;
        a.KW = KW;
        a.stride = stride;
        a.pad = pad;
        a.Ho = Ho > 0 ? Ho : conv_out_dim(H, KH, stride, pad);
        a.Wo = Wo > 0 ? Wo : conv_out_dim(W, KW, stride, pad);
        a.N = N;
        a.Npad = Npad;
        a.Kpad = Kpad;
        a.ldo = ldo;
        a.relu = relu;
        a.out_f32 = out_f32;
        a.split_k = split_k;
        a.ws = P<float>(ws);
        a.tile = tile;
        a.persistent = max_blocks > 0;
        a.max_blocks = max_blocks;
        a.in_fp8 = in_fp8;
        a.out_fp8 = out_fp8;
        a.alpha = P<float>(alpha);
        a.res_scale = res_scale;
        a.out_inv_scale = out_inv_scale;
        if (tile == kConv1x1Tile) {  // weight-stationary 1x1 conv (conv1x1.hip)
          a.tile = -1;
          hipDeviceProp_t prop;
          int dev = 0;
          DMLC_HIP_CHECK(hipGetDevice(&dev));
          DMLC_HIP_CHECK(hipGetDeviceProperties(&prop, dev));
          conv1x1(a, prop.multiProcessorCount, S(stream));
          return;
        }
        if (tile == kConv1x1Tile + 2) {  // fully connected (fc_gemm.hip); split_k 0: fc_gemm_splits
          a.tile = -1;
          hipDeviceProp_t prop;
          int dev = 0;
          DMLC_HIP_CHECK(hipGetDevice(&dev));
          DMLC_HIP_CHECK(hipGetDeviceProperties(&prop, dev));
          fc_gemm(a, split_k > 0 ? split_k : fc_gemm_splits(a, prop.multiProcessorCount), S(stream));
          return;
        }
        if (tile == kConv1x1Tile + 1) {  // support query only (no launch): raises if unsupported
          a.tile = -1;
          if (!conv1x1_supported(a)) throw std::invalid_argument("conv1x1: unsupported shape");
          return;
        }
        if (tile == kConvBigTile0 + 2) {  // persistent 256x128 big tiles
          a.tile = -1;
          hipDeviceProp_t prop;
          int dev = 0;
          DMLC_HIP_CHECK(hipGetDevice(&dev));
          DMLC_HIP_CHECK(hipGetDeviceProperties(&prop, dev));
          conv2d_bigtile_persistent(a, max_blocks > 0 ? max_blocks : conv_bigtile_persistent_grid(a, prop.multiProcessorCount),
                                    S(stream));
          return;
        }
        if (tile >= kConvBigTile0) {  // 8-wave big-tile configs (conv_bigtile.hip)
          a.tile = -1;
          conv2d_bigtile(a, tile - kConvBigTile0, bt_splits, P<void>(bt_ws), bt_ws_bytes, S(stream));
          return;
        }
        conv2d_igemm(a, S(stream));
      },
      py::arg("x"), py::arg("w"), py::arg("bias"), py::arg("res"), py::arg("y"), py::arg("B"),
      py::arg("H"), py::arg("W"), py::arg("Cin"), py::arg("KH"), py::arg("KW"), py::arg("stride"),
      py::arg("pad"), py::arg("N"), py::arg("Npad"), py::arg("Kpad"), py::arg("ldo"),
      py::arg("relu"), py::arg("out_f32"), py::arg("split_k"), py::arg("ws"), py::arg("tile"),
      py::arg("zero"), py::arg("stem"), py::arg("Ho"), py::arg("Wo"), py::arg("max_blocks"),
      py::arg("stream"), py::arg("in_fp8") = false, py::arg("out_fp8") = false, py::arg("alpha") = 0,
      py::arg("res_scale") = 1.f, py::arg("out_inv_scale") = 1.f, py::arg("bt_ws") = 0, py::arg("bt_ws_bytes") = 0,
      py::arg("bt_splits") = 1);
  m.def("conv_bigtile_ws_bytes", &conv_bigtile_ws_bytes);
  m.def("conv_bigtile_ws_header_bytes", &conv_bigtile_ws_header_bytes);
  m.def(
      "conv_bigtile_splits",
      [](int B, int Ho, int Wo, int Npad, int Kpad, int cfg, int num_cus) {
        ConvArgs a;
        a.B = B;
        a.Ho = Ho;
        a.Wo = Wo;
        a.Npad = Npad;
        a.Kpad = Kpad;
        return conv_bigtile_splits(a, cfg, num_cus);
      });
  m.attr("CONV_BIGTILE0") = kConvBigTile0;
  m.attr("CONV_1X1") = kConv1x1Tile;
  m.attr("CONV_FC") = kConv1x1Tile + 2;
  m.def("fc_gemm_splits", [](int M, int Kpad, int Npad, int num_cus) {
    ConvArgs a;
    a.B = M;
    a.Kpad = Kpad;
    a.Npad = Npad;
    return fc_gemm_splits(a, num_cus);
  });
  m.def("maxpool2d", [](uintptr_t x, uintptr_t y, int B, int H, int W, int C, int k, int stride,
                        int pad, uintptr_t stream) {
    maxpool2d(P<void>(x), P<void>(y), B, H, W, C, conv_out_dim(H, k, stride, pad),
              conv_out_dim(W, k, stride, pad), k, stride, pad, S(stream));
  });
  m.def("avgpool_global", [](uintptr_t x, uintptr_t y, int B, int HW, int C, uintptr_t stream) {
    avgpool_global(P<void>(x), P<void>(y), B, HW, C, S(stream));
  });
  m.def("avgpool_adaptive", [](uintptr_t x, uintptr_t y, int B, int H, int W, int C, int Ho, int Wo,
                               uintptr_t stream) {
    avgpool_adaptive(P<void>(x), P<void>(y), B, H, W, C, Ho, Wo, S(stream));
  });
  m.def(
      "preprocess_u8",
      [](uintptr_t x, uintptr_t y, int B, int Hin, int Win, int S_, int pad, int Wr, uintptr_t stream,
         bool paired) { preprocess_u8(P<uint8_t>(x), P<void>(y), B, Hin, Win, S_, pad, Wr, S(stream), paired); },
      py::arg("x"), py::arg("y"), py::arg("B"), py::arg("Hin"), py::arg("Win"), py::arg("S"), py::arg("pad"),
      py::arg("Wr"), py::arg("stream"), py::arg("paired") = false);
  m.attr("STEM_POOL_K") = kStemPoolK;
  m.def("stem_pool_pick_strip", &stem_pool_pick_strip);
  m.def("stem_pool_u8_pick_strip", &stem_pool_u8_pick_strip);
  m.def("conv3x3_stream_supported", &conv3x3_stream_supported, py::arg("Hin"), py::arg("Win"), py::arg("Cin"),
        py::arg("Cout"), py::arg("stride") = 1);
  m.def("conv3x3_stream", [](uintptr_t x, uintptr_t w, uintptr_t bias, uintptr_t res, uintptr_t y, uintptr_t zero,
                             int B, int H, int W, int Cin, int Cout, int stride, bool relu, uintptr_t stream,
                             uintptr_t stamps, uintptr_t wd, uintptr_t bd, uintptr_t yd, uintptr_t wfrag,
                             uintptr_t wdfrag) {
    conv3x3_stream(P<void>(x), P<void>(w), P<float>(bias), P<void>(res), P<void>(y), P<void>(zero), B, H, W, Cin, Cout,
                   stride, relu, S(stream), P<unsigned long long>(stamps), P<void>(wd), P<float>(bd), P<void>(yd),
                   P<void>(wfrag), P<void>(wdfrag));
  }, py::arg("x"), py::arg("w"), py::arg("bias"), py::arg("res"), py::arg("y"), py::arg("zero"), py::arg("B"),
        py::arg("H"), py::arg("W"), py::arg("Cin"), py::arg("Cout"), py::arg("stride"), py::arg("relu"),
        py::arg("stream"), py::arg("stamps") = 0, py::arg("wd") = 0, py::arg("bd") = 0, py::arg("yd") = 0,
        py::arg("wfrag") = 0, py::arg("wdfrag") = 0);
  m.def("conv3x3_stream_uses_frag", &conv3x3_stream_uses_frag);
  m.def("conv3x3_stream_set_variant", &conv3x3_stream_set_variant);
  m.def("conv3x3_rows_supported", &conv3x3_rows_supported);
  m.def("conv3x3_rows_pick_strip", &conv3x3_rows_pick_strip);
  m.def("conv3x3_rows", [](uintptr_t x, uintptr_t w, uintptr_t bias, uintptr_t res, uintptr_t y, uintptr_t zero,
                           int B, int H, int W, int C, bool relu, int strip, uintptr_t stream, uintptr_t wfrag) {
    conv3x3_rows(P<void>(x), P<void>(w), P<float>(bias), P<void>(res), P<void>(y), P<void>(zero), B, H, W, C, relu,
                 strip, S(stream), P<void>(wfrag));
  }, py::arg("x"), py::arg("w"), py::arg("bias"), py::arg("res"), py::arg("y"), py::arg("zero"), py::arg("B"),
        py::arg("H"), py::arg("W"), py::arg("C"), py::arg("relu"), py::arg("strip"), py::arg("stream"),
        py::arg("wfrag") = 0);
  m.def("conv3x3_block_supported", &conv3x3_block_supported);
  m.def("conv3x3_block", [](uintptr_t x, uintptr_t wf1, uintptr_t b1, uintptr_t wf2, uintptr_t b2, uintptr_t y,
                            uintptr_t zero, int B, uintptr_t stream) {
    conv3x3_block(P<void>(x), P<void>(wf1), P<float>(b1), P<void>(wf2), P<float>(b2), P<void>(y), P<void>(zero), B,
                  S(stream));
  }, py::arg("x"), py::arg("wf1"), py::arg("b1"), py::arg("wf2"), py::arg("b2"), py::arg("y"), py::arg("zero"),
        py::arg("B"), py::arg("stream"));
  m.def("bottleneck56", [](uintptr_t x, uintptr_t w1, uintptr_t a1, uintptr_t b1, uintptr_t wf2, uintptr_t b2,
                           uintptr_t wf3, uintptr_t b3, uintptr_t y, float res_scale, float out_inv_scale, int B,
                           uintptr_t stream) {
    bottleneck56(P<void>(x), P<void>(w1), P<float>(a1), P<float>(b1), P<void>(wf2), P<float>(b2), P<void>(wf3),
                 P<float>(b3), P<void>(y), res_scale, out_inv_scale, B, S(stream));
  }, py::arg("x"), py::arg("w1"), py::arg("a1"), py::arg("b1"), py::arg("wf2"), py::arg("b2"), py::arg("wf3"),
     py::arg("b3"), py::arg("y"), py::arg("res_scale"), py::arg("out_inv_scale"), py::arg("B"), py::arg("stream") = 0);
  m.def("conv3x3_stream8_supported", &conv3x3_stream8_supported);
  m.def("conv3x3_stream8_frag_offset", &conv3x3_stream8_frag_offset);
  m.def("conv3x3_stream8_set_variant", &conv3x3_stream8_set_variant);
  m.def("conv3x3_stream8", [](uintptr_t x, uintptr_t wf, uintptr_t alpha, uintptr_t bias, uintptr_t y, uintptr_t zero,
                              int B, int H, int W, int Cin, int Cout, int stride, bool relu, float out_inv_scale,
                              uintptr_t stream) {
    conv3x3_stream8(P<void>(x), P<void>(wf), P<float>(alpha), P<float>(bias), P<void>(y), P<void>(zero), B, H, W, Cin,
                    Cout, stride, relu, out_inv_scale, S(stream));
  }, py::arg("x"), py::arg("wf"), py::arg("alpha"), py::arg("bias"), py::arg("y"), py::arg("zero"), py::arg("B"),
        py::arg("H"), py::arg("W"), py::arg("Cin"), py::arg("Cout"), py::arg("stride"), py::arg("relu"),
        py::arg("out_inv_scale"), py::arg("stream") = 0);
  m.def("conv3x3_s2rows_supported", &conv3x3_s2rows_supported);
  m.def("conv3x3_s2rows128_supported", &conv3x3_s2rows128_supported);
  m.def("conv3x3_s2rows128", [](uintptr_t x, uintptr_t wf, uintptr_t bias, uintptr_t y, int B, bool relu,
                                float out_inv_scale, uintptr_t stream) {
    conv3x3_s2rows128(P<void>(x), P<void>(wf), P<float>(bias), P<void>(y), B, relu, out_inv_scale, S(stream));
  }, py::arg("x"), py::arg("wf"), py::arg("bias"), py::arg("y"), py::arg("B"), py::arg("relu"),
        py::arg("out_inv_scale"), py::arg("stream"));
  m.def("conv3x3_s2rows", [](uintptr_t x, uintptr_t wf, uintptr_t bias, uintptr_t wdf, uintptr_t bd, uintptr_t y,
                             uintptr_t yd, uintptr_t zero, int B, bool relu, uintptr_t stream) {
    conv3x3_s2rows(P<void>(x), P<void>(wf), P<float>(bias), P<void>(wdf), P<float>(bd), P<void>(y), P<void>(yd),
                   P<void>(zero), B, relu, S(stream));
  }, py::arg("x"), py::arg("wf"), py::arg("bias"), py::arg("wdf"), py::arg("bd"), py::arg("y"), py::arg("yd"),
        py::arg("zero"), py::arg("B"), py::arg("relu"), py::arg("stream"));
  m.def("conv_small_supported", &conv_small_supported);
  m.def("conv_small_pick_mf", &conv_small_pick_mf);
  m.def("conv_small_set_mf", &conv_small_set_mf);
  m.def("conv_small", [](uintptr_t x, uintptr_t wf, uintptr_t bias, uintptr_t res, uintptr_t y, int B, int H, int W,
                         int CI, int CO, int stride, bool relu, int mf, uintptr_t stream, uintptr_t wdf, uintptr_t bd,
                         uintptr_t yd) {
    conv_small(P<void>(x), P<void>(wf), P<float>(bias), P<void>(res), P<void>(y), B, H, W, CI, CO, stride, relu, mf,
               S(stream), P<void>(wdf), P<float>(bd), P<void>(yd));
  }, py::arg("x"), py::arg("wf"), py::arg("bias"), py::arg("res"), py::arg("y"), py::arg("B"), py::arg("H"),
        py::arg("W"), py::arg("CI"), py::arg("CO"), py::arg("stride"), py::arg("relu"), py::arg("mf"),
        py::arg("stream"), py::arg("wdf") = 0, py::arg("bd") = 0, py::arg("yd") = 0);
  m.def("conv3x3_rows28_supported", &conv3x3_rows28_supported);
  m.def("conv3x3_rows28", [](uintptr_t x, uintptr_t wf, uintptr_t bias, uintptr_t res, uintptr_t y, int B, bool relu,
                             uintptr_t stream) {
    conv3x3_rows28(P<void>(x), P<void>(wf), P<float>(bias), P<void>(res), P<void>(y), B, relu, S(stream));
  }, py::arg("x"), py::arg("wf"), py::arg("bias"), py::arg("res"), py::arg("y"), py::arg("B"), py::arg("relu"),
        py::arg("stream"));
  m.def("stem_conv_pool_u8", [](uintptr_t x, uintptr_t w, uintptr_t bias, uintptr_t y, int B, int S_, int strip,
                                uintptr_t stream, uintptr_t w_dense) {
    stem_conv_pool_u8(P<uint8_t>(x), P<void>(w), P<float>(bias), P<void>(y), B, S_, strip, S(stream),
                      P<void>(w_dense));
  }, py::arg("x"), py::arg("w"), py::arg("bias"), py::arg("y"), py::arg("B"), py::arg("S"), py::arg("strip"),
        py::arg("stream"), py::arg("w_dense") = 0);
  m.def("stem_dense_k_index", &stem_dense_k_index);
  m.def("stem_conv_pool_set_dbg", &stem_conv_pool_set_dbg);
  m.def("stem_conv_pool_set_stamps", [](uintptr_t p) { stem_conv_pool_set_stamps((void*)p); });
  m.def("kernel_stagger", &kernel_stagger);
  m.def("kernel_stagger_set", &kernel_stagger_set);
  m.def("kernel_stagger_for_lanes", &kernel_stagger_for_lanes);
  m.def("stem_conv_pool", [](uintptr_t x, uintptr_t w, uintptr_t bias, uintptr_t y, int B, int S_, int Wq,
                             int strip, uintptr_t stream) {
    stem_conv_pool(P<void>(x), P<void>(w), P<float>(bias), P<void>(y), B, S_, Wq, strip, S(stream));
  });
  m.def("mfma_fp8_probe", [](uintptr_t a, uintptr_t b, uintptr_t d, uintptr_t stream) {
    mfma_fp8_probe(P<void>(a), P<void>(b), P<float>(d), S(stream));
  });
  m.def("head_ws_bytes", &head_ws_bytes);
  m.def("head_pooled_splits", &head_pooled_splits);
  m.def("conv1x1_plan", [](bool in8, bool out8, int rb, int nw, bool res, int s, int wv, bool ch) {
    const C1Plan p = conv1x1_plan(in8, out8, rb, nw, res, s, wv, ch);
    py::dict d;
    d["s"] = p.s;
    d["dt"] = p.dt;
    d["rt"] = p.rt;
    d["st"] = p.st;
    d["st2"] = p.st2;
    d["pre"] = p.pre;
    d["n1"] = p.n1;
    d["n1_first"] = p.n1_first;
    d["pro_wait"] = p.pro_wait;
    d["pro_wait_ch"] = p.pro_wait_ch;
    d["res_wait"] = p.res_wait;
    return d;
  });
  m.def("head_pooled", [](uintptr_t pooled, uintptr_t w, uintptr_t bias, int B, int C, int N, int ldw, int Npad,
                          uintptr_t logits, uintptr_t idx, uintptr_t prob, uintptr_t ws, size_t ws_bytes, int num_cus,
                          uintptr_t stream, int ns, int ko) {
    head_pooled(P<void>(pooled), P<void>(w), P<float>(bias), B, C, N, ldw, Npad, P<float>(logits), P<int32_t>(idx),
                P<float>(prob), P<void>(ws), ws_bytes, num_cus, S(stream), ns, ko);
  }, py::arg("pooled"), py::arg("w"), py::arg("bias"), py::arg("B"), py::arg("C"), py::arg("N"), py::arg("ldw"),
        py::arg("Npad"), py::arg("logits"), py::arg("idx"), py::arg("prob"), py::arg("ws"), py::arg("ws_bytes"),
        py::arg("num_cus"), py::arg("stream"), py::arg("ns") = 0, py::arg("ko") = 0);
  m.def("softmax_top1", [](uintptr_t logits, int B, int N, int ld, uintptr_t idx, uintptr_t prob,
                           uintptr_t stream) {
    softmax_top1(P<float>(logits), B, N, ld, P<int32_t>(idx), P<float>(prob), S(stream));
  });

  // ---------------------------------------------------------------- jpeg
  m.def("decode_jpeg", [](py::bytes data) {
    std::string s = data;
    Image img;
    {
      py::gil_scoped_release nogil;
      img = decode_jpeg((const uint8_t*)s.data(), s.size());
    }
    py::array_t<uint8_t> a({img.height, img.width, 3});
    std::copy(img.rgb.begin(), img.rgb.end(), a.mutable_data());
    return a;
  });

  // ---------------------------------------------------------------- .ot
  m.def("ot_load", [](const std::string& path) { return from_weight_map(ot_load(path)); });
  m.def("ot_save", [](const std::string& path, const py::dict& d) { ot_save(path, to_weight_map(d)); });
  // where a staged shard replica's images live (csrc/serve/shard.h)
  m.def("shard_slices", [](int64_t n, const std::vector<int>& devices) {
    py::list out;
    for (const auto& s : shard_slices(n, devices)) out.append(py::make_tuple(s.device, s.first, s.n));
    return out;
  });
  m.def("shard_placement", [](int64_t n, const std::vector<std::vector<int>>& parts) {
    py::list out;
    for (const auto& p : shard_placement(n, parts))
      out.append(py::make_tuple(p.copy, p.slice.device, p.slice.first, p.slice.n));
    return out;
  });

  // ---------------------------------------------------------------- engine
  // host-only packing audit: [(layer, kind, off, bytes)], arena bytes
  m.def("pack_audit", [](const std::string& arch, const py::dict& weights, const std::map<std::string, bool>& options,
                         int num_classes, int image_size) {
    size_t total = 0;
    const auto regs = Engine::pack_audit(arch, to_weight_map(weights), engine_options(options), &total,
                                         num_classes, image_size);
    py::list out;
    for (const auto& r : regs) out.append(py::make_tuple(r.layer, r.kind, r.off, r.bytes));
    return py::make_tuple(out, total);
  }, py::arg("arch"), py::arg("weights"), py::arg("options") = std::map<std::string, bool>{},
     py::arg("num_classes") = 1000, py::arg("image_size") = 224);
  py::class_<Engine>(m, "Engine")
      .def(py::init([](const std::string& arch, const py::dict& weights, int device, int num_classes,
                       int image_size, const std::map<std::string, bool>& options) {
             return new Engine(arch, to_weight_map(weights), device, num_classes, image_size, engine_options(options));
           }),
           py::arg("arch"), py::arg("weights"), py::arg("device") = 0, py::arg("num_classes") = 1000,
           py::arg("image_size") = 224, py::arg("options") = std::map<std::string, bool>{})
      .def_static(
          "from_ot",
          [](const std::string& arch, const std::string& path, int device, int num_classes, int image_size,
             const std::map<std::string, bool>& options) {
            return new Engine(arch, ot_load(path), device, num_classes, image_size, engine_options(options));
          },
          py::arg("arch"), py::arg("path"), py::arg("device") = 0, py::arg("num_classes") = 1000,
          py::arg("image_size") = 224, py::arg("options") = std::map<std::string, bool>{})
      .def("reserve", &Engine::reserve, py::call_guard<py::gil_scoped_release>())
      .def(
          "forward",
          [](Engine& e, uintptr_t images, int B, int Hin, int Win, uintptr_t idx, uintptr_t prob,
             uintptr_t logits, uintptr_t stream, bool use_graph) {
            e.forward(P<uint8_t>(images), B, Hin, Win, P<int32_t>(idx), P<float>(prob), P<float>(logits),
                      S(stream), use_graph);
          },
          py::arg("images"), py::arg("B"), py::arg("Hin"), py::arg("Win"), py::arg("idx"),
          py::arg("prob"), py::arg("logits"), py::arg("stream"), py::arg("use_graph") = true,
          py::call_guard<py::gil_scoped_release>())
      .def("profile",
           [](Engine& e, uintptr_t images, int B, int Hin, int Win, uintptr_t stream) {
             return e.profile(P<uint8_t>(images), B, Hin, Win, S(stream));
           })
      .def("activation_ptr", [](const Engine& e, int id) { return reinterpret_cast<uintptr_t>(e.activation(id)); })
      .def("activation_shape",
           [](const Engine& e, int id) {
             auto s = e.activation_shape(id);
             return py::make_tuple(s.H, s.W, s.C, s.f32);
           })
      .def("op_list",
           [](const Engine& e) {
             py::list l;
             for (const auto& op : e.ops()) l.append(py::make_tuple(op.name, op.in, op.out, op.res));
             return l;
           })
      .def_property_readonly("num_activations", &Engine::num_activations)
      .def_property_readonly("arch", &Engine::arch)
      .def_property_readonly("device", &Engine::device)
      .def_property_readonly("num_classes", &Engine::num_classes)
      .def_property_readonly("image_size", &Engine::image_size)
      .def_property_readonly("max_batch", &Engine::max_batch)
      .def_property_readonly("weight_bytes", &Engine::weight_bytes)
      .def_property_readonly("activation_bytes", &Engine::activation_bytes)
      .def_property_readonly("gflop_per_image", &Engine::gflop_per_image);

  // ---------------------------------------------------------------- data parallel
  bind_dp(m);
}
