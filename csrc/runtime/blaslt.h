// Plain fully connected layers on hipBLASLt at throughput batch sizes.
//
// The AlexNet classifier (classifier.1 9216 -> 4096, .4 4096 -> 4096, .6
// 4096 -> 1000; reference: tch::vision::alexnet's Linear layers run by
// `forward_t`, src/services.rs:493) is a plain GEMM with a bias (+ ReLU)
// epilogue: at query batches (B <= 16) it runs on the weight-streaming
// fc_small.hip kernel; above that on hipBLASLt, whose gfx950 MFMA GEMMs stream
// the 75 MB classifier.1 weights near HBM rate (the implicit-GEMM conv kernel
// with split-K took ~120 us for it at B = 256, profiles/r3_alexnet_b256_kernel_stats.txt).
//
// y[M][N] (row-major, ld ldy) = x[M][K] (row-major, ld ldx) * w[N][K]^T
// (row-major, ld ldw) + bias[N], optional ReLU; x, w bf16; y bf16 or fp32.
// In hipBLASLt's column-major terms: D (N x M) = W^T-op(K x N) * X (K x M).
// The algorithm per shape is picked once, outside any graph capture
// (prepare(): heuristic candidates timed on the device), and every call
// after that is capture-safe (no allocation, no synchronisation).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <map>
#include <memory>
#include <tuple>

namespace dmlc {

class BlasLt {
 public:
  explicit BlasLt(int device);
  ~BlasLt();
  BlasLt(const BlasLt&) = delete;
  BlasLt& operator=(const BlasLt&) = delete;

  // Pick (and time) the algorithm for this shape; call outside capture.
  // Returns false if hipBLASLt has no algorithm for it.
  bool prepare(int M, int N, int K, int ldx, int ldw, int ldy, bool y_f32, bool relu, const void* x, const void* w,
               const float* bias, void* y, hipStream_t s);
  bool ready(int M, int N, int K, int ldx, int ldw, int ldy, bool y_f32, bool relu) const;
  void fc(const void* x, int ldx, const void* w, int ldw, const float* bias, void* y, int ldy, bool y_f32, int M,
          int N, int K, bool relu, hipStream_t s);
  int plans() const { return (int)plans_.size(); }

 private:
  struct Plan;
  using Key = std::tuple<int, int, int, int, int, int, bool, bool>;
  int device_;
  void* handle_ = nullptr;
  void* ws_ = nullptr;
  size_t ws_bytes_ = 0;
  std::map<Key, std::shared_ptr<Plan>> plans_;
};

}  // namespace dmlc
