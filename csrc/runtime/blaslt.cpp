#include "blaslt.h"

#include <hipblaslt/hipblaslt.h>

#include <algorithm>
#include <stdexcept>
#include <string>
#include <vector>

#include "../kernels/kernels.h"

namespace dmlc {

namespace {
void ck(hipblasStatus_t st, const char* what) {
  if (st != HIPBLAS_STATUS_SUCCESS) throw std::runtime_error(std::string("hipBLASLt ") + what + " failed: " + std::to_string((int)st));
}
constexpr size_t kWorkspace = (size_t)32 << 20;
}  // namespace

struct BlasLt::Plan {
  hipblasLtMatmulDesc_t op = nullptr;
  hipblasLtMatrixLayout_t a = nullptr, b = nullptr, d = nullptr;
  hipblasLtMatmulAlgo_t algo{};
  ~Plan() {
    if (a) hipblasLtMatrixLayoutDestroy(a);
    if (b) hipblasLtMatrixLayoutDestroy(b);
    if (d) hipblasLtMatrixLayoutDestroy(d);
    if (op) hipblasLtMatmulDescDestroy(op);
  }
};

BlasLt::BlasLt(int device) : device_(device) {
  DMLC_HIP_CHECK(hipSetDevice(device_));
  hipblasLtHandle_t h;
  ck(hipblasLtCreate(&h), "create");
  handle_ = h;
  ws_bytes_ = kWorkspace;
  DMLC_HIP_CHECK(hipMalloc(&ws_, ws_bytes_));
}

BlasLt::~BlasLt() {
  (void)hipSetDevice(device_);
  plans_.clear();
  if (ws_) (void)hipFree(ws_);
  if (handle_) hipblasLtDestroy((hipblasLtHandle_t)handle_);
}

bool BlasLt::ready(int M, int N, int K, int ldx, int ldw, int ldy, bool y_f32, bool relu) const {
  return plans_.count(Key{M, N, K, ldx, ldw, ldy, y_f32, relu}) > 0;
}

bool BlasLt::prepare(int M, int N, int K, int ldx, int ldw, int ldy, bool y_f32, bool relu, const void* x,
                     const void* w, const float* bias, void* y, hipStream_t s) {
  const Key key{M, N, K, ldx, ldw, ldy, y_f32, relu};
  if (plans_.count(key)) return true;
  DMLC_HIP_CHECK(hipSetDevice(device_));
  auto p = std::make_shared<Plan>();
  ck(hipblasLtMatmulDescCreate(&p->op, HIPBLAS_COMPUTE_32F, HIP_R_32F), "desc");
  const hipblasOperation_t tA = HIPBLAS_OP_T, tB = HIPBLAS_OP_N;
  ck(hipblasLtMatmulDescSetAttribute(p->op, HIPBLASLT_MATMUL_DESC_TRANSA, &tA, sizeof(tA)), "transA");
  ck(hipblasLtMatmulDescSetAttribute(p->op, HIPBLASLT_MATMUL_DESC_TRANSB, &tB, sizeof(tB)), "transB");
  const hipblasLtEpilogue_t epi = relu ? HIPBLASLT_EPILOGUE_RELU_BIAS : HIPBLASLT_EPILOGUE_BIAS;
  ck(hipblasLtMatmulDescSetAttribute(p->op, HIPBLASLT_MATMUL_DESC_EPILOGUE, &epi, sizeof(epi)), "epilogue");
  const hipDataType bt = HIP_R_32F;
  ck(hipblasLtMatmulDescSetAttribute(p->op, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bt, sizeof(bt)), "bias type");
  ck(hipblasLtMatmulDescSetAttribute(p->op, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &bias, sizeof(bias)), "bias");
  // A = W stored K x N (column-major, ld ldw), used transposed; B = X stored
  // K x M (ld ldx); D = Y stored N x M (ld ldy)
  ck(hipblasLtMatrixLayoutCreate(&p->a, HIP_R_16BF, K, N, ldw), "layout A");
  ck(hipblasLtMatrixLayoutCreate(&p->b, HIP_R_16BF, K, M, ldx), "layout B");
  ck(hipblasLtMatrixLayoutCreate(&p->d, y_f32 ? HIP_R_32F : HIP_R_16BF, N, M, ldy), "layout D");
  hipblasLtMatmulPreference_t pref;
  ck(hipblasLtMatmulPreferenceCreate(&pref), "pref");
  const uint64_t wsb = ws_bytes_;
  ck(hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wsb, sizeof(wsb)), "pref ws");
  std::vector<hipblasLtMatmulHeuristicResult_t> res(8);
  int got = 0;
  const hipblasStatus_t hs = hipblasLtMatmulAlgoGetHeuristic((hipblasLtHandle_t)handle_, p->op, p->a, p->b, p->d,
                                                             p->d, pref, (int)res.size(), res.data(), &got);
  hipblasLtMatmulPreferenceDestroy(pref);
  if (hs != HIPBLAS_STATUS_SUCCESS || got <= 0) return false;
  // time the candidates on the real operands (the bias epilogue included)
  const float alpha = 1.f, beta = 0.f;
  hipEvent_t e0, e1;
  DMLC_HIP_CHECK(hipEventCreate(&e0));
  DMLC_HIP_CHECK(hipEventCreate(&e1));
  float best = 1e30f;
  int besti = -1;
  for (int i = 0; i < got; ++i) {
    if (res[i].state != HIPBLAS_STATUS_SUCCESS || res[i].workspaceSize > ws_bytes_) continue;
    bool ok = true;
    for (int r = 0; r < 2 && ok; ++r)  // warm
      ok = hipblasLtMatmul((hipblasLtHandle_t)handle_, p->op, &alpha, w, p->a, x, p->b, &beta, y, p->d, y, p->d,
                           &res[i].algo, ws_, ws_bytes_, s) == HIPBLAS_STATUS_SUCCESS;
    if (!ok) continue;
    DMLC_HIP_CHECK(hipEventRecord(e0, s));
    constexpr int kReps = 5;
    for (int r = 0; r < kReps; ++r)
      (void)hipblasLtMatmul((hipblasLtHandle_t)handle_, p->op, &alpha, w, p->a, x, p->b, &beta, y, p->d, y, p->d,
                            &res[i].algo, ws_, ws_bytes_, s);
    DMLC_HIP_CHECK(hipEventRecord(e1, s));
    DMLC_HIP_CHECK(hipEventSynchronize(e1));
    float ms = 0.f;
    DMLC_HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
    if (ms < best) best = ms, besti = i;
  }
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  if (besti < 0) return false;
  p->algo = res[besti].algo;
  plans_[key] = p;
  return true;
}

void BlasLt::fc(const void* x, int ldx, const void* w, int ldw, const float* bias, void* y, int ldy, bool y_f32,
                int M, int N, int K, bool relu, hipStream_t s) {
  auto it = plans_.find(Key{M, N, K, ldx, ldw, ldy, y_f32, relu});
  if (it == plans_.end()) throw std::logic_error("BlasLt::fc: shape not prepared");
  Plan& p = *it->second;
  // the bias pointer may differ per call (weight arena of another instance)
  ck(hipblasLtMatmulDescSetAttribute(p.op, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &bias, sizeof(bias)), "bias");
  const float alpha = 1.f, beta = 0.f;
  ck(hipblasLtMatmul((hipblasLtHandle_t)handle_, p.op, &alpha, w, p.a, x, p.b, &beta, y, p.d, y, p.d, &p.algo, ws_,
                     ws_bytes_, s),
     "matmul");
}

}  // namespace dmlc
