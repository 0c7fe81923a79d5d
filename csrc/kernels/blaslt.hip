// hipBLASLt GEMMs with fused epilogues (host code; the library kernels are
// AMD's tuned MFMA assembly).  Used where a plain library GEMM is the best
// GEMM on gfx950 ("hipBLASLt/rocBLAS only for plain library
// GEMMs") — and the epilogue removes a separate memory-bound pass:
//
//   EPI_BIAS           C = A B + bias
//   EPI_GELU_BIAS      C = gelu(A B + bias)                         (inference: no aux)
//   EPI_BGRADB         C = A^T B, dbias = colsum(A)                 (dW^T = dY^T X with db)
//
// The training epilogues for GELU (GELU_AUX_BIAS, DGELU_BGRAD) and BGRADA
// have NO algorithm in the hipBLASLt build PyTorch-ROCm ships for gfx950
// (tools/blaslt_probe.py), and RELU_AUX_BIAS's aux did not match the
// pre-activation in our checks: BERT/GPT keep the custom GELU + bias-grad
// kernels (elementwise.hip colsum_act).
//
// Parity: lib/kernels/src/cuda/ops/linear_kernels.cu (cublasGemmEx :131/:231/
// :303, bias GEMM :152 and :280, activation :173, activation grad in place) —
// here one library call per product with the bias / activation / bias-grad
// folded into its epilogue.
//
// Row-major C[M,N] = op(A)[M,K] op(B)[K,N] is issued as the column-major
// product C^T = op(B)^T op(A)^T, so "bias over output columns" is the
// library's per-row bias and a colsum over our rows is its BGRADA.
// Descriptors, layouts and the heuristic's algorithm are cached per shape;
// launches are asynchronous and capturable (no allocation: the caller passes
// the workspace).
#include <hipblaslt/hipblaslt.h>
#include <hipblaslt/hipblaslt-ext.hpp>

#include <map>
#include <mutex>
#include <tuple>

#include "kernels.h"

namespace ffk {

namespace {

#define FFK_BLT(x)                                                                                   \
  do {                                                                                               \
    hipblasStatus_t s_ = (x);                                                                        \
    if (s_ != HIPBLAS_STATUS_SUCCESS)                                                                \
      throw std::runtime_error(std::string("hipBLASLt: ") + #x + " failed with status " +         \
                               std::to_string(static_cast<int>(s_)));                                \
  } while (0)

constexpr int kMaxAlgos = 16;

struct Plan {
  hipblasLtMatmulDesc_t desc = nullptr;
  hipblasLtMatrixLayout_t a = nullptr, b = nullptr, c = nullptr;
  // the heuristic's top candidates: index 0 is the library's pick, the
  // GEMM autotuner (ops/gemm.py) times the others per shape
  hipblasLtMatmulAlgo_t algo[kMaxAlgos]{};
  size_t ws_needed[kMaxAlgos]{};
  int n_algos = 0;
  // library solutions addressed by their solution index (beyond the
  // heuristic's top 16: an offline sweep over every solution that supports
  // the problem, tools/blaslt_sweep.py), resolved + checked once per plan
  std::map<int, std::pair<hipblasLtMatmulAlgo_t, size_t>> by_index;
};

using Key = std::tuple<int, int, int, int, int, int, bool, bool, int, int, bool, int>;

hipblasLtHandle_t handle() {
  static hipblasLtHandle_t h = [] {
    hipblasLtHandle_t x;
    FFK_BLT(hipblasLtCreate(&x));
    return x;
  }();
  return h;
}

std::mutex mu;
std::map<Key, Plan>& plans() {
  static std::map<Key, Plan> p;
  return p;
}

hipblasLtEpilogue_t epi_of(int e) {
  switch (e) {
    case EPI_BIAS: return HIPBLASLT_EPILOGUE_BIAS;
    case EPI_GELU_BIAS: return HIPBLASLT_EPILOGUE_GELU_BIAS;
    case EPI_BGRADB: return HIPBLASLT_EPILOGUE_BGRADB;
    default: return HIPBLASLT_EPILOGUE_DEFAULT;
  }
}

Plan& get_plan(int M, int N, int K, int lda, int ldb, int ldc, bool ta, bool tb, int epi, int out_f32, bool has_beta,
               int aux_ld, size_t ws_bytes) {
  Key key{M, N, K, lda, ldb, ldc, ta, tb, epi, out_f32, has_beta, aux_ld};
  auto it = plans().find(key);
  if (it != plans().end()) return it->second;
  Plan p;
  // column-major view: D'[N x M] = op(B)'[N x K] * op(A)'[K x M]
  const hipblasOperation_t opa = tb ? HIPBLAS_OP_T : HIPBLAS_OP_N;  // library A = our B
  const hipblasOperation_t opb = ta ? HIPBLAS_OP_T : HIPBLAS_OP_N;  // library B = our A
  FFK_BLT(hipblasLtMatmulDescCreate(&p.desc, HIPBLAS_COMPUTE_32F, HIP_R_32F));
  FFK_BLT(hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSA, &opa, sizeof(opa)));
  FFK_BLT(hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSB, &opb, sizeof(opb)));
  const hipblasLtEpilogue_t e = epi_of(epi);
  FFK_BLT(hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_EPILOGUE, &e, sizeof(e)));
  if (epi != EPI_NONE) {
    // bias input is bf16; bias-gradient outputs are fp32 (the flat gradient buffer)
    const hipDataType bt = epi == EPI_BGRADB ? HIP_R_32F : HIP_R_16BF;
    FFK_BLT(hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bt, sizeof(bt)));
  }
  if (!tb) FFK_BLT(hipblasLtMatrixLayoutCreate(&p.a, HIP_R_16BF, N, K, ldb));
  else FFK_BLT(hipblasLtMatrixLayoutCreate(&p.a, HIP_R_16BF, K, N, ldb));
  if (!ta) FFK_BLT(hipblasLtMatrixLayoutCreate(&p.b, HIP_R_16BF, K, M, lda));
  else FFK_BLT(hipblasLtMatrixLayoutCreate(&p.b, HIP_R_16BF, M, K, lda));
  FFK_BLT(hipblasLtMatrixLayoutCreate(&p.c, out_f32 ? HIP_R_32F : HIP_R_16BF, N, M, ldc));
  hipblasLtMatmulPreference_t pref;
  FFK_BLT(hipblasLtMatmulPreferenceCreate(&pref));
  uint64_t wsb = ws_bytes;
  FFK_BLT(hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wsb, sizeof(wsb)));
  hipblasLtMatmulHeuristicResult_t res[kMaxAlgos];
  int n = 0;
  FFK_BLT(hipblasLtMatmulAlgoGetHeuristic(handle(), p.desc, p.a, p.b, p.c, p.c, pref, kMaxAlgos, res, &n));
  hipblasLtMatmulPreferenceDestroy(pref);
  if (n <= 0)
    throw std::runtime_error("hipBLASLt: no algorithm for this GEMM / epilogue (M=" + std::to_string(M) +
                             " N=" + std::to_string(N) + " K=" + std::to_string(K) + " epi=" + std::to_string(epi) +
                             ")");
  for (int i = 0; i < n && i < kMaxAlgos; ++i) {
    p.algo[p.n_algos] = res[i].algo;
    p.ws_needed[p.n_algos] = res[i].workspaceSize;
    ++p.n_algos;
  }
  return plans().emplace(key, p).first->second;
}

}  // namespace

// Diagnostic: number of heuristic algorithms for a raw epilogue / type combination
// (-1 = attribute rejected).  bias_t / aux_t: -1 leave unset, else hipDataType.
int blaslt_probe(int M, int N, int K, bool ta, bool tb, int raw_epi, int bias_t, int aux_t, int out_f32) {
  hipblasLtMatmulDesc_t desc;
  FFK_BLT(hipblasLtMatmulDescCreate(&desc, HIPBLAS_COMPUTE_32F, HIP_R_32F));
  const hipblasOperation_t opa = tb ? HIPBLAS_OP_T : HIPBLAS_OP_N, opb = ta ? HIPBLAS_OP_T : HIPBLAS_OP_N;
  hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_TRANSA, &opa, sizeof(opa));
  hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_TRANSB, &opb, sizeof(opb));
  const hipblasLtEpilogue_t e = static_cast<hipblasLtEpilogue_t>(raw_epi);
  if (hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_EPILOGUE, &e, sizeof(e)) != HIPBLAS_STATUS_SUCCESS)
    return -1;
  if (bias_t >= 0) {
    const hipDataType bt = static_cast<hipDataType>(bias_t);
    if (hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bt, sizeof(bt)) !=
        HIPBLAS_STATUS_SUCCESS)
      return -1;
  }
  if (aux_t >= 0) {
    const int64_t ld = N;
    hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_LD, &ld, sizeof(ld));
    const hipDataType at = static_cast<hipDataType>(aux_t);
    if (hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_DATA_TYPE, &at, sizeof(at)) !=
        HIPBLAS_STATUS_SUCCESS)
      return -1;
  }
  hipblasLtMatrixLayout_t a, b, c;
  hipblasLtMatrixLayoutCreate(&a, HIP_R_16BF, tb ? K : N, tb ? N : K, tb ? K : N);
  hipblasLtMatrixLayoutCreate(&b, HIP_R_16BF, ta ? M : K, ta ? K : M, ta ? M : K);
  hipblasLtMatrixLayoutCreate(&c, out_f32 ? HIP_R_32F : HIP_R_16BF, N, M, N);
  hipblasLtMatmulPreference_t pref;
  hipblasLtMatmulPreferenceCreate(&pref);
  uint64_t wsb = 64 << 20;
  hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wsb, sizeof(wsb));
  hipblasLtMatmulHeuristicResult_t res[8];
  int n = 0;
  if (hipblasLtMatmulAlgoGetHeuristic(handle(), desc, a, b, c, c, pref, 8, res, &n) != HIPBLAS_STATUS_SUCCESS) n = 0;
  hipblasLtMatmulPreferenceDestroy(pref);
  hipblasLtMatrixLayoutDestroy(a);
  hipblasLtMatrixLayoutDestroy(b);
  hipblasLtMatrixLayoutDestroy(c);
  hipblasLtMatmulDescDestroy(desc);
  return n;
}

int blaslt_num_algos(int M, int N, int K, int lda, int ldb, int ldc, bool ta, bool tb, int epi, int out_f32,
                     bool has_beta, int aux_ld, size_t ws_bytes) {
  std::lock_guard<std::mutex> g(mu);
  try {
    return get_plan(M, N, K, lda, ldb, ldc, ta, tb, epi, out_f32, has_beta, aux_ld, ws_bytes).n_algos;
  } catch (const std::runtime_error&) {
    return 0;
  }
}

bool blaslt_supported(int M, int N, int K, int lda, int ldb, int ldc, bool ta, bool tb, int epi, int out_f32,
                      bool has_beta, int aux_ld, size_t ws_bytes) {
  return blaslt_num_algos(M, N, K, lda, ldb, ldc, ta, tb, epi, out_f32, has_beta, aux_ld, ws_bytes) > 0;
}

void blaslt_gemm(const void* A, const void* B, void* C, int M, int N, int K, int lda, int ldb, int ldc, bool ta,
                 bool tb, int epi, const void* bias, void* aux, int aux_ld, float alpha, float beta, int out_f32,
                 void* ws, size_t ws_bytes, hipStream_t st, int algo) {
  if (M <= 0 || N <= 0 || K <= 0) return;
  if ((epi == EPI_BIAS || epi == EPI_GELU_BIAS) && !bias)
    throw std::invalid_argument("blaslt: epilogue needs a bias");
  if (epi == EPI_BGRADB && !bias) throw std::invalid_argument("blaslt: BGRADB needs its fp32 output vector");
  std::lock_guard<std::mutex> g(mu);
  Plan& p = get_plan(M, N, K, lda, ldb, ldc, ta, tb, epi, out_f32, beta != 0.f, aux_ld, ws_bytes);
  if (algo < 0 || algo >= p.n_algos) throw std::invalid_argument("blaslt: algorithm index out of range");
  if (p.ws_needed[algo] > ws_bytes) throw std::invalid_argument("blaslt: workspace too small");
  if (epi != EPI_NONE)
    FFK_BLT(hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &bias, sizeof(bias)));
  (void)aux;
  (void)aux_ld;
  FFK_BLT(hipblasLtMatmul(handle(), p.desc, &alpha, B, p.a, A, p.b, &beta, C, p.c, C, p.c, &p.algo[algo], ws, ws_bytes, st));
}

// Every library solution (index) that supports this problem, in the library's
// order; plain GEMMs only (no epilogue).
std::vector<int> blaslt_solutions(int M, int N, int K, int lda, int ldb, int ldc, bool ta, bool tb, int out_f32,
                                  bool has_beta, size_t ws_bytes) {
  std::lock_guard<std::mutex> g(mu);
  Plan& p = get_plan(M, N, K, lda, ldb, ldc, ta, tb, EPI_NONE, out_f32, has_beta, 0, ws_bytes);
  const hipblasOperation_t opa = tb ? HIPBLAS_OP_T : HIPBLAS_OP_N, opb = ta ? HIPBLAS_OP_T : HIPBLAS_OP_N;
  std::vector<hipblasLtMatmulHeuristicResult_t> all;
  const hipDataType ct = out_f32 ? HIP_R_32F : HIP_R_16BF;
  FFK_BLT(hipblaslt_ext::getAllAlgos(handle(), hipblaslt_ext::GemmType::HIPBLASLT_GEMM, opa, opb, HIP_R_16BF,
                                     HIP_R_16BF, ct, ct, HIPBLAS_COMPUTE_32F, all));
  const float alpha = 1.f, beta = has_beta ? 1.f : 0.f;
  std::vector<int> out;
  for (auto& r : all) {
    size_t ws = 0;
    hipblasLtMatmulAlgo_t a = r.algo;
    if (hipblaslt_ext::matmulIsAlgoSupported(handle(), p.desc, &alpha, p.a, p.b, &beta, p.c, p.c, a, ws) !=
        HIPBLAS_STATUS_SUCCESS || ws > ws_bytes)
      continue;
    const int idx = hipblaslt_ext::getIndexFromAlgo(a);
    p.by_index[idx] = {a, ws};
    out.push_back(idx);
  }
  return out;
}

std::string blaslt_solution_name(int index) {
  std::vector<int> ids{index};
  std::vector<hipblasLtMatmulHeuristicResult_t> r;
  if (hipblaslt_ext::getAlgosFromIndex(handle(), ids, r) != HIPBLAS_STATUS_SUCCESS || r.empty()) return "";
  return hipblaslt_ext::getKernelNameFromAlgo(handle(), r[0].algo);
}

// Plain GEMM with the library solution `index` (from blaslt_solutions or a
// tuned table); throws if that solution does not support the problem.
void blaslt_gemm_solution(const void* A, const void* B, void* C, int M, int N, int K, int lda, int ldb, int ldc,
                          bool ta, bool tb, float alpha, float beta, int out_f32, void* ws, size_t ws_bytes,
                          hipStream_t st, int index) {
  if (M <= 0 || N <= 0 || K <= 0) return;
  std::lock_guard<std::mutex> g(mu);
  Plan& p = get_plan(M, N, K, lda, ldb, ldc, ta, tb, EPI_NONE, out_f32, beta != 0.f, 0, ws_bytes);
  auto it = p.by_index.find(index);
  if (it == p.by_index.end()) {
    std::vector<int> ids{index};
    std::vector<hipblasLtMatmulHeuristicResult_t> r;
    if (hipblaslt_ext::getAlgosFromIndex(handle(), ids, r) != HIPBLAS_STATUS_SUCCESS || r.empty())
      throw std::invalid_argument("blaslt: unknown solution index " + std::to_string(index));
    size_t need = 0;
    hipblasLtMatmulAlgo_t a = r[0].algo;
    const float al = 1.f, be = beta != 0.f ? 1.f : 0.f;
    if (hipblaslt_ext::matmulIsAlgoSupported(handle(), p.desc, &al, p.a, p.b, &be, p.c, p.c, a, need) !=
        HIPBLAS_STATUS_SUCCESS)
      throw std::invalid_argument("blaslt: solution " + std::to_string(index) + " does not support this GEMM");
    it = p.by_index.emplace(index, std::make_pair(a, need)).first;
  }
  if (it->second.second > ws_bytes) throw std::invalid_argument("blaslt: workspace too small");
  FFK_BLT(hipblasLtMatmul(handle(), p.desc, &alpha, B, p.a, A, p.b, &beta, C, p.c, C, p.c, &it->second.first, ws,
                          ws_bytes, st));
}

}  // namespace ffk
