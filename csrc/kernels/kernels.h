// Host-side launch API of the gfx950 kernel library (all launches are
// asynchronous on the given stream; pointers are device pointers).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace ffk {

// ---- layernorm.hip
void layernorm_fwd(int dtype, const void* x, const void* res, void* sum_out, const void* gamma, const void* beta,
                   void* y, float* mean, float* rstd, int M, int N, float eps, hipStream_t st);
// ws: 2 * layernorm_bwd_grid(M, N) * N floats (block partials of dgamma/dbeta)
int layernorm_bwd_grid(int M, int N);
void layernorm_bwd(int dtype, const void* dy, const void* s, const float* mean, const float* rstd,
                   const void* gamma, void* dx, float* dgamma, float* dbeta, float* ws, int M, int N,
                   hipStream_t st);

// ---- elementwise.hip  (op: 0 identity, 1 relu, 2 sigmoid, 3 tanh, 4 gelu, 5 elu, 6 exp)
void bias_act_fwd(int dtype, const void* x, const void* bias, void* pre, void* y, int64_t M, int64_t N, int op,
                  float alpha, hipStream_t st);
void act_bwd(int dtype, const void* dy, const void* pre, void* dx, int64_t n, int op, float alpha, hipStream_t st);
void colsum_act(int dtype, const void* dy, const void* pre, void* dx, float* dbias, int64_t M, int64_t N, int op,
                float alpha, hipStream_t st);
void dropout_fwd(int dtype, const void* x, void* y, int64_t n, float p, uint64_t seed, hipStream_t st);
void cast(int dtype_in, int dtype_out, const void* x, void* y, int64_t n, hipStream_t st);
void axpby(int dtype, const void* x, void* y, int64_t n, float a, float b, hipStream_t st);

// ---- softmax.hip
void softmax_ce(int dtype, int label_bits, void* logits, const void* labels, float* row_loss, float* metrics, int M,
                int V, int V_valid, float grad_scale, int ignore_index, int write_grad, hipStream_t st);
void softmax_fwd(int dtype, const void* x, void* y, int M, int N, hipStream_t st);
void softmax_bwd(int dtype, const void* dy, const void* y, void* dx, int M, int N, hipStream_t st);

// ---- optimizer.hip
void adam_step(float* w, const void* g, int grad_dtype, float* m, float* v, void* w_bf16, int64_t n, float lr,
               float beta1, float beta2, float eps, float weight_decay, int step, float grad_scale, int decoupled,
               const float* hp, hipStream_t st);  // hp: optional device {lr, step} (graph replay)
void sgd_step(float* w, const void* g, int grad_dtype, float* mom, void* w_bf16, int64_t n, float lr,
              float momentum, float weight_decay, int nesterov, float grad_scale, hipStream_t st);
void sum_squares(const float* x, int64_t n, float* out, hipStream_t st);

// ---- embedding.hip  (mode: 0 none, 1 sum, 2 avg)
void embedding_fwd(int dtype, int index_bits, const void* idx, const void* W, void* out, int64_t B, int L, int D,
                   int mode, int64_t num_entries, hipStream_t st);
void embedding_bwd(int dtype, int index_bits, const void* idx, const void* dout, float* dW, int64_t B, int L, int D,
                   int mode, int64_t num_entries, float* workspace, int copies, hipStream_t st);

// ---- attention.hip
struct AttnTensors {
  struct T {
    const void* p = nullptr;
    int64_t sb = 0, ss = 0, sh = 0;
  };
  T q, k, v, o, dout, dq, dk, dv;
  float* lse = nullptr;
  float* delta = nullptr;
};
void attention_fwd(const AttnTensors& t, int B, int H, int Sq, int Sk, int D, float scale, bool causal,
                   hipStream_t st);
void attention_bwd(const AttnTensors& t, int B, int H, int Sq, int Sk, int D, float scale, bool causal,
                   hipStream_t st);

// ---- gemm.hip (bf16 MFMA GEMM with fused epilogues)
// C[M,N] = act(alpha * op(A)[M,K] @ op(B)[K,N] + bias[N]) (+ beta*C)
void gemm_bf16(const void* A, const void* B, void* C, const void* bias, int M, int N, int K, int lda, int ldb,
               int ldc, bool trans_a, bool trans_b, int act, float alpha, float beta, int out_f32,
               hipStream_t st);
// Same, additionally storing the pre-activation (bf16, ldc) when `pre` != null.
void gemm_bf16_ex(const void* A, const void* B, void* C, const void* bias, void* pre, int M, int N, int K, int lda,
                  int ldb, int ldc, bool trans_a, bool trans_b, int act, float alpha, float beta, int out_f32,
                  hipStream_t st);

// ---- gemm256.hip: 256x256 tiles, LDS-DMA staging, split-K (fp32 partials
// in `workspace` [splits][M][N] + reduce pass); needs K % 64 == 0.
bool gemm256_supported(int M, int N, int K, int lda, int ldb, bool trans_a, bool trans_b);
void gemm256_bf16(const void* A, const void* B, void* C, const void* bias, void* pre, int M, int N, int K, int lda,
                  int ldb, int ldc, bool trans_a, bool trans_b, int act, float alpha, float beta, int out_f32,
                  int splits, float* workspace, hipStream_t st);

}  // namespace ffk
