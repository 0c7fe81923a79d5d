// Host-side launch API of the gfx950 kernel library (all launches are
// asynchronous on the given stream; pointers are device pointers).
#pragma once
#include <hip/hip_runtime.h>
#include <string>
#include <vector>

#include <algorithm>
#include <cstdint>

namespace ffk {

// ---- layernorm.hip
void layernorm_fwd(int dtype, const void* x, const void* res, void* sum_out, const void* gamma, const void* beta,
                   void* y, float* mean, float* rstd, int M, int N, float eps, hipStream_t st);
// ws: 3 * layernorm_bwd_grid(M, N) * N floats (block partials of dgamma/dbeta/dsum).
// dx = LN'(dy) [+ dres]; dsum += colsum(dx) (the producer Linear's bias grad).
int layernorm_bwd_grid(int M, int N);
void layernorm_bwd(int dtype, const void* dy, const void* s, const float* mean, const float* rstd,
                   const void* gamma, void* dx, float* dgamma, float* dbeta, float* ws, int M, int N,
                   hipStream_t st, const void* dres = nullptr,
                   float* dsum = nullptr);

// ---- elementwise.hip  (op: 0 identity, 1 relu, 2 sigmoid, 3 tanh, 4 gelu, 5 elu, 6 exp)
void bias_act_fwd(int dtype, const void* x, const void* bias, void* pre, void* y, int64_t M, int64_t N, int op,
                  float alpha, hipStream_t st);
void act_bwd(int dtype, const void* dy, const void* pre, void* dx, int64_t n, int op, float alpha, hipStream_t st);
void colsum_act(int dtype, const void* dy, const void* pre, void* dx, float* dbias, int64_t M, int64_t N, int op,
                float alpha, hipStream_t st);
void dropout_fwd(int dtype, const void* x, void* y, int64_t n, float p, uint64_t seed, hipStream_t st);
void cast(int dtype_in, int dtype_out, const void* x, void* y, int64_t n, hipStream_t st);
void axpby(int dtype, const void* x, void* y, int64_t n, float a, float b, hipStream_t st);
void zero_fill(void* p, int64_t bytes, hipStream_t st);

// ---- softmax.hip
// row_stats: optional [M, 3] fp32 scratch; with metrics, per-row metric terms
// are written there and reduced by one block instead of per-row atomics
void softmax_ce(int dtype, int label_bits, void* logits, const void* labels, float* row_loss, float* metrics,
                float* row_stats, int M, int V, int V_valid, float grad_scale, int ignore_index, int write_grad,
                hipStream_t st);
void softmax_fwd(int dtype, const void* x, void* y, int M, int N, hipStream_t st);
void softmax_bwd(int dtype, const void* dy, const void* y, void* dx, int M, int N, hipStream_t st);

// ---- optimizer.hip
void adam_step(float* w, const void* g, int grad_dtype, float* m, float* v, void* w_bf16, int64_t n, float lr,
               float beta1, float beta2, float eps, float weight_decay, int step, float grad_scale, int decoupled,
               const float* hp, hipStream_t st);  // hp: optional device {lr, step} (graph replay)
void sgd_step(float* w, const void* g, int grad_dtype, float* mom, void* w_bf16, int64_t n, float lr,
              float momentum, float weight_decay, int nesterov, float grad_scale, hipStream_t st);
void sum_squares(const float* x, int64_t n, float* out, hipStream_t st);
// row-sparse SGD over up to kMaxSparseTables embedding tables (two launches)
constexpr int kMaxSparseTables = 16;
struct SparseSgdTable {
  float* master;       // [rows, dim] fp32
  void* grad;          // [rows, dim] fp32 or bf16 (grad_bf16)
  void* compute;       // optional [rows, dim] bf16 copy
  const void* idx;     // [n_idx] int32 or int64 (idx64)
  int64_t n_idx, rows, scratch_off;
  int dim, grad_bf16, idx64;
};
struct SparseSgdArgs {
  SparseSgdTable t[kMaxSparseTables];
  int nt;
};
void sparse_sgd_rows(const SparseSgdArgs& a, float* scratch, float step, hipStream_t st);


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
  // optional fp32 [H*D] bias gradients of the q / k / v projections: the
  // backward adds the column sums of dq / dk / dv (sum over batch and sequence)
  float* dbq = nullptr;
  float* dbk = nullptr;
  float* dbv = nullptr;
  // > 0: dbq / dbk / dbv point at per-32-row partial slabs (row stride db_ld
  // floats; dq rows b * ceil(Sq/32) + q/32, dk / dv rows b * ceil(Sk/32) +
  // k/32, columns h * D + d) written without atomics; the caller sums rows
  int64_t db_ld = 0;
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
// splits > 1: split-K over blockIdx.y into `ws` ([splits][M][N] fp32), then one
// pass applying the epilogue (small-M GEMMs that cannot fill 256 CUs).
void gemm_bf16_ex(const void* A, const void* B, void* C, const void* bias, void* pre, int M, int N, int K, int lda,
                  int ldb, int ldc, bool trans_a, bool trans_b, int act, float alpha, float beta, int out_f32,
                  hipStream_t st, int splits = 1, float* ws = nullptr);

// ---- gemm256.hip: 256x256 tiles, LDS-DMA staging, split-K (fp32 partials
// in `workspace` [splits][M][N] + reduce pass); needs K % 64 == 0.
bool gemm256_supported(int M, int N, int K, int lda, int ldb, bool trans_a, bool trans_b);
void gemm256_bf16(const void* A, const void* B, void* C, const void* bias, void* pre, int M, int N, int K, int lda,
                  int ldb, int ldc, bool trans_a, bool trans_b, int act, float alpha, float beta, int out_f32,
                  int splits, float* workspace, hipStream_t st);

// out[m][n] = sum_s ws[s][m][n] + beta * out[m][n] (split-K reduce; gemm256.hip)
void splitk_reduce(const float* ws, void* out, int M, int N, int ldc, int S, float beta, int out_f32,
                   hipStream_t st);

// ---- gemmp.hip: phase-pipelined 256x256 GEMM with fused training epilogues
struct GemmPParams {
  const void* A = nullptr;
  const void* B = nullptr;
  void* C = nullptr;
  const void* bias = nullptr;   // [N] bf16
  void* pre = nullptr;          // pre-activation out, bf16 (ldc)
  const void* aux = nullptr;    // pre-activation in for act_bwd, bf16 (ldc)
  float* dbias = nullptr;       // += column sums of the result (fp32 atomics)
  float* workspace = nullptr;   // split-K fp32 [splits][M][N]
  int M = 0, N = 0, K = 0, lda = 0, ldb = 0, ldc = 0;
  bool trans_a = false, trans_b = false;
  int act = 0;                  // activation code (elementwise.hip numbering 0-4)
  bool act_bwd = false;         // result = acc * act'(aux) instead of act(acc)
  float alpha = 1.f, beta = 0.f;
  int out_f32 = 0, splits = 1;
  int dbg = 0;                  // ablation bits for timing experiments (gemmp.hip)
  int variant = 0;              // 0: 32x32x16 MFMA (gemmp.hip), 1: 16x16x32 (gemmq.hip), 2: ping-pong (gemmr.hip), 5: persistent gemmt, 6: gemmt with both operands by LDS-DMA,
                                // 3 / 4: one wave per SIMD, 128x128 wave tile, B staged
                                // through registers / by LDS-DMA (gemmt.hip),
                                // 8: 64x64 tiles for MLP-sized products (gemms.hip),
                                // 9: eight-wave multistage NT kernel (gemmn.hip; other layouts -> gemmq),
                                // 11: eight-wave ping-pong A B^T kernel (gemmpp.hip; other layouts -> gemmq)
};
bool gemmp_supported(int M, int N, int K, int lda, int ldb, bool trans_a, bool trans_b);
void gemmp_bf16(const GemmPParams& p, hipStream_t st);
void gemmq_launch(const GemmPParams& p, int splits, int n_cu, hipStream_t st);
void gemmr_launch(const GemmPParams& p, int splits, int n_cu, hipStream_t st);
void gemmt_launch(const GemmPParams& p, int splits, int stage_mode, hipStream_t st);
bool gemmt_supported(const GemmPParams& p);
// eight-wave multistage NT GEMM, variant 9 (gemmn.hip)
bool gemmn_supported(const GemmPParams& p);
void gemmn_launch(const GemmPParams& p, hipStream_t st);
// eight-wave ping-pong A B^T GEMM, variant 11 (gemmpp.hip)
bool gemmpp_supported(const GemmPParams& p);
void gemmpp_launch(const GemmPParams& p, hipStream_t st);
// small-tile (64 x 64) MLP GEMM, variant 8 (gemms.hip)
bool gemms_supported(const GemmPParams& p);
void gemms_launch(const GemmPParams& p, int splits, hipStream_t st);
void gemms_launch_batched(const GemmPParams& p, int splits, int batch, int64_t sA, int64_t sB, int64_t sC,
                          hipStream_t st);
// batched C[z] = alpha op(A[z]) op(B[z]) + beta C[z] on the 64x64-tile kernel
// (the reference's batch_matmul_kernels.cu); K % 64 == 0, M / N % 8 == 0
void bmm_bf16(const void* A, const void* B, void* C, int batch, int M, int N, int K, int lda, int ldb, int ldc,
              int64_t sA, int64_t sB, int64_t sC, bool trans_a, bool trans_b, float alpha, float beta, int out_f32,
              hipStream_t st);

// ---- tensorops.hip: general tensor operators (N-d, <= 6 dims)
struct NdShape {
  int nd = 0;
  int64_t size[6] = {1, 1, 1, 1, 1, 1};
};
struct NdStrides {
  int64_t s[6] = {0, 0, 0, 0, 0, 0};
};
// op: 0 add 1 sub 2 mul 3 div 4 max 5 min 6 eq 7 gt 8 lt; strides 0 on broadcast dims
void binary_nd(int dtype, const void* a, const void* b, void* y, const NdShape& s, const NdStrides& sa,
               const NdStrides& sb, int op, hipStream_t st);
// fp32 full-shape gradient w.r.t. a (which = 0) or b (which = 1)
void binary_grad_nd(int dtype, const void* dy, const void* a, const void* b, float* g, const NdShape& s,
                    const NdStrides& sa, const NdStrides& sb, int op, int which, hipStream_t st);
// out (shape `target`, same rank as s, 1 on broadcast dims) = sum_broadcast(full) + beta*out
void sum_to(int dtype, const float* full, void* out, const NdShape& s, const NdShape& target, float beta,
            hipStream_t st);
void permute_nd(int dtype, const void* x, void* y, const NdShape& out_shape, const NdStrides& in_strides_permuted,
                hipStream_t st);
constexpr int kMaxSlicePieces = 16;
struct SlicePieces {
  void* ptr[kMaxSlicePieces];
  int64_t len[kMaxSlicePieces], off[kMaxSlicePieces];
  int n;
};
// all pieces of a concat (to_slice = 0) or split (1) along one axis in one launch
void slice_copy_multi(int dtype, void* big, const SlicePieces& p, int64_t outer, int64_t inner, int64_t total,
                      int to_slice, hipStream_t st);
void slice_copy(int dtype, const void* x, void* y, int64_t outer, int64_t len, int64_t inner, int64_t total,
                int64_t off, int to_slice, int accumulate, hipStream_t st);
void reverse_axis(int dtype, const void* x, void* y, int64_t outer, int64_t len, int64_t inner, hipStream_t st);
void gather_axis(int dtype, int index_bits, const void* x, const void* idx, void* y, int64_t outer, int64_t len_x,
                 int64_t len_i, int64_t inner, hipStream_t st);
void scatter_add_axis(int dtype, int index_bits, const void* dy, const void* idx, float* dx, int64_t outer,
                      int64_t len_x, int64_t len_i, int64_t inner, hipStream_t st);
// op: 0 sum 1 mean 2 max 3 min 4 prod over the middle dim of [outer, red, inner]
void reduce_axis(int dtype, const void* x, void* y, int64_t outer, int64_t red, int64_t inner, int op,
                 hipStream_t st);
void topk_rows(int dtype, const void* x, void* vals, int64_t* idx, int64_t rows, int n, int k, hipStream_t st);
// op: 0 +s 1 -s 2 *s 3 /s 4 pow 5 log 6 sqrt 7 rsqrt 8 sin 9 cos 10 leaky_relu 11 ceil 12 round 13 identity
void unary_op(int dtype, const void* x, const void* dy, void* y, int64_t n, int op, float scalar, int backward,
              hipStream_t st);
// narrow Linear (N <= 8 outputs): forward with bias + activation, input
// gradient and weight / bias gradient with the activation derivative fused
void narrow_linear_fwd(const void* x, const void* w, const float* bias, void* y, void* pre, int64_t M, int64_t K,
                       int64_t N, int act, hipStream_t st);
void narrow_linear_dgrad(const void* dy, const void* pre, const void* w, void* dx, int64_t M, int64_t K, int64_t N,
                         int act, float beta, hipStream_t st);
int narrow_wgrad_blocks(int64_t M);
void narrow_linear_wgrad(const void* x, const void* dy, const void* pre, float* part, int blocks, void* dw,
                         int dw_dtype, float beta, float* db, int64_t M, int64_t K, int64_t N, int act,
                         hipStream_t st);
void mse_loss(int dtype, const void* pred, const void* label, void* grad, float* metrics, int64_t n, float scale,
              hipStream_t st);
void mse_loss_full(int dtype, int label_dtype, const void* pred, const void* label, void* grad, float* metrics,
                   int64_t n, float scale, int full, int64_t cols, int64_t rows, hipStream_t st);
// kind: 0 uniform[a,b) 1 normal(a,b) 2 truncated normal(a,b) in [c,d] 3 constant a
void init_tensor(int dtype, void* out, const NdShape& piece, const NdShape& full, const NdStrides& box_lo, int kind,
                 uint64_t seed, float a, float b, float c, float d, hipStream_t st);

// ---- conv.hip: implicit-GEMM convolution, NHWC bf16 activations, weight
// physically [K][R][S][C]; C % 8 == 0 and K % 8 == 0.
struct ConvShape {
  int N = 0, H = 0, W = 0, C = 0, K = 0, R = 1, S = 1;
  int sh = 1, sw = 1, ph = 0, pw = 0, dh = 1, dw = 1;
};
// y = act(conv(x, w) + bias); stats (optional, [2][K] fp32, overwritten):
// per-channel sum / sum of squares of y for a following BatchNorm, reduced
// from per-tile partials in stats_ws (conv2d_stats_ws_floats(s) floats).
int conv2d_stats_ws_floats(const ConvShape& s);
void conv2d_fwd(const ConvShape& s, const void* x, const void* w, const void* bias, void* y, float* stats,
                float* stats_ws, int act, hipStream_t st);
// dx = conv_transpose(dy, w) + beta * dx
// BN backward sums fused into a dgrad (stride 1, beta 0): sums [2][C] = sum g,
// sum g * (x - mean) * rstd with g the ReLU-masked dx; ws holds
// conv2d_dgrad_bn_ws_floats floats
struct ConvBnBwd {
  const void* x;
  const float* mean;
  const float* rstd;
  const float* scale_shift;   // null: no ReLU mask
  float* sums;
  float* ws;
};
int conv2d_dgrad_bn_ws_floats(const ConvShape& s);
void conv2d_dgrad(const ConvShape& s, const void* dy, const void* w, void* dx, float beta, hipStream_t st,
                  const ConvBnBwd* bn_sums = nullptr);
// strided bf16 [N][C][H][W] -> NHWC [N][H][W][Cp], pad channels zero (conv.hip)
void pad_channels_nhwc(const void* x, void* y, int64_t N, int C, int H, int W, int64_t sn, int64_t sc, int64_t sh,
                       int64_t sw, int Cp, hipStream_t st);
// dw (fp32, [K][R][S][C]) += wgrad; split-K partial slabs in ws
// (conv2d_wgrad_ws_floats(s, splits) floats; splits <= 0: auto)
int64_t conv2d_wgrad_ws_floats(const ConvShape& s, int splits);
void conv2d_wgrad(const ConvShape& s, const void* x, const void* dy, float* dw, float* ws, int splits,
                  hipStream_t st);
// Grouped bf16 convolutions on the same MFMA kernels: super-groups of whole
// groups as block-diagonal dense convs (blockIdx.z), the weight expanded
// once per step (conv2d_grouped_expand: [K][R][S][C/groups] ->
// [K][R][S][Cs], conv2d_grouped_wexp_elems elements); wgrad += into the
// compact fp32 [K][R][S][C/groups] (ws: conv2d_grouped_wgrad_ws_floats)
int64_t conv2d_grouped_wexp_elems(const ConvShape& s, int groups);
void conv2d_grouped_expand(const ConvShape& s, int groups, const void* w, void* wexp, hipStream_t st);
void conv2d_grouped_fwd(const ConvShape& s, int groups, const void* x, const void* wexp, const void* bias, void* y,
                        float* stats, float* stats_ws, int act, hipStream_t st);
void conv2d_grouped_dgrad(const ConvShape& s, int groups, const void* dy, const void* wexp, void* dx, float beta,
                          hipStream_t st);
int64_t conv2d_grouped_wgrad_ws_floats(const ConvShape& s, int groups);
void conv2d_grouped_wgrad(const ConvShape& s, int groups, const void* x, const void* dy, float* dw, float* ws,
                          hipStream_t st);

// ---- igemm32.hip: exact-fp32 MFMA (v_mfma_f32_32x32x2_f32) GEMM and
// convolutions; fp32 or bf16 inputs (in_f32), fp32 accumulation.
// GEMM: C = act(alpha op(A) op(B) + bias) [pre := pre-activation] (+ beta C),
// bias / pre / C in the output dtype (out_f32).
void gemm_f32(const void* A, const void* B, void* C, const void* bias, void* pre, int64_t M, int64_t N, int64_t K,
              int64_t lda, int64_t ldb, int64_t ldc, bool trans_a, bool trans_b, int act, float alpha, float beta,
              int in_f32, int out_f32, hipStream_t st, int batch = 1, int64_t sa = 0, int64_t sb = 0,
              int64_t sc = 0);
// Grouped NHWC convolutions (any groups dividing C and K; weight
// [K][R][S][C/groups]); outputs in the input dtype, dw fp32 (+=).
void conv32_fwd(const ConvShape& cs, int groups, const void* x, const void* w, const void* bias, void* y, int act,
                int in_f32, hipStream_t st);
void conv32_dgrad(const ConvShape& cs, int groups, const void* dy, const void* w, void* dx, float beta, int in_f32,
                  hipStream_t st);
void conv32_wgrad(const ConvShape& cs, int groups, const void* x, const void* dy, float* dw, int in_f32,
                  hipStream_t st);

// ---- bnpool.hip: BatchNorm (training) + pooling over NHWC bf16 [M][C]
// ws (optional, 32*C floats): 16 atomic buckets -> full-grid reduction (else the grid is capped);
// ws_clean bit 0: ws is zero on entry and is left zero (a persistent workspace: no memset per call);
// bit 1: write stats instead of adding to them
void bn_stats(const void* x, float* stats, int64_t M, int C, hipStream_t st, float* ws = nullptr, int ws_clean = 0);
void bn_finalize(const float* stats, const void* gamma, const void* beta, int param_dtype, float* running_mean,
                 float* running_var, float* scale, float* shift, float* mean, float* rstd, int C, double count,
                 float momentum, float eps, hipStream_t st);
void bn_apply(const void* x, const void* residual, const float* scale, const float* shift, void* y, int64_t M, int C,
              int relu, hipStream_t st);
// ws: 35*C floats (16 partial [2][C] buckets + 3C coefficients); dgamma / dbeta (fp32) accumulate; dres (optional) = dy
// masked by the ReLU (the residual branch's gradient of relu(bn(x) + res)).
// relu: 0 none, 1 mask from y, 2 mask recomputed from x with the forward's
// scale_shift ([2][C]: scale, shift) — y is not read
void bn_bwd(const void* dy, const void* x, const void* y, const float* mean, const float* rstd, const void* gamma,
            int param_dtype, void* dx, void* dres, float* dgamma, float* dbeta, float* ws, int64_t M, int C,
            int relu, hipStream_t st, const float* scale_shift = nullptr, int ws_clean = 0,
            const float* pre_sums = nullptr);   // [2][C] sums from the consumer's dgrad: no reduction pass
struct PoolShape {
  int N = 0, H = 0, W = 0, C = 0, R = 1, S = 1, sh = 1, sw = 1, ph = 0, pw = 0;
  int avg = 0, count_pad = 0;
};
// argmax: one byte per output element (max pooling; may be null when no backward)
void pool2d_fwd(const PoolShape& s, const void* x, void* y, void* argmax, hipStream_t st);
void pool2d_bwd(const PoolShape& s, const void* dy, const void* argmax, void* dx, float beta, hipStream_t st);

// ---- blaslt.hip: hipBLASLt GEMMs with fused epilogues (row-major operands,
// bf16 in, bf16 / fp32 out).  bias: bf16 input (BIAS, GELU_BIAS) or fp32
// bias-gradient output (BGRADB); aux: reserved (no aux epilogue is usable).
enum { EPI_NONE = 0, EPI_BIAS = 1, EPI_GELU_BIAS = 3, EPI_BGRADB = 4 };
int blaslt_probe(int M, int N, int K, bool ta, bool tb, int raw_epi, int bias_t, int aux_t, int out_f32);
bool blaslt_supported(int M, int N, int K, int lda, int ldb, int ldc, bool ta, bool tb, int epi, int out_f32,
                      bool has_beta, int aux_ld, size_t ws_bytes);
// number of heuristic candidates (0: unsupported); `algo` picks one of them
int blaslt_num_algos(int M, int N, int K, int lda, int ldb, int ldc, bool ta, bool tb, int epi, int out_f32,
                     bool has_beta, int aux_ld, size_t ws_bytes);
void blaslt_gemm(const void* A, const void* B, void* C, int M, int N, int K, int lda, int ldb, int ldc, bool ta,
                 bool tb, int epi, const void* bias, void* aux, int aux_ld, float alpha, float beta, int out_f32,
                 void* ws, size_t ws_bytes, hipStream_t st, int algo = 0);
std::vector<int> blaslt_solutions(int M, int N, int K, int lda, int ldb, int ldc, bool ta, bool tb, int out_f32,
                                  bool has_beta, size_t ws_bytes);
std::string blaslt_solution_name(int index);
void blaslt_gemm_solution(const void* A, const void* B, void* C, int M, int N, int K, int lda, int ldb, int ldc,
                          bool ta, bool tb, float alpha, float beta, int out_f32, void* ws, size_t ws_bytes,
                          hipStream_t st, int index);

}  // namespace ffk
