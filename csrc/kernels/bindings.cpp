// pybind11 module `_ffkernels`: thin launchers over the gfx950 kernel library.
// Pointers and streams cross as integers (tensor.data_ptr(),
// torch.cuda.current_stream().cuda_stream); validation of shapes / dtypes /
// contiguity happens in flexflow_train_amd/kernels/__init__.py before any
// launch.  Errors from the launch path surface as Python exceptions.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "kernels.h"

namespace py = pybind11;
using namespace ffk;

static inline void* P(uintptr_t p) { return reinterpret_cast<void*>(p); }
static inline float* F(uintptr_t p) { return reinterpret_cast<float*>(p); }
static inline hipStream_t S(uintptr_t s) { return reinterpret_cast<hipStream_t>(s); }

static AttnTensors::T tview(const py::tuple& t) {
  AttnTensors::T r;
  if (t.size() != 4) throw std::invalid_argument("attention tensor view must be (ptr, sb, ss, sh)");
  r.p = P(t[0].cast<uintptr_t>());
  r.sb = t[1].cast<int64_t>();
  r.ss = t[2].cast<int64_t>();
  r.sh = t[3].cast<int64_t>();
  return r;
}

PYBIND11_MODULE(_ffkernels, m) {
  m.doc() = "flexflow_train_amd gfx950 HIP kernels";
  m.attr("ARCH") = "gfx950";

  m.def("layernorm_fwd", [](int dt, uintptr_t x, uintptr_t res, uintptr_t sum_out, uintptr_t g, uintptr_t b,
                            uintptr_t y, uintptr_t mean, uintptr_t rstd, int M, int N, float eps, uintptr_t st) {
    layernorm_fwd(dt, P(x), P(res), P(sum_out), P(g), P(b), P(y), F(mean), F(rstd), M, N, eps, S(st));
  });
  m.def("layernorm_bwd_grid", &layernorm_bwd_grid);
  m.def("layernorm_bwd", [](int dt, uintptr_t dy, uintptr_t s, uintptr_t mean, uintptr_t rstd, uintptr_t g,
                            uintptr_t dx, uintptr_t dg, uintptr_t db, uintptr_t ws, int M, int N, uintptr_t st,
                            uintptr_t dres, uintptr_t dsum) {
    layernorm_bwd(dt, P(dy), P(s), F(mean), F(rstd), P(g), P(dx), F(dg), F(db), F(ws), M, N, S(st), P(dres),
                  F(dsum));
  }, py::arg("dt"), py::arg("dy"), py::arg("s"), py::arg("mean"), py::arg("rstd"), py::arg("g"), py::arg("dx"),
        py::arg("dg"), py::arg("db"), py::arg("ws"), py::arg("M"), py::arg("N"), py::arg("st"), py::arg("dres") = 0,
        py::arg("dsum") = 0);
  m.def("bias_act_fwd", [](int dt, uintptr_t x, uintptr_t bias, uintptr_t pre, uintptr_t y, int64_t M, int64_t N,
                           int op, float alpha, uintptr_t st) {
    bias_act_fwd(dt, P(x), P(bias), P(pre), P(y), M, N, op, alpha, S(st));
  });
  m.def("act_bwd", [](int dt, uintptr_t dy, uintptr_t pre, uintptr_t dx, int64_t n, int op, float alpha,
                      uintptr_t st) { act_bwd(dt, P(dy), P(pre), P(dx), n, op, alpha, S(st)); });
  m.def("colsum_act", [](int dt, uintptr_t dy, uintptr_t pre, uintptr_t dx, uintptr_t dbias, int64_t M, int64_t N,
                         int op, float alpha, uintptr_t st) {
    colsum_act(dt, P(dy), P(pre), P(dx), F(dbias), M, N, op, alpha, S(st));
  });
  m.def("dropout_fwd", [](int dt, uintptr_t x, uintptr_t y, int64_t n, float p, uint64_t seed, uintptr_t st) {
    dropout_fwd(dt, P(x), P(y), n, p, seed, S(st));
  });
  m.def("cast", [](int di, int dout, uintptr_t x, uintptr_t y, int64_t n, uintptr_t st) {
    cast(di, dout, P(x), P(y), n, S(st));
  });
  m.def("axpby", [](int dt, uintptr_t x, uintptr_t y, int64_t n, float a, float b, uintptr_t st) {
    axpby(dt, P(x), P(y), n, a, b, S(st));
  });
  m.def("softmax_ce", [](int dt, int label_bits, uintptr_t logits, uintptr_t labels, uintptr_t row_loss,
                         uintptr_t metrics, uintptr_t row_stats, int M, int V, int V_valid, float grad_scale,
                         int ignore_index, int write_grad, uintptr_t st) {
    softmax_ce(dt, label_bits, P(logits), P(labels), F(row_loss), F(metrics), F(row_stats), M, V, V_valid,
               grad_scale, ignore_index, write_grad, S(st));
  });
  m.def("softmax_fwd", [](int dt, uintptr_t x, uintptr_t y, int M, int N, uintptr_t st) {
    softmax_fwd(dt, P(x), P(y), M, N, S(st));
  });
  m.def("softmax_bwd", [](int dt, uintptr_t dy, uintptr_t y, uintptr_t dx, int M, int N, uintptr_t st) {
    softmax_bwd(dt, P(dy), P(y), P(dx), M, N, S(st));
  });
  m.def("adam_step", [](uintptr_t w, uintptr_t g, int gdt, uintptr_t mm, uintptr_t v, uintptr_t wb, int64_t n,
                        float lr, float b1, float b2, float eps, float wd, int step, float gs, int decoupled,
                        uintptr_t hp, uintptr_t st) {
    adam_step(F(w), P(g), gdt, F(mm), F(v), P(wb), n, lr, b1, b2, eps, wd, step, gs, decoupled,
              reinterpret_cast<const float*>(hp), S(st));
  });
  m.def("sgd_step", [](uintptr_t w, uintptr_t g, int gdt, uintptr_t mom, uintptr_t wb, int64_t n, float lr,
                       float momentum, float wd, int nesterov, float gs, uintptr_t st) {
    sgd_step(F(w), P(g), gdt, F(mom), P(wb), n, lr, momentum, wd, nesterov, gs, S(st));
  });
  // tables: [(master, grad, grad_bf16, compute, idx, idx64, n_idx, rows, dim, scratch_off), ...]
  m.def("sparse_sgd_rows", [](const std::vector<py::tuple>& tables, uintptr_t scratch, float step, uintptr_t st) {
    SparseSgdArgs a{};
    if (tables.size() > static_cast<size_t>(kMaxSparseTables))
      throw std::invalid_argument("sparse_sgd_rows: too many tables");
    a.nt = static_cast<int>(tables.size());
    for (size_t i = 0; i < tables.size(); ++i) {
      const py::tuple& t = tables[i];
      if (t.size() != 10) throw std::invalid_argument("sparse_sgd_rows: table tuple must have 10 fields");
      SparseSgdTable& d = a.t[i];
      d.master = F(t[0].cast<uintptr_t>());
      d.grad = P(t[1].cast<uintptr_t>());
      d.grad_bf16 = t[2].cast<int>();
      d.compute = P(t[3].cast<uintptr_t>());
      d.idx = P(t[4].cast<uintptr_t>());
      d.idx64 = t[5].cast<int>();
      d.n_idx = t[6].cast<int64_t>();
      d.rows = t[7].cast<int64_t>();
      d.dim = t[8].cast<int>();
      d.scratch_off = t[9].cast<int64_t>();
    }
    sparse_sgd_rows(a, F(scratch), step, S(st));
  });
  // pieces: [(ptr, len, off), ...] along the axis of `big` ([outer, total, inner])
  m.def("slice_copy_multi", [](int dt, uintptr_t big, const std::vector<py::tuple>& pieces, int64_t outer,
                               int64_t inner, int64_t total, int to_slice, uintptr_t st) {
    SlicePieces p{};
    if (pieces.size() > static_cast<size_t>(kMaxSlicePieces))
      throw std::invalid_argument("slice_copy_multi: too many pieces");
    p.n = static_cast<int>(pieces.size());
    for (size_t k = 0; k < pieces.size(); ++k) {
      p.ptr[k] = P(pieces[k][0].cast<uintptr_t>());
      p.len[k] = pieces[k][1].cast<int64_t>();
      p.off[k] = pieces[k][2].cast<int64_t>();
    }
    slice_copy_multi(dt, P(big), p, outer, inner, total, to_slice, S(st));
  });
  m.def("sum_squares", [](uintptr_t x, int64_t n, uintptr_t out, uintptr_t st) {
    sum_squares(F(x), n, F(out), S(st));
  });
  m.def("embedding_fwd", [](int dt, int ib, uintptr_t idx, uintptr_t W, uintptr_t out, int64_t B, int L, int D,
                            int mode, int64_t n, uintptr_t st) {
    embedding_fwd(dt, ib, P(idx), P(W), P(out), B, L, D, mode, n, S(st));
  });
  m.def("embedding_bwd", [](int dt, int ib, uintptr_t idx, uintptr_t dout, uintptr_t dW, int64_t B, int L, int D,
                            int mode, int64_t n, uintptr_t ws, int copies, uintptr_t st) {
    embedding_bwd(dt, ib, P(idx), P(dout), F(dW), B, L, D, mode, n, F(ws), copies, S(st));
  });
  m.def("attention_fwd", [](py::tuple q, py::tuple k, py::tuple v, py::tuple o, uintptr_t lse, int B, int H, int Sq,
                            int Sk, int D, float scale, bool causal, uintptr_t st) {
    AttnTensors t;
    t.q = tview(q);
    t.k = tview(k);
    t.v = tview(v);
    t.o = tview(o);
    t.lse = F(lse);
    attention_fwd(t, B, H, Sq, Sk, D, scale, causal, S(st));
  });
  m.def("attention_bwd", [](py::tuple q, py::tuple k, py::tuple v, py::tuple o, py::tuple dout, py::tuple dq,
                            py::tuple dk, py::tuple dv, uintptr_t lse, uintptr_t delta, int B, int H, int Sq, int Sk,
                            int D, float scale, bool causal, uintptr_t st, uintptr_t dbq, uintptr_t dbk,
                            uintptr_t dbv, int64_t db_ld) {
    AttnTensors t;
    t.q = tview(q);
    t.k = tview(k);
    t.v = tview(v);
    t.o = tview(o);
    t.dout = tview(dout);
    t.dq = tview(dq);
    t.dk = tview(dk);
    t.dv = tview(dv);
    t.lse = F(lse);
    t.delta = F(delta);
    t.dbq = F(dbq);
    t.dbk = F(dbk);
    t.dbv = F(dbv);
    t.db_ld = db_ld;
    attention_bwd(t, B, H, Sq, Sk, D, scale, causal, S(st));
  }, py::arg("q"), py::arg("k"), py::arg("v"), py::arg("o"), py::arg("dout"), py::arg("dq"), py::arg("dk"),
        py::arg("dv"), py::arg("lse"), py::arg("delta"), py::arg("B"), py::arg("H"), py::arg("Sq"), py::arg("Sk"),
        py::arg("D"), py::arg("scale"), py::arg("causal"), py::arg("st"), py::arg("dbq") = 0, py::arg("dbk") = 0,
        py::arg("dbv") = 0, py::arg("db_ld") = 0);
  m.def("gemm", [](uintptr_t A, uintptr_t B, uintptr_t C, uintptr_t bias, uintptr_t pre, int M, int N, int K,
                   int lda, int ldb, int ldc, bool ta, bool tb, int act, float alpha, float beta, int out_f32,
                   uintptr_t st, int splits, uintptr_t ws) {
    gemm_bf16_ex(P(A), P(B), P(C), P(bias), P(pre), M, N, K, lda, ldb, ldc, ta, tb, act, alpha, beta, out_f32, S(st),
                 splits, F(ws));
  }, py::arg("A"), py::arg("B"), py::arg("C"), py::arg("bias"), py::arg("pre"), py::arg("M"), py::arg("N"),
     py::arg("K"), py::arg("lda"), py::arg("ldb"), py::arg("ldc"), py::arg("ta"), py::arg("tb"), py::arg("act"),
     py::arg("alpha"), py::arg("beta"), py::arg("out_f32"), py::arg("st"), py::arg("splits") = 1,
     py::arg("ws") = 0);
  // ---- tensorops
  auto shape = [](const std::vector<int64_t>& v) {
    if (v.size() > 6) throw std::invalid_argument("tensorops: at most 6 dims");
    NdShape s;
    s.nd = static_cast<int>(v.size());
    for (size_t i = 0; i < v.size(); ++i) s.size[i] = v[i];
    return s;
  };
  auto strides = [](const std::vector<int64_t>& v) {
    if (v.size() > 6) throw std::invalid_argument("tensorops: at most 6 dims");
    NdStrides s;
    for (size_t i = 0; i < v.size(); ++i) s.s[i] = v[i];
    return s;
  };
  m.def("binary_nd", [=](int dt, uintptr_t a, uintptr_t b, uintptr_t y, std::vector<int64_t> s,
                         std::vector<int64_t> sa, std::vector<int64_t> sb, int op, uintptr_t st) {
    binary_nd(dt, P(a), P(b), P(y), shape(s), strides(sa), strides(sb), op, S(st));
  });
  m.def("binary_grad_nd", [=](int dt, uintptr_t dy, uintptr_t a, uintptr_t b, uintptr_t g, std::vector<int64_t> s,
                              std::vector<int64_t> sa, std::vector<int64_t> sb, int op, int which, uintptr_t st) {
    binary_grad_nd(dt, P(dy), P(a), P(b), F(g), shape(s), strides(sa), strides(sb), op, which, S(st));
  });
  m.def("sum_to", [=](int dt, uintptr_t full, uintptr_t out, std::vector<int64_t> s, std::vector<int64_t> t,
                      float beta, uintptr_t st) {
    sum_to(dt, F(full), P(out), shape(s), shape(t), beta, S(st));
  });
  m.def("permute_nd", [=](int dt, uintptr_t x, uintptr_t y, std::vector<int64_t> out_shape,
                          std::vector<int64_t> in_strides, uintptr_t st) {
    permute_nd(dt, P(x), P(y), shape(out_shape), strides(in_strides), S(st));
  });
  m.def("slice_copy", [](int dt, uintptr_t x, uintptr_t y, int64_t outer, int64_t len, int64_t inner, int64_t total,
                         int64_t off, int to_slice, int acc, uintptr_t st) {
    slice_copy(dt, P(x), P(y), outer, len, inner, total, off, to_slice, acc, S(st));
  });
  m.def("reverse_axis", [](int dt, uintptr_t x, uintptr_t y, int64_t outer, int64_t len, int64_t inner,
                           uintptr_t st) { reverse_axis(dt, P(x), P(y), outer, len, inner, S(st)); });
  m.def("gather_axis", [](int dt, int ib, uintptr_t x, uintptr_t idx, uintptr_t y, int64_t outer, int64_t lx,
                          int64_t li, int64_t inner, uintptr_t st) {
    gather_axis(dt, ib, P(x), P(idx), P(y), outer, lx, li, inner, S(st));
  });
  m.def("scatter_add_axis", [](int dt, int ib, uintptr_t dy, uintptr_t idx, uintptr_t dx, int64_t outer, int64_t lx,
                               int64_t li, int64_t inner, uintptr_t st) {
    scatter_add_axis(dt, ib, P(dy), P(idx), F(dx), outer, lx, li, inner, S(st));
  });
  m.def("reduce_axis", [](int dt, uintptr_t x, uintptr_t y, int64_t outer, int64_t red, int64_t inner, int op,
                          uintptr_t st) { reduce_axis(dt, P(x), P(y), outer, red, inner, op, S(st)); });
  m.def("topk_rows", [](int dt, uintptr_t x, uintptr_t vals, uintptr_t idx, int64_t rows, int n, int k,
                        uintptr_t st) {
    topk_rows(dt, P(x), P(vals), reinterpret_cast<int64_t*>(idx), rows, n, k, S(st));
  });
  m.def("unary_op", [](int dt, uintptr_t x, uintptr_t dy, uintptr_t y, int64_t n, int op, float s, int bwd,
                       uintptr_t st) { unary_op(dt, P(x), P(dy), P(y), n, op, s, bwd, S(st)); });
  m.def("zero_fill", [](uintptr_t p, int64_t bytes, uintptr_t st) { zero_fill(P(p), bytes, S(st)); });
  m.def("mse_loss_full", [](int dt, int ldt, uintptr_t p, uintptr_t y, uintptr_t g, uintptr_t metrics, int64_t n,
                            float scale, int full, int64_t cols, int64_t rows, uintptr_t st) {
    mse_loss_full(dt, ldt, P(p), P(y), P(g), F(metrics), n, scale, full, cols, rows, S(st));
  });
  m.def("narrow_linear_fwd", [](uintptr_t x, uintptr_t w, uintptr_t bias, uintptr_t y, uintptr_t pre, int64_t M,
                                int64_t K, int64_t N, int act, uintptr_t st) {
    narrow_linear_fwd(P(x), P(w), F(bias), P(y), P(pre), M, K, N, act, S(st));
  });
  m.def("narrow_linear_dgrad", [](uintptr_t dy, uintptr_t pre, uintptr_t w, uintptr_t dx, int64_t M, int64_t K,
                                  int64_t N, int act, float beta, uintptr_t st) {
    narrow_linear_dgrad(P(dy), P(pre), P(w), P(dx), M, K, N, act, beta, S(st));
  });
  m.def("narrow_wgrad_blocks", [](int64_t M) { return narrow_wgrad_blocks(M); });
  m.def("narrow_linear_wgrad", [](uintptr_t x, uintptr_t dy, uintptr_t pre, uintptr_t part, int blocks, uintptr_t dw,
                                  int dw_dtype, float beta, uintptr_t db, int64_t M, int64_t K, int64_t N, int act,
                                  uintptr_t st) {
    narrow_linear_wgrad(P(x), P(dy), P(pre), F(part), blocks, P(dw), dw_dtype, beta, F(db), M, K, N, act, S(st));
  });
  m.def("mse_loss", [](int dt, uintptr_t p, uintptr_t y, uintptr_t g, uintptr_t metrics, int64_t n, float scale,
                       uintptr_t st) { mse_loss(dt, P(p), P(y), P(g), F(metrics), n, scale, S(st)); });
  m.def("init_tensor", [=](int dt, uintptr_t out, std::vector<int64_t> piece, std::vector<int64_t> full,
                           std::vector<int64_t> lo, int kind, uint64_t seed, float a, float b, float c, float d,
                           uintptr_t st) {
    init_tensor(dt, P(out), shape(piece), shape(full), strides(lo), kind, seed, a, b, c, d, S(st));
  });
  m.def("gemmp_supported", &gemmp_supported);
  m.def("bmm", [](uintptr_t A, uintptr_t B, uintptr_t C, int batch, int M, int N, int K, int lda, int ldb, int ldc,
                  int64_t sA, int64_t sB, int64_t sC, bool ta, bool tb, float alpha, float beta, int out_f32,
                  uintptr_t st) {
    bmm_bf16(P(A), P(B), P(C), batch, M, N, K, lda, ldb, ldc, sA, sB, sC, ta, tb, alpha, beta, out_f32, S(st));
  });
  m.def("gemmp", [](uintptr_t A, uintptr_t B, uintptr_t C, uintptr_t bias, uintptr_t pre, uintptr_t aux,
                    uintptr_t dbias, int M, int N, int K, int lda, int ldb, int ldc, bool ta, bool tb, int act,
                    bool act_bwd, float alpha, float beta, int out_f32, int splits, uintptr_t ws, uintptr_t st,
                    int dbg, int variant) {
    GemmPParams p;
    p.A = P(A); p.B = P(B); p.C = P(C); p.bias = P(bias); p.pre = P(pre); p.aux = P(aux); p.dbias = F(dbias);
    p.workspace = F(ws);
    p.M = M; p.N = N; p.K = K; p.lda = lda; p.ldb = ldb; p.ldc = ldc; p.trans_a = ta; p.trans_b = tb;
    p.act = act; p.act_bwd = act_bwd; p.alpha = alpha; p.beta = beta; p.out_f32 = out_f32; p.splits = splits;
    p.dbg = dbg;
    p.variant = variant;
    gemmp_bf16(p, S(st));
  }, py::arg("A"), py::arg("B"), py::arg("C"), py::arg("bias"), py::arg("pre"), py::arg("aux"), py::arg("dbias"),
        py::arg("M"), py::arg("N"), py::arg("K"), py::arg("lda"), py::arg("ldb"), py::arg("ldc"), py::arg("ta"),
        py::arg("tb"), py::arg("act"), py::arg("act_bwd"), py::arg("alpha"), py::arg("beta"), py::arg("out_f32"),
        py::arg("splits"), py::arg("ws"), py::arg("st"), py::arg("dbg") = 0, py::arg("variant") = 0);
  m.def("gemm256_supported", &gemm256_supported);
  m.def("gemm256", [](uintptr_t A, uintptr_t B, uintptr_t C, uintptr_t bias, uintptr_t pre, int M, int N, int K,
                      int lda, int ldb, int ldc, bool ta, bool tb, int act, float alpha, float beta, int out_f32,
                      int splits, uintptr_t ws, uintptr_t st) {
    gemm256_bf16(P(A), P(B), P(C), P(bias), P(pre), M, N, K, lda, ldb, ldc, ta, tb, act, alpha, beta, out_f32,
                 splits, reinterpret_cast<float*>(ws), S(st));
  });

  // conv geometry crosses as a list [N,H,W,C,K,R,S,sh,sw,ph,pw,dh,dw]
  auto cshape = [](const std::vector<int>& v) {
    if (v.size() != 13) throw std::invalid_argument("conv shape must have 13 entries");
    ConvShape c;
    c.N = v[0]; c.H = v[1]; c.W = v[2]; c.C = v[3]; c.K = v[4]; c.R = v[5]; c.S = v[6];
    c.sh = v[7]; c.sw = v[8]; c.ph = v[9]; c.pw = v[10]; c.dh = v[11]; c.dw = v[12];
    return c;
  };
  m.def("pad_channels_nhwc", [=](uintptr_t x, uintptr_t y, int64_t N, int C, int H, int W, int64_t sn, int64_t sc,
                                 int64_t sh, int64_t sw, int Cp, uintptr_t st) {
    pad_channels_nhwc(P(x), P(y), N, C, H, W, sn, sc, sh, sw, Cp, S(st));
  });
  m.def("conv2d_stats_ws_floats", [=](std::vector<int> shp) { return conv2d_stats_ws_floats(cshape(shp)); });
  m.def("conv2d_wgrad_ws_floats",
        [=](std::vector<int> shp, int splits) { return conv2d_wgrad_ws_floats(cshape(shp), splits); });
  m.def("conv2d_fwd", [=](std::vector<int> shp, uintptr_t x, uintptr_t w, uintptr_t bias, uintptr_t y,
                          uintptr_t stats, uintptr_t ws, int act, uintptr_t st) {
    conv2d_fwd(cshape(shp), P(x), P(w), P(bias), P(y), F(stats), F(ws), act, S(st));
  });
  m.def("conv2d_dgrad", [=](std::vector<int> shp, uintptr_t dy, uintptr_t w, uintptr_t dx, float beta,
                            uintptr_t st) { conv2d_dgrad(cshape(shp), P(dy), P(w), P(dx), beta, S(st)); });
  m.def("conv2d_dgrad_bn_ws_floats", [=](std::vector<int> shp) { return conv2d_dgrad_bn_ws_floats(cshape(shp)); });
  m.def("conv2d_dgrad_bn", [=](std::vector<int> shp, uintptr_t dy, uintptr_t w, uintptr_t dx, uintptr_t x,
                               uintptr_t mean, uintptr_t rstd, uintptr_t ss, uintptr_t sums, uintptr_t ws,
                               uintptr_t st) {
    ConvBnBwd b{P(x), F(mean), F(rstd), F(ss), F(sums), F(ws)};
    conv2d_dgrad(cshape(shp), P(dy), P(w), P(dx), 0.f, S(st), &b);
  });
  m.def("conv2d_wgrad", [=](std::vector<int> shp, uintptr_t x, uintptr_t dy, uintptr_t dw, uintptr_t ws, int splits,
                            uintptr_t st) { conv2d_wgrad(cshape(shp), P(x), P(dy), F(dw), F(ws), splits, S(st)); });
  m.def("conv2d_grouped_wexp_elems",
        [=](std::vector<int> shp, int groups) { return conv2d_grouped_wexp_elems(cshape(shp), groups); });
  m.def("conv2d_grouped_wgrad_ws_floats",
        [=](std::vector<int> shp, int groups) { return conv2d_grouped_wgrad_ws_floats(cshape(shp), groups); });
  m.def("conv2d_grouped_expand", [=](std::vector<int> shp, int groups, uintptr_t w, uintptr_t wexp, uintptr_t st) {
    conv2d_grouped_expand(cshape(shp), groups, P(w), P(wexp), S(st));
  });
  m.def("conv2d_grouped_fwd", [=](std::vector<int> shp, int groups, uintptr_t x, uintptr_t wexp, uintptr_t bias,
                                  uintptr_t y, uintptr_t stats, uintptr_t ws, int act, uintptr_t st) {
    conv2d_grouped_fwd(cshape(shp), groups, P(x), P(wexp), P(bias), P(y), F(stats), F(ws), act, S(st));
  });
  m.def("conv2d_grouped_dgrad", [=](std::vector<int> shp, int groups, uintptr_t dy, uintptr_t wexp, uintptr_t dx,
                                    float beta, uintptr_t st) {
    conv2d_grouped_dgrad(cshape(shp), groups, P(dy), P(wexp), P(dx), beta, S(st));
  });
  m.def("conv2d_grouped_wgrad", [=](std::vector<int> shp, int groups, uintptr_t x, uintptr_t dy, uintptr_t dw,
                                    uintptr_t ws, uintptr_t st) {
    conv2d_grouped_wgrad(cshape(shp), groups, P(x), P(dy), F(dw), F(ws), S(st));
  });
  m.def("gemm_f32", [](uintptr_t A, uintptr_t B, uintptr_t C, uintptr_t bias, uintptr_t pre, int64_t M, int64_t N,
                       int64_t K, int64_t lda, int64_t ldb, int64_t ldc, bool ta, bool tb, int act, float alpha,
                       float beta, int in_f32, int out_f32, uintptr_t st, int batch, int64_t sa, int64_t sb,
                       int64_t sc) {
    gemm_f32(P(A), P(B), P(C), P(bias), P(pre), M, N, K, lda, ldb, ldc, ta, tb, act, alpha, beta, in_f32, out_f32,
             S(st), batch, sa, sb, sc);
  });
  m.def("conv32_fwd", [=](std::vector<int> shp, int groups, uintptr_t x, uintptr_t w, uintptr_t bias, uintptr_t y,
                          int act, int in_f32, uintptr_t st) {
    conv32_fwd(cshape(shp), groups, P(x), P(w), P(bias), P(y), act, in_f32, S(st));
  });
  m.def("conv32_dgrad", [=](std::vector<int> shp, int groups, uintptr_t dy, uintptr_t w, uintptr_t dx, float beta,
                            int in_f32, uintptr_t st) {
    conv32_dgrad(cshape(shp), groups, P(dy), P(w), P(dx), beta, in_f32, S(st));
  });
  m.def("conv32_wgrad", [=](std::vector<int> shp, int groups, uintptr_t x, uintptr_t dy, uintptr_t dw, int in_f32,
                            uintptr_t st) { conv32_wgrad(cshape(shp), groups, P(x), P(dy), F(dw), in_f32, S(st)); });
  m.def("bn_stats", [](uintptr_t x, uintptr_t stats, int64_t M, int C, uintptr_t st, uintptr_t ws, int ws_clean) {
    bn_stats(P(x), F(stats), M, C, S(st), F(ws), ws_clean);
  });
  m.def("bn_finalize", [](uintptr_t stats, uintptr_t g, uintptr_t b, int pdt, uintptr_t rm, uintptr_t rv,
                          uintptr_t scale, uintptr_t shift, uintptr_t mean, uintptr_t rstd, int C, double count,
                          float momentum, float eps, uintptr_t st) {
    bn_finalize(F(stats), P(g), P(b), pdt, F(rm), F(rv), F(scale), F(shift), F(mean), F(rstd), C, count, momentum,
                eps, S(st));
  });
  m.def("bn_apply", [](uintptr_t x, uintptr_t res, uintptr_t scale, uintptr_t shift, uintptr_t y, int64_t M, int C,
                       int relu, uintptr_t st) { bn_apply(P(x), P(res), F(scale), F(shift), P(y), M, C, relu, S(st)); });
  m.def("bn_bwd", [](uintptr_t dy, uintptr_t x, uintptr_t y, uintptr_t mean, uintptr_t rstd, uintptr_t g, int pdt,
                     uintptr_t dx, uintptr_t dres, uintptr_t dg, uintptr_t db, uintptr_t ws, int64_t M, int C,
                     int relu, uintptr_t st, uintptr_t ss, int ws_clean, uintptr_t pre_sums) {
    bn_bwd(P(dy), P(x), P(y), F(mean), F(rstd), P(g), pdt, P(dx), P(dres), F(dg), F(db), F(ws), M, C, relu, S(st),
           F(ss), ws_clean, F(pre_sums));
  }, py::arg("dy"), py::arg("x"), py::arg("y"), py::arg("mean"), py::arg("rstd"), py::arg("g"), py::arg("pdt"),
     py::arg("dx"), py::arg("dres"), py::arg("dg"), py::arg("db"), py::arg("ws"), py::arg("M"), py::arg("C"),
     py::arg("relu"), py::arg("st"), py::arg("ss"), py::arg("ws_clean"), py::arg("pre_sums") = 0);
  // pool geometry: [N,H,W,C,R,S,sh,sw,ph,pw,avg,count_pad]
  auto pshape = [](const std::vector<int>& v) {
    if (v.size() != 12) throw std::invalid_argument("pool shape must have 12 entries");
    PoolShape p;
    p.N = v[0]; p.H = v[1]; p.W = v[2]; p.C = v[3]; p.R = v[4]; p.S = v[5];
    p.sh = v[6]; p.sw = v[7]; p.ph = v[8]; p.pw = v[9]; p.avg = v[10]; p.count_pad = v[11];
    return p;
  };
  m.def("pool2d_fwd", [=](std::vector<int> shp, uintptr_t x, uintptr_t y, uintptr_t arg, uintptr_t st) {
    pool2d_fwd(pshape(shp), P(x), P(y), P(arg), S(st));
  });
  m.def("pool2d_bwd", [=](std::vector<int> shp, uintptr_t dy, uintptr_t arg, uintptr_t dx, float beta,
                          uintptr_t st) { pool2d_bwd(pshape(shp), P(dy), P(arg), P(dx), beta, S(st)); });

  m.def("blaslt_supported", &blaslt_supported);
  m.def("blaslt_num_algos", &blaslt_num_algos);
  m.def("blaslt_probe", &blaslt_probe);
  m.def("blaslt_gemm", [](uintptr_t A, uintptr_t B, uintptr_t C, int M, int N, int K, int lda, int ldb, int ldc,
                          bool ta, bool tb, int epi, uintptr_t bias, uintptr_t aux, int aux_ld, float alpha, float beta,
                          int out_f32, uintptr_t ws, size_t ws_bytes, uintptr_t st, int algo) {
    blaslt_gemm(P(A), P(B), P(C), M, N, K, lda, ldb, ldc, ta, tb, epi, P(bias), P(aux), aux_ld, alpha, beta, out_f32,
                P(ws), ws_bytes, S(st), algo);
  });
  m.def("blaslt_solutions", &blaslt_solutions);
  m.def("blaslt_solution_name", &blaslt_solution_name);
  m.def("blaslt_gemm_solution", [](uintptr_t A, uintptr_t B, uintptr_t C, int M, int N, int K, int lda, int ldb,
                                   int ldc, bool ta, bool tb, float alpha, float beta, int out_f32, uintptr_t ws,
                                   size_t ws_bytes, uintptr_t st, int index) {
    blaslt_gemm_solution(P(A), P(B), P(C), M, N, K, lda, ldb, ldc, ta, tb, alpha, beta, out_f32, P(ws), ws_bytes,
                         S(st), index);
  });
}
