"""Numerics of the gfx950 HIP kernels against plain PyTorch fp32 references.

Every test runs the native kernel (asserting via kernels.STATS that it ran)
and compares to an fp32 computation of the same op.  Inputs are random and
asymmetric (guide: never validate MFMA layouts with symmetric operands).
"""
import math

import functools

import pytest
import torch

from flexflow_train_amd import kernels as K

pytestmark = pytest.mark.gpu

DEV = "cuda"


# bf16 GEMM outputs against the fp32 product of the same bf16 operands: only
# the output rounding remains (2^-9 per element, ~1.2e-3 relative Frobenius);
# fp32 outputs (beta accumulate into fp32) differ by summation order only
_BF, _F32 = 3e-3, 1e-4


def _rel(a, b):
    a = a.float()
    b = b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def _rel64(a, b):
    """Relative Frobenius error in fp64 (references computed in fp64)."""
    a = a.double()
    b = b.double()
    return ((a - b).norm() / (b.norm() + 1e-300)).item()


# non-GEMM bf16 kernels against fp64 references on the same bf16 inputs: the
# bound is the output rounding plus the bf16 rounding of the kernels' own
# intermediates (attention's P / dS operands), measured at 1.6-2.5e-3
# (profiles/r6/g01_tol_probe.jsonl); a 1 % error in one tile phase fails
_BF_OP = 5e-3


@pytest.mark.parametrize("N", [1024, 768, 4096, 200 * 8])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_layernorm_fwd_bwd(N, dtype):
    torch.manual_seed(0)
    M = 257
    x = torch.randn(M, N, device=DEV, dtype=dtype)
    r = torch.randn(M, N, device=DEV, dtype=dtype)
    g = (1 + 0.1 * torch.randn(N, device=DEV)).to(dtype)
    b = (0.1 * torch.randn(N, device=DEV)).to(dtype)
    n0 = K.STATS["layernorm_fwd"]
    y, s, mean, rstd = K.layernorm_fwd(x, g, b, 1e-5, residual=r)
    assert K.STATS["layernorm_fwd"] == n0 + 1
    bf16 = dtype == torch.bfloat16
    ref = torch.nn.functional.layer_norm(x.double() + r.double(), (N,), g.double(), b.double(), 1e-5)
    assert _rel64(y, ref) < (_BF_OP if bf16 else 1e-5)
    # backward against fp64 LN of the sum the kernel stored (and reads back)
    xs = s.double().requires_grad_(True)
    gf = g.double().requires_grad_(True)
    bf = b.double().requires_grad_(True)
    ref2 = torch.nn.functional.layer_norm(xs, (N,), gf, bf, 1e-5)
    dy = torch.randn(M, N, device=DEV, dtype=dtype)
    ref2.backward(dy.double())
    dg = torch.zeros(N, device=DEV)
    db = torch.zeros(N, device=DEV)
    dx = K.layernorm_bwd(dy, s, mean, rstd, g, dg, db)
    assert _rel64(dx, xs.grad) < (_BF_OP if bf16 else 1e-4)
    assert _rel64(dg, gf.grad) < (1e-3 if bf16 else 1e-4)
    assert _rel64(db, bf.grad) < (1e-5 if bf16 else 1e-4)


@pytest.mark.parametrize("act", ["gelu", "relu", "sigmoid", "tanh"])
def test_bias_act_and_colsum(act):
    torch.manual_seed(1)
    M, N = 1000, 3072
    x = torch.randn(M, N, device=DEV, dtype=torch.bfloat16)
    bias = torch.randn(N, device=DEV, dtype=torch.bfloat16)
    y, pre = K.bias_act_fwd(x, bias, act)
    u = x.float() + bias.float()
    fn = {"gelu": lambda t: torch.nn.functional.gelu(t, approximate="tanh"), "relu": torch.relu,
          "sigmoid": torch.sigmoid, "tanh": torch.tanh}[act]
    uu = u.clone().requires_grad_(True)
    ref = fn(uu)
    assert _rel(y, ref) < 1e-2
    dy = torch.randn(M, N, device=DEV, dtype=torch.bfloat16)
    ref.backward(dy.float())
    dbias = torch.zeros(N, device=DEV)
    g = K.colsum_act(dy, pre, act, dbias)
    assert _rel(g, uu.grad) < 2e-2
    assert _rel(dbias, uu.grad.sum(0)) < 2e-2


@pytest.mark.parametrize("V,Vv,ldt", [(30528, 30522, torch.int64), (50264, 50257, torch.int32), (4096, 4096, torch.int64)])
def test_softmax_ce(V, Vv, ldt):
    """Register-resident fused softmax + CE (NIT 16 / 32 paths, padding
    columns, ignored rows): loss, per-row loss, the gradient (the label column
    explicitly), accuracy against torch."""
    torch.manual_seed(2)
    M = 300
    logits = torch.randn(M, V, device=DEV, dtype=torch.bfloat16) * 3
    lf0 = logits.float()[:, :Vv]
    labels = torch.randint(0, Vv, (M,), device=DEV, dtype=torch.int64)
    labels[::2] = lf0[::2].argmax(1)            # half the rows are "correct"
    labels[5] = -100                            # ignored row
    lf = lf0.clone().requires_grad_(True)
    ref_rows = torch.nn.functional.cross_entropy(lf, labels, reduction="none", ignore_index=-100)
    (ref_rows.sum() / M).backward()
    metrics = torch.zeros(4, device=DEV)
    row_loss = torch.zeros(M, device=DEV)
    g = logits.clone()
    K.softmax_ce(g, labels.to(ldt), 1.0 / M, metrics=metrics, valid_cols=Vv, row_loss=row_loss)
    torch.testing.assert_close(row_loss, ref_rows, rtol=1e-2, atol=1e-2)
    assert abs(metrics[0].item() - ref_rows.sum().item()) < 1e-2 * abs(ref_rows.sum().item())
    assert metrics[2].item() == M - 1
    assert _rel(g[:, :Vv], lf.grad) < 2e-2
    rows = torch.arange(M, device=DEV)[labels >= 0]
    lab_g, lab_ref = g[rows, labels[rows]].float(), lf.grad[rows, labels[rows]]
    assert (lab_g < 0).all() and _rel(lab_g, lab_ref) < 2e-2
    assert g[5].abs().max().item() == 0         # ignored row: zero gradient
    if V > Vv:
        assert g[:, Vv:].abs().max().item() == 0
    valid = labels >= 0
    acc = (lf0.argmax(1) == labels)[valid].float().sum().item()
    assert abs(metrics[1].item() - acc) <= 2


def test_softmax_fwd_bwd():
    torch.manual_seed(3)
    x = torch.randn(64, 1000, device=DEV, dtype=torch.float32).requires_grad_(True)
    y = K.softmax_fwd(x.detach())
    ref = torch.softmax(x, -1)
    assert _rel(y, ref) < 1e-5
    dy = torch.randn_like(y)
    ref.backward(dy)
    dx = K.softmax_bwd(dy, y)
    assert _rel(dx, x.grad) < 1e-4


def test_adam_and_sgd():
    torch.manual_seed(4)
    n = 4096 * 3
    w = torch.randn(n, device=DEV)
    g = torch.randn(n, device=DEV)
    m = torch.zeros(n, device=DEV)
    v = torch.zeros(n, device=DEV)
    wb = torch.empty(n, device=DEV, dtype=torch.bfloat16)
    ref_p = torch.nn.Parameter(w.clone())
    opt = torch.optim.AdamW([ref_p], lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.01)
    for step in range(1, 4):
        ref_p.grad = g.clone()
        opt.step()
        K.adam_step(w, g, m, v, wb, 1e-3, 0.9, 0.999, 1e-8, 0.01 * 1e-3 / 1e-3, step, decoupled=True)
    # AdamW decoupled decay in torch multiplies by lr: w -= lr*wd*w; ours adds wd*w to the update scaled by lr
    assert _rel(w, ref_p.detach()) < 1e-5
    assert _rel(wb, w) < 1e-2
    # SGD with momentum + nesterov + weight decay against torch.optim.SGD
    w2 = torch.randn(n, device=DEV)
    mom = torch.zeros(n, device=DEV)
    p2 = torch.nn.Parameter(w2.clone())
    opt2 = torch.optim.SGD([p2], lr=0.1, momentum=0.9, nesterov=True, weight_decay=1e-4)
    for _ in range(3):
        p2.grad = g.clone()
        opt2.step()
        K.sgd_step(w2, g, mom, None, 0.1, 0.9, 1e-4, True)
    assert _rel(w2, p2.detach()) < 1e-5


@pytest.mark.parametrize("aggr", ["none", "sum", "avg"])
def test_embedding(aggr):
    torch.manual_seed(5)
    n, D = 5000, 256
    W = torch.randn(n, D, device=DEV, dtype=torch.bfloat16)
    idx = torch.randint(0, n, (32, 7), device=DEV)
    out = K.embedding_fwd(idx, W, aggr)
    ref = W.float()[idx]
    if aggr == "sum":
        ref = ref.sum(-2)
    elif aggr == "avg":
        ref = ref.mean(-2)
    assert _rel(out, ref) < _BF
    dout = torch.randn_like(out)
    dW = torch.zeros(n, D, device=DEV)
    K.embedding_bwd(idx, dout, dW, aggr)
    Wf = W.float().requires_grad_(True)
    r = Wf[idx]
    r = r.sum(-2) if aggr == "sum" else (r.mean(-2) if aggr == "avg" else r)
    r.backward(dout.float())
    assert _rel(dW, Wf.grad) < 1e-5   # fp32 accumulation of the same bf16 gradients


@pytest.mark.parametrize("n,rows,D", [(2, 32768, 1024), (5, 3000, 768), (8, 100, 64), (1, 513, 136)])
def test_embedding_small_table_backward(n, rows, D):
    """Token-type sized tables (<= 8 rows): register-accumulated backward."""
    torch.manual_seed(12)
    idx = torch.randint(0, n, (rows,), device=DEV)
    dout = torch.randn(rows, D, device=DEV, dtype=torch.bfloat16)
    dW = torch.full((n, D), 0.5, device=DEV)
    K.embedding_bwd(idx, dout, dW, "none")
    ref = torch.full((n, D), 0.5, device=DEV).index_add_(0, idx, dout.float())
    torch.cuda.synchronize()
    assert _rel(dW, ref) < 1e-4
    # a non-finite gradient row stays in its own table row
    if n > 1 and rows >= 2:
        dout[0] = float("inf")
        dW2 = torch.zeros(n, D, device=DEV)
        K.embedding_bwd(idx, dout, dW2, "none")
        torch.cuda.synchronize()
        other = [e for e in range(n) if e != int(idx[0])]
        assert torch.isfinite(dW2[other]).all()


def _ref_attn(q, k, v, causal):
    """Attention in the inputs' precision (pass fp64 tensors for the bounds)."""
    qf, kf, vf = (t.transpose(1, 2) for t in (q, k, v))  # [B,H,S,D]
    s = qf @ kf.transpose(-1, -2) / math.sqrt(q.shape[-1])
    if causal:
        Sq, Sk = s.shape[-2:]
        mask = torch.ones(Sq, Sk, device=q.device, dtype=torch.bool).triu(1)
        s = s.masked_fill(mask, float("-inf"))
    p = torch.softmax(s, -1)
    return (p @ vf).transpose(1, 2)


@pytest.mark.parametrize("dbias_atomic", [False, True], ids=["slab", "atomic"])
@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("D", [64, 128])
@pytest.mark.parametrize("S", [512, 320])
def test_attention_fwd_bwd(causal, D, S, dbias_atomic):
    torch.manual_seed(6)
    B, H = 2, 4
    qkv = torch.randn(B, S, 3, H, D, device=DEV, dtype=torch.bfloat16)
    q, k, v = qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]
    o, lse = K.attention_fwd(q, k, v, causal=causal)
    qf, kf, vf = (t.double().requires_grad_(True) for t in (q, k, v))
    ref = _ref_attn(qf, kf, vf, causal)
    assert _rel64(o, ref) < _BF_OP, _rel64(o, ref)
    do = torch.randn_like(o)
    ref.backward(do.double())
    dqkv = torch.empty_like(qkv)
    dbias = [torch.full((H * D,), 0.25, device=DEV) for _ in range(3)]
    K.attention_bwd(q, k, v, o, lse, do, dqkv[:, :, 0], dqkv[:, :, 1], dqkv[:, :, 2], causal=causal, dbias=dbias,
                    dbias_atomic=dbias_atomic)
    assert _rel64(dqkv[:, :, 2], vf.grad) < _BF_OP, "dV"
    assert _rel64(dqkv[:, :, 1], kf.grad) < _BF_OP, "dK"
    assert _rel64(dqkv[:, :, 0], qf.grad) < _BF_OP, "dQ"
    # fused projection-bias gradients = column sums over (batch, sequence) of dq / dk / dv
    for i, g in enumerate((qf.grad, kf.grad, vf.grad)):
        ref_sum = g.sum((0, 1)).reshape(-1)
        err = (dbias[i] - 0.25 - ref_sum).abs().max()
        # the key-bias gradient is 0 in exact arithmetic (softmax rows sum to 1):
        # bound the error by the size of the summed terms instead of the sum
        scale = g.abs().sum((0, 1)).max()
        assert err < 3e-2 * scale, ("dbias", i, float(err), float(scale))


@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("S", [512, 320, 64, 100])
def test_attention_fwd_pipelined(causal, S, monkeypatch):
    """The software-pipelined forward (FFK_ATTN_FWD_PIPE=1: S of tile t+1 beside
    tile t's softmax, K one tile ahead of V) matches the default kernel and
    fp32 torch, including one- and two-tile sequences and ragged ends."""
    torch.manual_seed(9)
    B, H, D = 2, 4, 64
    qkv = torch.randn(B, S, 3, H, D, device=DEV, dtype=torch.bfloat16)
    q, k, v = qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]
    monkeypatch.setenv("FFK_ATTN_FWD_PIPE", "0")
    o0, lse0 = K.attention_fwd(q, k, v, causal=causal)
    monkeypatch.setenv("FFK_ATTN_FWD_PIPE", "1")
    o1, lse1 = K.attention_fwd(q, k, v, causal=causal)
    torch.cuda.synchronize()
    ref = _ref_attn(q.double(), k.double(), v.double(), causal)
    assert _rel64(o1, ref) < _BF_OP, _rel64(o1, ref)
    assert _rel(o1, o0) < 1e-2
    assert torch.allclose(lse1, lse0, rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("D,S", [(64, 512), (64, 200), (128, 320)])
def test_attention_bwd_fused_delta(causal, D, S, monkeypatch):
    """delta = rowsum(dO * O) computed inside the dQ kernel (default) gives the
    same gradients as the separate delta pass (FFK_ATTN_BWD_FUSED_DELTA=0)."""
    torch.manual_seed(10)
    B, H = 2, 4
    qkv = torch.randn(B, S, 3, H, D, device=DEV, dtype=torch.bfloat16)
    q, k, v = qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]
    o, lse = K.attention_fwd(q, k, v, causal=causal)
    do = torch.randn_like(o)
    outs = []
    for fused in ("0", "1"):
        monkeypatch.setenv("FFK_ATTN_BWD_FUSED_DELTA", fused)
        dqkv = torch.empty_like(qkv)
        K.attention_bwd(q, k, v, o, lse, do, dqkv[:, :, 0], dqkv[:, :, 1], dqkv[:, :, 2], causal=causal)
        torch.cuda.synchronize()
        outs.append(dqkv.float())
    for i, name in enumerate(("dQ", "dK", "dV")):
        assert _rel(outs[1][:, :, i], outs[0][:, :, i]) < 2e-3, name
    qf, kf, vf = (t.double().requires_grad_(True) for t in (q, k, v))
    _ref_attn(qf, kf, vf, causal).backward(do.double())
    assert _rel64(outs[1][:, :, 0], qf.grad) < _BF_OP


@pytest.mark.parametrize("ta,tb", [(False, False), (False, True), (True, False), (True, True)])
@pytest.mark.parametrize("M,N,Kd", [(512, 1024, 768), (304, 136, 200), (1024, 4096, 1024)])
def test_gemm(ta, tb, M, N, Kd):
    torch.manual_seed(7)
    a = torch.randn(Kd, M, device=DEV, dtype=torch.bfloat16) if ta else torch.randn(M, Kd, device=DEV,
                                                                                     dtype=torch.bfloat16)
    b = torch.randn(N, Kd, device=DEV, dtype=torch.bfloat16) if tb else torch.randn(Kd, N, device=DEV,
                                                                                     dtype=torch.bfloat16)
    af = a.float().t() if ta else a.float()
    bf = b.float().t() if tb else b.float()
    ref = af @ bf
    c = K.gemm(a, b, trans_a=ta, trans_b=tb)
    assert _rel(c, ref) < _BF
    bias = torch.randn(N, device=DEV, dtype=torch.bfloat16)
    pre = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    c2 = K.gemm(a, b, trans_a=ta, trans_b=tb, bias=bias, act="gelu", pre=pre)
    u = ref + bias.float()
    assert _rel(pre, u) < _BF
    assert _rel(c2, torch.nn.functional.gelu(u, approximate="tanh")) < _BF
    c3 = torch.ones(M, N, device=DEV, dtype=torch.float32)
    K.gemm(a, b, trans_a=ta, trans_b=tb, beta=1.0, out=c3)
    assert _rel(c3, ref + 1) < _F32


@pytest.mark.parametrize("ta,tb", [(False, False), (False, True), (True, False), (True, True)])
@pytest.mark.parametrize("M,N,Kd,splits", [(1024, 1024, 1024, 4), (304, 136, 200, 3), (1024, 512, 960, 8)])
def test_gemm_splitk(ta, tb, M, N, Kd, splits):
    """128x128-tile GEMM split over K (uneven K-tile ranges, ragged M / N / K
    edges) with the epilogue (bias, pre-activation, activation, beta) applied
    by the reduction pass."""
    torch.manual_seed(11)
    a = torch.randn(Kd, M, device=DEV, dtype=torch.bfloat16) if ta else torch.randn(M, Kd, device=DEV,
                                                                                     dtype=torch.bfloat16)
    b = torch.randn(N, Kd, device=DEV, dtype=torch.bfloat16) if tb else torch.randn(Kd, N, device=DEV,
                                                                                     dtype=torch.bfloat16)
    ref = (a.float().t() if ta else a.float()) @ (b.float().t() if tb else b.float())
    n0 = K.STATS["gemm_splitk"]
    c = K.gemm(a, b, trans_a=ta, trans_b=tb, splits=splits)
    assert K.STATS["gemm_splitk"] == n0 + 1
    assert _rel(c, ref) < _BF
    bias = torch.randn(N, device=DEV, dtype=torch.bfloat16)
    pre = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    c2 = K.gemm(a, b, trans_a=ta, trans_b=tb, bias=bias, act="relu", pre=pre, splits=splits)
    u = ref + bias.float()
    assert _rel(pre, u) < _BF
    assert _rel(c2, torch.relu(u)) < _BF
    c3 = torch.ones(M, N, device=DEV, dtype=torch.float32)
    K.gemm(a, b, trans_a=ta, trans_b=tb, beta=1.0, out=c3, splits=splits)
    assert _rel(c3, ref + 1) < _F32


@pytest.mark.parametrize("ta,tb", [(False, False), (False, True), (True, False), (True, True)])
@pytest.mark.parametrize("M,N,Kd,splits", [(512, 768, 256, 1), (264, 520, 512, 1), (1024, 1024, 4096, 8),
                                            (296, 136, 1024, 3)])
def test_gemm256(ta, tb, M, N, Kd, splits):
    torch.manual_seed(11)
    a = torch.randn(Kd, M, device=DEV, dtype=torch.bfloat16) if ta else torch.randn(M, Kd, device=DEV,
                                                                                     dtype=torch.bfloat16)
    b = torch.randn(N, Kd, device=DEV, dtype=torch.bfloat16) if tb else torch.randn(Kd, N, device=DEV,
                                                                                     dtype=torch.bfloat16)
    af = a.float().t() if ta else a.float()
    bf = b.float().t() if tb else b.float()
    ref = af @ bf
    c = K.gemm256(a, b, trans_a=ta, trans_b=tb, splits=splits)
    assert _rel(c, ref) < _BF
    c3 = torch.ones(M, N, device=DEV, dtype=torch.float32)
    K.gemm256(a, b, trans_a=ta, trans_b=tb, beta=1.0, out=c3, splits=splits)
    assert _rel(c3, ref + 1) < _F32
    if splits == 1:
        bias = torch.randn(N, device=DEV, dtype=torch.bfloat16)
        pre = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
        c2 = K.gemm256(a, b, trans_a=ta, trans_b=tb, bias=bias, act="gelu", pre=pre)
        u = ref + bias.float()
        assert _rel(pre, u) < _BF
        assert _rel(c2, torch.nn.functional.gelu(u, approximate="tanh")) < _BF


@pytest.mark.parametrize("variant", [0, 1, 2, 3, 4, 5, 6, 8, 9, 10, 11],
                         ids=["mfma32x32x16", "mfma16x16x32", "pingpong", "wave128", "wave128dma", "wave128pers",
                              "wave128dma2", "tile64", "nt8wave", "wave128regstage", "pingpong8"])
@pytest.mark.parametrize("ta,tb", [(False, False), (False, True), (True, False), (True, True)])
@pytest.mark.parametrize("M,N,Kd,splits", [(512, 768, 256, 1), (264, 520, 512, 1), (1024, 1024, 4096, 8),
                                            (296, 136, 1024, 3), (2048, 1536, 640, 1),
                                            # more work items than CUs: the persistent kernels loop
                                            (4096, 4352, 128, 1), (2048, 2048, 1024, 8),
                                            # 17 K-tiles over 5 splits: gemmt's uneven split (4,4,3,3,3)
                                            (512, 768, 1088, 5),
                                            # DLRM MLP shapes (one K-tile; a 64-wide output)
                                            (1024, 512, 64, 1), (1024, 64, 512, 1)])
def test_gemmp(ta, tb, M, N, Kd, splits, variant):
    """Phase-pipelined persistent GEMM (gemmp.hip; variant 1 = gemmq.hip on
    16x16x32 MFMAs, variant 2 = gemmr.hip ping-pong schedule, 3-6 = gemmt.hip
    one wave per SIMD: register / B by LDS-DMA staging, persistent, both by LDS-DMA; 8 = gemms.hip 64x64 tiles):
    plain / beta / split-K, the fused
    bias+activation+pre-activation epilogue and the activation-gradient +
    bias-gradient epilogue, against fp32 torch."""
    import functools
    gemmp = functools.partial(K.gemmp, variant=variant)
    torch.manual_seed(13)
    a = torch.randn(Kd, M, device=DEV, dtype=torch.bfloat16) if ta else torch.randn(M, Kd, device=DEV,
                                                                                     dtype=torch.bfloat16)
    b = torch.randn(N, Kd, device=DEV, dtype=torch.bfloat16) if tb else torch.randn(Kd, N, device=DEV,
                                                                                     dtype=torch.bfloat16)
    af = a.float().t() if ta else a.float()
    bf = b.float().t() if tb else b.float()
    ref = af @ bf
    # bf16 inputs, fp32 accumulation: against the fp32 product of the same
    # bf16 values only the output rounding remains (bf16: 2^-9 per element,
    # ~1.2e-3 relative Frobenius); a systematic 0.5 % error in one K-tile
    # phase would exceed these bounds
    BF, F32 = 3e-3, 2e-5
    c = gemmp(a, b, trans_a=ta, trans_b=tb, splits=splits)
    assert _rel(c, ref) < BF
    c3 = torch.ones(M, N, device=DEV, dtype=torch.float32)
    gemmp(a, b, trans_a=ta, trans_b=tb, beta=1.0, out=c3, splits=splits)
    assert _rel(c3, ref + 1) < F32
    # bf16 accumulate (gemmt: the paired 16-B read-modify-write epilogue)
    c4 = torch.full((M, N), 0.5, device=DEV, dtype=torch.bfloat16)
    gemmp(a, b, trans_a=ta, trans_b=tb, beta=1.0, out=c4, splits=splits)
    assert _rel(c4, ref + 0.5) < BF
    if splits == 1:
        bias = torch.randn(N, device=DEV, dtype=torch.bfloat16)
        pre = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
        c2 = gemmp(a, b, trans_a=ta, trans_b=tb, bias=bias, act="gelu", pre=pre)
        u = ref + bias.float()
        assert _rel(gemmp(a, b, trans_a=ta, trans_b=tb, bias=bias), u) < BF   # bias only
        assert _rel(pre, u) < BF
        assert _rel(c2, torch.nn.functional.gelu(u, approximate="tanh")) < BF
        aux = torch.randn(M, N, device=DEV, dtype=torch.bfloat16)
        db = torch.full((N,), 0.5, device=DEV)
        g = gemmp(a, b, trans_a=ta, trans_b=tb, act="gelu", aux=aux, act_bwd=True, dbias=db)
        x = aux.float().requires_grad_(True)
        torch.nn.functional.gelu(x, approximate="tanh").backward(torch.ones_like(x))
        gr = ref * x.grad
        assert _rel(g, gr) < BF
        if variant >= 3:   # gemmt / gemms sum the fp32 gradient (before its bf16 rounding)
            assert _rel(db, gr.sum(0) + 0.5) < 1e-3
        else:              # the other kernels sum the stored bf16 values
            assert _rel(db, g.float().sum(0) + 0.5) < 1e-4


@pytest.mark.parametrize("mode", [0, 1, 2, 4, 5, 6])
@pytest.mark.parametrize("M,N,Kd", [(512, 768, 128), (264, 520, 512), (1040, 264, 1216), (2048, 1024, 3072),
                                    (256, 256, 64), (520, 264, 192)])
def test_gemmpp_modes(mode, M, N, Kd):
    """Eight-wave ping-pong A B^T kernel (gemmpp.hip, variant 11) in every
    DMA / priority mode (GemmPParams.dbg = 16 | mode): plain, bf16 accumulate
    and bias epilogues against the fp32 product of the same bf16 operands,
    partial edge tiles included."""
    torch.manual_seed(5)
    a = torch.randn(M, Kd, device=DEV, dtype=torch.bfloat16)
    b = torch.randn(N, Kd, device=DEV, dtype=torch.bfloat16)
    ref = a.float() @ b.float().t()
    run = functools.partial(K.gemmp, a, b, trans_b=True, variant=11, _dbg=16 | mode)
    assert _rel(run(), ref) < 3e-3
    c = torch.full((M, N), 0.5, device=DEV, dtype=torch.bfloat16)
    run(beta=1.0, out=c)
    assert _rel(c, ref + 0.5) < 3e-3
    bias = torch.randn(N, device=DEV, dtype=torch.bfloat16)
    assert _rel(run(bias=bias), ref + bias.float()) < 3e-3


def test_dropout_and_cast():
    x = torch.randn(1 << 16, device=DEV, dtype=torch.bfloat16)
    y = K.dropout(x, 0.25, 1234)
    keep = (y != 0).float().mean().item()
    assert abs(keep - 0.75) < 0.02
    y2 = K.dropout(x, 0.25, 1234)
    assert torch.equal(y, y2)
    nz = y != 0
    assert torch.allclose(y[nz].float(), x[nz].float() / 0.75, rtol=1e-2, atol=1e-2)
    f = torch.empty(x.numel(), device=DEV)
    K.cast_(x, f)
    assert torch.equal(f, x.float())


@pytest.mark.parametrize("ta,tb", [(False, False), (False, True), (True, False), (True, True)])
@pytest.mark.parametrize("Z,M,N,Kd", [(12, 128, 64, 64), (3, 264, 136, 192), (2, 512, 512, 512)])
def test_bmm(ta, tb, Z, M, N, Kd):
    """Batched product on the 64x64-tile kernel (gemms.hip, blockIdx.z =
    product), against fp32 torch; plain and beta-accumulate."""
    torch.manual_seed(5)
    a = torch.randn(Z, Kd, M, device=DEV, dtype=torch.bfloat16) if ta else torch.randn(Z, M, Kd, device=DEV,
                                                                                       dtype=torch.bfloat16)
    b = torch.randn(Z, N, Kd, device=DEV, dtype=torch.bfloat16) if tb else torch.randn(Z, Kd, N, device=DEV,
                                                                                       dtype=torch.bfloat16)
    assert K.bmm_supported(a, b, ta, tb)
    ref = (a.float().transpose(-1, -2) if ta else a.float()) @ (b.float().transpose(-1, -2) if tb else b.float())
    c = K.bmm(a, b, ta, tb)
    assert _rel(c, ref) < _BF
    acc = torch.ones(Z, M, N, device=DEV, dtype=torch.float32)
    K.bmm(a, b, ta, tb, out=acc, beta=1.0)
    assert _rel(acc, ref + 1) < _F32
