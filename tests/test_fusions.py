"""Executor fusion passes against the unfused step (FFConfig.perform_fusion
= False), parameter by parameter after a few training steps:

* pre-LN residual stream (GPT): EW_ADD -> LAYERNORM where the sum also feeds
  the next residual add -> one FUSED_ADD_LAYERNORM step with two outputs;
  its backward adds the other consumers' gradient (layernorm_bwd dres);
* LINEAR(+bias) -> add+LayerNorm: the norm backward accumulates the Linear's
  bias gradient (layernorm_bwd dsum) — GPU path only;
* LINEAR(GELU) -> LINEAR: input-gradient GEMM with the activation-gradient
  epilogue (gemmp) — GPU path, when measured faster.

CPU runs the torch fallbacks of the same steps; the gpu-marked test runs the
HIP kernels in bf16."""
import pytest
import torch

from flexflow_train_amd.core import AdamOptimizer, FFConfig, FFModel, LossType, MetricsType
from flexflow_train_amd.models.transformer import GPTConfig, build_gpt


def _gpt(fuse: bool):
    cfg = FFConfig()
    cfg.perform_fusion = fuse
    m = FFModel(cfg)
    gc = GPTConfig(vocab_size=128, hidden_size=64, num_layers=2, num_heads=2, sequence_length=16, batch_size=4,
                   pad_vocab_to=64)
    build_gpt(m, gc)
    m.compile(optimizer=AdamOptimizer(m, alpha=1e-3), loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY,
              metrics=[MetricsType.METRICS_SPARSE_CATEGORICAL_CROSSENTROPY])
    ex = m.executor
    g = torch.Generator().manual_seed(1)
    for n in sorted(ex.parameter_names()):
        ex.set_parameter(n, torch.randn(ex.get_parameter(n).shape, generator=g) * 0.05)
    dev = ex.cfg.device
    ids = torch.randint(0, 128, (4, 17), generator=g, dtype=torch.int32)
    feeds = {"input_ids": ids[:, :16].contiguous().to(dev),
             "position_ids": torch.arange(16, dtype=torch.int32).expand(4, 16).contiguous().to(dev)}
    return ex, feeds, ids[:, 1:].long().to(dev)


def _compare(tol):
    a, feeds, labels = _gpt(True)
    b, _, _ = _gpt(False)
    fused = [s for s in a.steps if s.op_type == "FUSED_ADD_LAYERNORM"]
    assert sum(1 for s in fused if s.ctx.extra.get("emit_sum")) >= 4, "pre-LN add+norm not fused"
    srcs = [s.ctx.extra["dbias_src"][0].op_type for s in fused if "dbias_src" in s.ctx.extra]
    assert "LINEAR" in srcs
    assert not any(s.op_type == "FUSED_ADD_LAYERNORM" for s in b.steps)
    for _ in range(3):
        a.train_step(feeds, labels)
        b.train_step(feeds, labels)
    for n in a.parameter_names():
        torch.testing.assert_close(a.get_parameter(n), b.get_parameter(n), **tol)
    return a


@pytest.mark.skipif(torch.cuda.is_available(), reason="exercises the CPU fallback path")
def test_pre_ln_fusion_matches_unfused_cpu():
    _compare(dict(rtol=1e-4, atol=1e-5))


@pytest.mark.gpu
def test_pre_ln_and_bias_fusions_match_unfused_gpu():
    from flexflow_train_amd import kernels as K
    a = _compare(dict(rtol=3e-2, atol=3e-3))
    assert a.cfg.device.type == "cuda" and K.available()


def _bert(fuse: bool):
    from flexflow_train_amd.models.bert import BertConfig, build_bert
    cfg = FFConfig()
    cfg.perform_fusion = fuse
    m = FFModel(cfg)
    bc = BertConfig(vocab_size=128, hidden_size=64, num_heads=2, dim_feedforward=128, num_encoder_layers=2,
                    sequence_length=16, batch_size=4, max_position_embeddings=16, type_vocab_size=2)
    build_bert(m, bc)
    m.compile(optimizer=AdamOptimizer(m, alpha=1e-3), loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY,
              metrics=[MetricsType.METRICS_SPARSE_CATEGORICAL_CROSSENTROPY])
    ex = m.executor
    g = torch.Generator().manual_seed(2)
    for n in sorted(ex.parameter_names()):
        ex.set_parameter(n, torch.randn(ex.get_parameter(n).shape, generator=g) * 0.05)
    dev = ex.cfg.device
    feeds = {"input_ids": torch.randint(0, 128, (4, 16), generator=g, dtype=torch.int32).to(dev),
             "position_ids": torch.arange(16, dtype=torch.int32).expand(4, 16).contiguous().to(dev),
             "token_type_ids": torch.randint(0, 2, (4, 16), generator=g, dtype=torch.int32).to(dev)}
    return ex, feeds, torch.randint(0, 128, (4, 16), generator=g).to(dev)


def _compare_bert(tol):
    a, feeds, labels = _bert(True)
    b, _, _ = _bert(False)
    srcs = [s.ctx.extra["dbias_src"][0].op_type for s in a.steps if "dbias_src" in s.ctx.extra]
    assert "MULTIHEAD_ATTENTION" in srcs and "LINEAR" in srcs, srcs
    for _ in range(3):
        a.train_step(feeds, labels)
        b.train_step(feeds, labels)
    for n in a.parameter_names():
        torch.testing.assert_close(a.get_parameter(n), b.get_parameter(n), **tol)


@pytest.mark.skipif(torch.cuda.is_available(), reason="exercises the CPU fallback path")
def test_post_ln_bias_fusion_matches_unfused_cpu():
    _compare_bert(dict(rtol=1e-4, atol=1e-5))


@pytest.mark.gpu
def test_post_ln_bias_fusion_matches_unfused_gpu():
    _compare_bert(dict(rtol=3e-2, atol=3e-3))


def _side_consumer_model(fuse: bool):
    """x -> dense -> s = add(h, x); a consumer of s ("side") is created BEFORE
    the LayerNorm of s, so it sits between the add and the norm in
    topological order.  The fused add+norm must run at the add's position."""
    from flexflow_train_amd.core import ActiMode, DataType, SGDOptimizer
    cfg = FFConfig()
    cfg.perform_fusion = fuse
    m = FFModel(cfg)
    x = m.create_tensor([8, 16], DataType.DT_FLOAT, name="x")
    h = m.dense(x, 16, ActiMode.AC_MODE_RELU, name="h")
    s = m.add(h, x, name="sum")
    r = m.dense(s, 16, name="side")
    n = m.layer_norm(s, axes=[-1], name="ln")
    o = m.add(n, r, name="join")
    m.softmax(m.dense(o, 4, name="head"))
    m.compile(optimizer=SGDOptimizer(m, lr=0.05), loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY,
              metrics=[MetricsType.METRICS_ACCURACY])
    ex = m.executor
    g = torch.Generator().manual_seed(3)
    for nm in sorted(ex.parameter_names()):
        ex.set_parameter(nm, torch.randn(ex.get_parameter(nm).shape, generator=g) * 0.2)
    dev = ex.cfg.device
    feeds = {"x": torch.randn(8, 16, generator=g).to(dev)}
    return ex, feeds, torch.randint(0, 4, (8,), generator=g).to(dev)


def test_add_ln_fusion_with_sum_consumer_before_norm():
    a, feeds, labels = _side_consumer_model(True)
    b, _, _ = _side_consumer_model(False)
    names = [s.name for s in b.steps if s.kind == "compute"]
    assert names.index("side") < names.index("ln"), names
    fused = [s for s in a.steps if s.op_type == "FUSED_ADD_LAYERNORM"]
    assert len(fused) == 1 and fused[0].ctx.extra.get("emit_sum")
    order = [s.name for s in a.steps if s.kind == "compute"]
    assert order.index("ln") < order.index("side"), order
    for _ in range(3):
        a.train_step(feeds, labels)
        b.train_step(feeds, labels)
    tol = dict(rtol=1e-4, atol=1e-5) if a.cfg.device.type == "cpu" else dict(rtol=3e-2, atol=3e-3)
    for nm in a.parameter_names():
        torch.testing.assert_close(a.get_parameter(nm), b.get_parameter(nm), **tol)


def _softmax_mse(identity: bool):
    from flexflow_train_amd.core import DataType, SGDOptimizer
    cfg = FFConfig()
    cfg.softmax_identity_backward = identity
    m = FFModel(cfg)
    x = m.create_tensor([8, 16], DataType.DT_FLOAT, name="x")
    m.softmax(m.dense(x, 4, name="fc"))
    m.compile(optimizer=SGDOptimizer(m, lr=0.1), loss_type=LossType.LOSS_MEAN_SQUARED_ERROR_AVG_REDUCE,
              metrics=[MetricsType.METRICS_MEAN_SQUARED_ERROR])
    ex = m.executor
    g = torch.Generator().manual_seed(4)
    for nm in sorted(ex.parameter_names()):
        ex.set_parameter(nm, torch.randn(ex.get_parameter(nm).shape, generator=g) * 0.3)
    dev = ex.cfg.device
    feeds = {"x": torch.randn(8, 16, generator=g).to(dev)}
    return ex, feeds, torch.rand(8, 4, generator=g).to(dev)


@pytest.mark.skipif(torch.cuda.is_available(), reason="exercises the CPU fallback path")
@pytest.mark.parametrize("identity", [False, True])
def test_softmax_backward_under_mse(identity):
    """MSE after a softmax.  Default: the loss gradient goes through the
    softmax Jacobian.  Reference-parity flag: the softmax backward is the
    reference's identity copy (softmax_kernels.cu:63-72), so the MSE
    gradient lands on the logits unchanged.  Checked on the bias update."""
    ex, feeds, y = _softmax_mse(identity)
    assert any(s.ctx is not None and s.ctx.extra.get("identity_backward") for s in ex.steps) == identity
    bname = next(n for n in ex.parameter_names() if n.endswith("bias"))
    wname = next(n for n in ex.parameter_names() if n != bname)
    W, b = ex.get_parameter(wname).clone().double(), ex.get_parameter(bname).clone().double()
    x = feeds["x"].double()
    z = x @ (W if W.shape[0] == 16 else W.t()) + b
    p = torch.softmax(z, -1)
    dp = 2.0 * (p - y.double()) / p.numel()
    dz = dp if identity else p * (dp - (dp * p).sum(-1, keepdim=True))
    ex.train_step(feeds, y)
    torch.testing.assert_close(ex.get_parameter(bname).double(), b - 0.1 * dz.sum(0), rtol=1e-5, atol=1e-6)
