"""Native CPU local execution (csrc/ffcore/src/local_exec.cc, the reference's
lib/local-execution: LocalTrainingBacking + task registry + slots backing +
LocalCostEstimator) against the framework's PyTorch-backed executor on the
same graphs and weights — BASELINE config 1 runs through it."""
import numpy as np
import pytest
import torch

from flexflow_train_amd import _ffcore as C
from flexflow_train_amd.core import (ActiMode, AdamOptimizer, AggrMode, DataType, FFConfig, FFModel, LossType,
                                     MetricsType, PoolType, SGDOptimizer)


def _mlp(m, B):
    x = m.create_tensor([B, 32], DataType.DT_FLOAT, name="x")
    t = m.dense(x, 24, ActiMode.AC_MODE_RELU, name="d1")
    t = m.dense(t, 16, ActiMode.AC_MODE_TANH, name="d2")
    m.softmax(m.dense(t, 10, name="d3"))
    return ["x"]


def _encoder(m, B):
    x = m.create_tensor([B, 8, 16], DataType.DT_FLOAT, name="x")
    h = m.dense(x, 16, ActiMode.AC_MODE_GELU, name="ff1")
    h = m.layer_norm(m.add(x, h, name="res"), [-1], name="ln")
    h = m.scalar_multiply(h, 0.5, name="half")
    h = m.flat(h, name="flat")
    m.softmax(m.dense(h, 6, name="out"))
    return ["x"]


def _embed_concat(m, B):
    ids = m.create_tensor([B, 3], DataType.DT_INT32, name="ids")
    d = m.create_tensor([B, 4], DataType.DT_FLOAT, name="dense")
    e = m.embedding(ids, 50, 4, AggrMode.AGGR_MODE_SUM, name="emb")
    t = m.concat([e, d], 1, name="cat")
    m.dense(t, 1, ActiMode.AC_MODE_SIGMOID, name="out")
    return ["ids", "dense"]


def _cnn(m, B):
    x = m.create_tensor([B, 3, 8, 8], DataType.DT_FLOAT, name="img")
    t = m.conv2d(x, 6, 3, 3, 1, 1, 1, 1, ActiMode.AC_MODE_RELU, name="c1")
    t = m.batch_norm(t, relu=True, name="bn")
    t = m.pool2d(t, 2, 2, 2, 2, 0, 0, PoolType.POOL_MAX, name="mp")
    t = m.conv2d(t, 4, 3, 3, 2, 2, 1, 1, groups=2, name="c2")
    t = m.pool2d(t, 2, 2, 1, 1, 1, 1, PoolType.POOL_AVG, name="ap")
    m.softmax(m.dense(m.flat(t, name="fl"), 5, name="out"))
    return ["img"]


def _math_shapes(m, B):
    x = m.create_tensor([B, 4, 6], DataType.DT_FLOAT, name="x")
    s = m.sigmoid(x, name="sg")
    a = m.add(m.rsqrt(m.scalar_add(s, 0.5, name="sh"), name="rs"), m.pow(s, 3.0, name="p3"), name="a1")
    b = m.add(m.sin(x, name="si"), m.cos(m.exp(m.scalar_multiply(x, 0.3, name="sc"), name="ex"), name="co"), name="a2")
    c = m.add(a, m.elu(b, inplace=False, name="el"), name="a3")
    c = m.reverse(m.transpose(c, [0, 2, 1], name="tr"), 1, name="rv")          # [B, 6, 4]
    l, r = m.split(c, [2, 4], 1, name="sp")
    t = m.concat([m.reduce_sum(l, [1], keepdims=True, name="rsum"), m.mean(r, [1], keepdims=True, name="rmean")], 1,
                 name="cc")                                                     # [B, 2, 4]
    m.softmax(m.dense(m.flat(t, name="fl"), 3, name="out"))
    return ["x"]


def _attention(m, B):
    x = m.create_tensor([B, 5, 16], DataType.DT_FLOAT, name="x")
    kv = m.create_tensor([B, 7, 12], DataType.DT_FLOAT, name="kv")
    h = m.multihead_attention(x, x, x, 16, 4, name="self")
    h = m.multihead_attention(h, kv, kv, 16, 2, kdim=6, vdim=5, name="cross")
    m.softmax(m.dense(m.flat(h, name="fl"), 4, name="out"))
    return ["x", "kv"]


def _run(build, opt, loss, feeds, labels, steps=3, B=8):
    cfg = FFConfig()
    cfg.batch_size = B
    cfg.cpu_only = True
    m = FFModel(cfg)
    build(m, B)
    ce = loss == "ce"
    o = SGDOptimizer(m, lr=0.1, momentum=0.9, weight_decay=1e-3) if opt == "sgd" else \
        AdamOptimizer(m, alpha=0.01, weight_decay=1e-3)
    m.compile(optimizer=o, loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY if ce
              else LossType.LOSS_MEAN_SQUARED_ERROR_AVG_REDUCE,
              metrics=[MetricsType.METRICS_ACCURACY] if ce else [MetricsType.METRICS_MEAN_SQUARED_ERROR])
    ex = m.executor
    kw = dict(optimizer="sgd", lr=0.1, momentum=0.9, weight_decay=1e-3) if opt == "sgd" else \
        dict(optimizer="adam", lr=0.01, weight_decay=1e-3)
    b = C.LocalTrainingBacking(m.cg, loss="sparse_categorical_crossentropy" if ce else "mean_squared_error", **kw)
    for n in ex.parameter_names():
        b.set_weight(n, ex.get_parameter(n).numpy())
    for _ in range(steps):
        ex.train_step({k: torch.as_tensor(v) for k, v in feeds.items()}, torch.as_tensor(labels))
        for k, v in feeds.items():
            b.set_input(k, v.astype(np.float32))
        b.train_step(labels.astype(np.float32))
    for n in ex.parameter_names():
        np.testing.assert_allclose(np.asarray(b.get_weight(n)), ex.get_parameter(n).numpy(), rtol=2e-4, atol=2e-5,
                                   err_msg=n)
    return b, ex


@pytest.mark.parametrize("opt", ["sgd", "adam"])
def test_mlp_matches_executor(opt):
    rng = np.random.default_rng(0)
    X = rng.standard_normal((8, 32)).astype(np.float32)
    Y = rng.integers(0, 10, (8, 1)).astype(np.int32)
    b, ex = _run(_mlp, opt, "ce", {"x": X}, Y)
    mm = b.metrics()
    pm = ex.perf_metrics()
    assert mm["samples"] == pm.train_all and mm["correct"] == pm.train_correct
    assert abs(mm["loss_sum"] / mm["samples"] - pm.loss) < 1e-4


def test_encoder_block_matches_executor():
    rng = np.random.default_rng(1)
    X = rng.standard_normal((8, 8, 16)).astype(np.float32)
    Y = rng.integers(0, 6, (8, 1)).astype(np.int32)
    _run(_encoder, "sgd", "ce", {"x": X}, Y)


def test_embedding_concat_mse_matches_executor():
    rng = np.random.default_rng(2)
    ids = rng.integers(0, 50, (8, 3)).astype(np.int32)
    d = rng.standard_normal((8, 4)).astype(np.float32)
    Y = rng.random((8, 1)).astype(np.float32)
    _run(_embed_concat, "adam", "mse", {"ids": ids, "dense": d}, Y)


def test_cnn_conv_bn_pool_matches_executor():
    rng = np.random.default_rng(4)
    X = rng.standard_normal((8, 3, 8, 8)).astype(np.float32)
    Y = rng.integers(0, 5, (8, 1)).astype(np.int32)
    _run(_cnn, "sgd", "ce", {"img": X}, Y)


def test_math_and_shape_ops_match_executor():
    rng = np.random.default_rng(5)
    X = rng.standard_normal((8, 4, 6)).astype(np.float32)
    Y = rng.integers(0, 3, (8, 1)).astype(np.int32)
    _run(_math_shapes, "adam", "ce", {"x": X}, Y)


def test_attention_matches_executor():
    rng = np.random.default_rng(6)
    X = rng.standard_normal((8, 5, 16)).astype(np.float32)
    KV = rng.standard_normal((8, 7, 12)).astype(np.float32)
    Y = rng.integers(0, 4, (8, 1)).astype(np.int32)
    _run(_attention, "sgd", "ce", {"x": X, "kv": KV}, Y)


def test_fit_local_execution_flag():
    cfg = FFConfig()
    cfg.batch_size = 16
    cfg.print_freq = 0
    cfg.local_execution = True
    m = FFModel(cfg)
    _mlp(m, 16)
    m.compile(optimizer=SGDOptimizer(m, lr=0.1), loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY,
              metrics=[MetricsType.METRICS_ACCURACY])
    assert m.local_backing is not None
    rng = np.random.default_rng(3)
    X = rng.standard_normal((64, 32)).astype(np.float32)
    Y = (X[:, :10].argmax(1)).astype(np.int32).reshape(-1, 1)     # learnable labels
    before = m.executor.get_parameter("d3.kernel").clone()
    m.fit(x=X, y=Y, epochs=20)
    assert not torch.equal(before, m.executor.get_parameter("d3.kernel"))   # synced back
    mm = m.local_backing.metrics()
    assert mm["correct"] / mm["samples"] > 0.5
    times = m.local_backing.layer_times_ms()
    assert set(times) >= {"d1", "d2", "d3"}


def test_cost_estimator_and_registry():
    ops = C.LocalTrainingBacking.registered_ops()
    for t in ("LINEAR", "SOFTMAX", "LAYERNORM", "EMBEDDING", "CONCAT", "BATCHMATMUL", "EW_ADD", "RELU", "CONV2D",
              "POOL2D", "BATCHNORM", "MULTIHEAD_ATTENTION", "TRANSPOSE", "SPLIT", "REDUCE_SUM", "GATHER", "EXP"):
        assert t in ops
    lin = C.OpAttrs("LINEAR", out_channels=64)
    ms = C.measure_op_cost_ms(lin, [C.TensorShape([32, 128], C.DataType.FLOAT)])
    ms_big = C.measure_op_cost_ms(lin, [C.TensorShape([512, 128], C.DataType.FLOAT)])
    assert 0 < ms < ms_big


def test_unsupported_op_is_rejected():
    cfg = FFConfig()
    cfg.batch_size = 2
    m = FFModel(cfg)
    x = m.create_tensor([2, 16], DataType.DT_FLOAT, name="x")
    m.top_k(x, 4)
    with pytest.raises(ValueError):
        C.LocalTrainingBacking(m.cg)
