"""Single-process executor / FFModel API tests on CPU (reference analogue:
lib/local-execution/test — LocalTrainingBacking end-to-end on one device,
and the python examples that train small models)."""
import json

import numpy as np
import pytest
import torch

import dist_models as M
from dist_util import assert_params_close, run_distributed, run_single
from flexflow_train_amd.core import (ActiMode, AdamOptimizer, DataType, FFConfig, FFModel, LossType, MetricsType,
                                     SGDOptimizer)
from flexflow_train_amd.ops import base as opbase


def _mlp_model(batch=32):
    cfg = FFConfig()
    cfg.batch_size = batch
    cfg.print_freq = 0
    m = FFModel(cfg)
    x = m.create_tensor([batch, 16], DataType.DT_FLOAT, name="x")
    t = m.dense(x, 64, ActiMode.AC_MODE_RELU, name="fc0")
    t = m.dense(t, 4, name="fc1")
    m.softmax(t, name="sm")
    m.compile(optimizer=SGDOptimizer(m, lr=0.2), loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY,
              metrics=[MetricsType.METRICS_ACCURACY, MetricsType.METRICS_SPARSE_CATEGORICAL_CROSSENTROPY])
    return m


def _blobs(n=512, seed=0):
    rng = np.random.default_rng(seed)
    centers = rng.normal(size=(4, 16)) * 3
    y = rng.integers(0, 4, size=n)
    x = centers[y] + rng.normal(size=(n, 16))
    return x.astype(np.float32), y.astype(np.int32).reshape(n, 1)


def test_fit_learns_blobs(capsys):
    m = _mlp_model()
    x, y = _blobs()
    m.fit(x=x, y=y, epochs=3)
    out = capsys.readouterr().out
    assert "THROUGHPUT" in out and "samples/s" in out
    pm = m.get_perf_metrics()
    assert pm.accuracy > 0.9


def test_get_set_parameter_roundtrip():
    m = _mlp_model()
    ex = m.executor
    w = torch.randn(16, 64)
    ex.set_parameter("fc0.kernel", w)
    torch.testing.assert_close(ex.get_parameter("fc0.kernel"), w)


def test_mha_physical_layout_roundtrip():
    impl = opbase.get_impl("MULTIHEAD_ATTENTION")
    attrs = {"embed_dim": 32, "num_heads": 4, "kdim": 0, "vdim": 0, "_in_features": [32, 32, 32]}
    P = 32 * 8 * 3 + 8 * 32
    for Hl in (4, 2):
        w = torch.randn(P, Hl)
        phys = impl.to_physical(attrs, 0, w)
        torch.testing.assert_close(impl.to_logical(attrs, 0, phys.view(P, Hl)), w)
        b = torch.randn(24, Hl)
        torch.testing.assert_close(impl.to_logical(attrs, 1, impl.to_physical(attrs, 1, b).view(24, Hl)), b)
    # head h of the full weight == head 0 of a 1-head shard
    w = torch.randn(P, 4)
    full = impl.to_physical(attrs, 0, w)
    shard = impl.to_physical(attrs, 0, w[:, 2:3].contiguous())
    qkv_full = full[:32 * 3 * 4 * 8].view(32, 3, 4, 8)
    qkv_shard = shard[:32 * 3 * 1 * 8].view(32, 3, 1, 8)
    torch.testing.assert_close(qkv_full[:, :, 2], qkv_shard[:, :, 0])


def test_grad_clip_norm_counts_each_element_once():
    m = _mlp_model()
    ex = m.executor
    x, y = _blobs(32)
    ex.forward({"x": torch.as_tensor(x)})
    ex.backward(ex.compute_loss(torch.as_tensor(y)))
    n1 = ex.grad_norm()
    ref = sum(float(p.grad.double().pow(2).sum()) for p in ex.params if p.grad is not None) ** 0.5
    assert n1 == pytest.approx(ref, rel=1e-6)


def test_checkpoint_exact_resume(tmp_path):
    x, y = _blobs(64)
    xb, yb = torch.as_tensor(x[:32]), torch.as_tensor(y[:32])
    m1 = _mlp_model()
    for _ in range(2):
        m1.executor.train_step({"x": xb}, yb)
    m1.save_checkpoint(str(tmp_path / "ck"))
    m1.executor.train_step({"x": xb}, yb)
    a = {n: m1.executor.get_parameter(n) for n in m1.executor.parameter_names()}
    m2 = _mlp_model()
    meta = m2.load_checkpoint(str(tmp_path / "ck"))
    assert meta["step"] == 2
    m2.executor.train_step({"x": xb}, yb)
    b = {n: m2.executor.get_parameter(n) for n in m2.executor.parameter_names()}
    assert_params_close(a, b, rtol=1e-6, atol=1e-7)


def test_bert_tiny_trains_on_cpu():
    cfg = FFConfig()
    m = FFModel(cfg)
    feeds, labels = M.bert_tiny(m)
    m.compile(optimizer=AdamOptimizer(m, alpha=3e-3), loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY,
              metrics=[MetricsType.METRICS_SPARSE_CATEGORICAL_CROSSENTROPY])
    ex = m.executor
    losses = []
    for _ in range(15):
        ex.zero_metrics()
        ex.train_step(feeds, labels)
        losses.append(ex.perf_metrics().sparse_cce_loss if hasattr(ex.perf_metrics(), "sparse_cce_loss")
                      else ex.perf_metrics().loss)
    assert losses[-1] < losses[0] * 0.8


def test_strategy_export_import_roundtrip(tmp_path):
    from flexflow_train_amd import _ffcore as C
    from flexflow_train_amd.search.strategy import export_strategy, import_strategy

    m = FFModel(FFConfig())
    M.mlp(m)
    pcg = C.data_parallel_pcg(m.cg, 4)
    path = str(tmp_path / "s.json")
    export_strategy(path, pcg, {3: (0, 1, 2, 3)}, {"world": 4})
    p2, views = import_strategy(path, 4)
    assert p2.structural_hash() == pcg.structural_hash() and views == {3: (0, 1, 2, 3)}
    doc = json.load(open(path))
    assert doc["ops"] and all("device_ids" in o for o in doc["ops"])
    with pytest.raises(ValueError):
        import_strategy(path, 2)
    # round <= 3 files carried contiguous blocks [start, block]
    doc.pop("placements")
    doc["views"] = {"3": [0, 4]}
    json.dump(doc, open(path, "w"))
    assert import_strategy(path, 4)[1] == {3: (0, 1, 2, 3)}


def test_tracing_chrome_export(tmp_path):
    """ExecConfig.profiling: per-op spans, aggregate report and a chrome
    trace (reference: profiling wrapper + --taskgraph export)."""
    import json as _json
    import dist_models as M
    from flexflow_train_amd.core import FFConfig, FFModel, LossType, SGDOptimizer

    cfg = FFConfig()
    cfg.profiling = True
    m = FFModel(cfg)
    feeds, labels = M.mlp(m)
    m.compile(optimizer=SGDOptimizer(m, lr=0.01), loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY)
    m.executor.train_step(feeds, labels)
    rep = m.executor.profile_report()
    assert any(k.endswith(":fwd") for k in rep) and any(k.endswith(":bwd") for k in rep)
    path = m.executor.export_chrome_trace(str(tmp_path / "trace.json"))
    doc = _json.load(open(path))
    xs = [e for e in doc["traceEvents"] if e["ph"] == "X"]
    assert len(xs) >= 6 and all(e["dur"] >= 0 for e in xs)


def test_logging_categories(monkeypatch):
    from flexflow_train_amd.utils.logging import get_logger
    lg = get_logger("search")
    assert lg.name == "flexflow.search"


def test_training_forward_frees_values_after_their_last_reader(monkeypatch):
    """train_step's forward drops each value after its last forward reader
    (the backward reads only saved tensors): intermediate values are gone from
    the environment once the step's forward is done, and the trained
    parameters are bit-identical to a run that keeps every value."""
    def run(free):
        monkeypatch.setenv("FF_FREE_ENV", "1" if free else "0")
        torch.manual_seed(0)
        cfg = FFConfig()
        m = FFModel(cfg)
        feeds, labels = M.bert_tiny(m)
        m.compile(optimizer=AdamOptimizer(m, alpha=3e-3), loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY,
                  metrics=[MetricsType.METRICS_SPARSE_CATEGORICAL_CROSSENTROPY])
        ex = m.executor
        g = torch.Generator().manual_seed(0)
        for n in sorted(ex.parameter_names()):
            ex.set_parameter(n, torch.randn(ex.get_parameter(n).shape, generator=g) * 0.05)
        ex.forward(feeds, training=True, free_env=True)
        weights = {p.terminal for p in ex.params}
        kept = len([v for v in ex._env if v not in weights])
        ex._saved, ex._env = {}, {}
        for _ in range(3):
            ex.train_step(feeds, labels)
        return kept, {n: ex.get_parameter(n).clone() for n in ex.parameter_names()}

    kept_free, p_free = run(True)
    kept_all, p_all = run(False)
    assert kept_free < kept_all / 2, (kept_free, kept_all)
    for n in p_all:
        assert torch.equal(p_free[n], p_all[n]), n
