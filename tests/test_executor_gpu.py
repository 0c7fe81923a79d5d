"""Executor on the GPU: whole-model numerics of the HIP path against the CPU
fp32 path, and hipGraph replay of the training step against eager steps."""
import pytest
import torch

import dist_models as M
from flexflow_train_amd import kernels as K
from flexflow_train_amd.core import AdamOptimizer, FFConfig, FFModel, LossType, MetricsType

pytestmark = pytest.mark.gpu


def _model(device_cpu: bool = False):
    cfg = FFConfig()
    m = FFModel(cfg)
    feeds, labels = M.bert_tiny(m)
    m.compile(optimizer=AdamOptimizer(m, alpha=1e-3), loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY,
              metrics=[MetricsType.METRICS_SPARSE_CATEGORICAL_CROSSENTROPY])
    return m, feeds, labels


def test_native_kernels_loaded():
    assert K.available(), "the HIP extension must load on a GPU box"


def test_graphed_step_matches_eager():
    torch.manual_seed(0)
    a, feeds, labels = _model()
    b, _, _ = _model()
    dev = a.executor.cfg.device
    feeds = {k: v.to(dev) for k, v in feeds.items()}
    labels = labels.to(dev)
    for _ in range(3):
        a.executor.train_step(feeds, labels)
    step = b.executor.make_graphed_train_step(feeds, labels, warmup=2)
    step()
    torch.cuda.synchronize()
    for n in a.executor.parameter_names():
        torch.testing.assert_close(b.executor.get_parameter(n), a.executor.get_parameter(n), rtol=2e-2, atol=2e-3)
    # replays keep training (loss goes down)
    b.executor.zero_metrics()
    for _ in range(20):
        step()
    first = b.executor.perf_metrics().loss
    b.executor.zero_metrics()
    for _ in range(5):
        step()
    assert b.executor.perf_metrics().loss < first


def test_gpu_loss_matches_cpu_fp32():
    m, feeds, labels = _model()
    ex = m.executor
    names = ex.parameter_names()
    params = {n: ex.get_parameter(n).cpu() for n in names}
    ex.zero_metrics()
    ex.forward({k: v.to(ex.cfg.device) for k, v in feeds.items()})
    ex.compute_loss(labels.to(ex.cfg.device))
    gpu_loss = ex.perf_metrics().loss
    # CPU reference executor with the same weights
    from flexflow_train_amd.parallel.comm import DistContext
    from flexflow_train_amd.runtime.executor import ExecConfig, Executor
    from flexflow_train_amd.runtime.optimizer import AdamConfig

    cpu = Executor(m.pcg, DistContext(0, 1, torch.device("cpu")), ExecConfig(compute_dtype=torch.float32),
                   loss_type="sparse_categorical_crossentropy", optimizer=AdamConfig(),
                   valid_classes=m.valid_classes)
    cpu.init_parameters()
    for n, t in params.items():
        cpu.set_parameter(n, t)
    cpu.zero_metrics()
    cpu.forward(feeds)
    cpu.compute_loss(labels)
    assert abs(cpu.perf_metrics().loss - gpu_loss) < 0.02 * abs(cpu.perf_metrics().loss) + 1e-3


def test_trace_api_replays_hipgraph():
    """ffconfig.begin_trace/end_trace around forward/backward/update (the
    reference's Legion-trace idiom) captures and replays a hipGraph; the
    result matches the same loop run eagerly."""
    import numpy as np

    def run(traced):
        cfg = FFConfig()
        m = FFModel(cfg)
        feeds, labels = M.bert_tiny(m)
        m.compile(optimizer=AdamOptimizer(m, alpha=1e-3),
                  loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY,
                  metrics=[MetricsType.METRICS_SPARSE_CATEGORICAL_CROSSENTROPY])
        for it in range(5):
            for k, v in feeds.items():
                m._pending_feeds[k] = v.numpy()
            m._pending_feeds["label"] = np.roll(labels.numpy(), it, axis=1)
            if traced:
                cfg.begin_trace(111)
            m.forward()
            m.zero_gradients()
            m.backward()
            m.update()
            if traced:
                cfg.end_trace(111)
        torch.cuda.synchronize()
        return m, {n: m.executor.get_parameter(n) for n in m.executor.parameter_names()}

    mt, pt = run(True)
    assert mt._traces[111]["step"] is not None, "the traced iteration was not captured"
    _, pe = run(False)
    for n in pe:
        torch.testing.assert_close(pt[n], pe[n], rtol=2e-2, atol=2e-3)


def test_fit_uses_hipgraph():
    import numpy as np
    from flexflow_train_amd.core import ActiMode, DataType, SGDOptimizer

    cfg = FFConfig()
    cfg.batch_size = 32
    cfg.print_freq = 0
    m = FFModel(cfg)
    x = m.create_tensor([32, 64], DataType.DT_FLOAT, name="x")
    t = m.dense(x, 128, ActiMode.AC_MODE_RELU, name="fc1")
    t = m.dense(t, 10, name="fc2")
    m.softmax(t, name="sm")
    m.compile(optimizer=SGDOptimizer(m, lr=0.05), loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY,
              metrics=[MetricsType.METRICS_ACCURACY, MetricsType.METRICS_SPARSE_CATEGORICAL_CROSSENTROPY])
    rng = np.random.default_rng(0)
    xs = rng.standard_normal((256, 64)).astype(np.float32)
    ys = (xs[:, :10].argmax(1)).astype(np.int32).reshape(-1, 1)
    m.fit(x=xs, y=ys, epochs=6)
    assert getattr(m.executor, "_graph", None) is not None
    assert m.executor.perf_metrics().get_accuracy() > 50.0


def _mlp_gelu(fuse: bool):
    from flexflow_train_amd.core import ActiMode, DataType
    cfg = FFConfig()
    cfg.perform_fusion = fuse
    m = FFModel(cfg)
    x = m.create_tensor([256, 128], DataType.DT_FLOAT, name="x")
    t = m.dense(x, 512, ActiMode.AC_MODE_GELU, name="fc1")
    t = m.dense(t, 128, name="fc2")
    t = m.dense(t, 16, name="out")
    m.softmax(t, name="sm")
    m.compile(optimizer=AdamOptimizer(m, alpha=1e-3), loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY,
              metrics=[MetricsType.METRICS_SPARSE_CATEGORICAL_CROSSENTROPY])
    ex = m.executor
    g = torch.Generator().manual_seed(5)
    for n in sorted(ex.parameter_names()):
        ex.set_parameter(n, torch.randn(ex.get_parameter(n).shape, generator=g) * 0.1)
    dev = ex.cfg.device
    feeds = {"x": torch.randn(256, 128, generator=g).to(dev)}
    labels = torch.randint(0, 16, (256,), generator=g).to(dev)
    return ex, feeds, labels


def test_linear_activation_gradient_fusion():
    """fc1(GELU) -> fc2: fc2's input-gradient GEMM applies GELU' and fc1's
    bias gradient in its epilogue (gemmp); the result equals the unfused
    backward (colsum_act) parameter by parameter."""
    a, feeds, labels = _mlp_gelu(True)
    b, _, _ = _mlp_gelu(False)
    fc2 = next(s for s in a.steps if s.name == "fc2")
    assert "dact_src" in fc2.ctx.extra
    before = K.STATS["gemmp"]
    for _ in range(3):
        a.train_step(feeds, labels)
        b.train_step(feeds, labels)
    torch.cuda.synchronize()
    assert K.STATS["gemmp"] > before, "fused path not taken"
    for n in a.parameter_names():
        torch.testing.assert_close(a.get_parameter(n), b.get_parameter(n), rtol=2e-2, atol=2e-3)


def test_overlapped_bucket_update_matches_end_of_step_update():
    """Bucket-wise optimizer updates on a side stream during the backward
    pass (ExecConfig.overlap_update) equal the single update at the end,
    eagerly and inside a captured hipGraph."""
    torch.manual_seed(0)
    a, feeds, labels = _model()
    b, _, _ = _model()
    dev = a.executor.cfg.device
    feeds = {k: v.to(dev) for k, v in feeds.items()}
    labels = labels.to(dev)
    a.executor.cfg.overlap_update = True
    b.executor.cfg.overlap_update = False
    assert a.executor._overlap_flats(), "no flat eligible for the overlapped update"
    for _ in range(3):
        a.executor.train_step(feeds, labels)
        b.executor.train_step(feeds, labels)
    torch.cuda.synchronize()
    for n in a.executor.parameter_names():
        torch.testing.assert_close(a.executor.get_parameter(n), b.executor.get_parameter(n), rtol=1e-5, atol=1e-6)
    sa = a.executor.make_graphed_train_step(feeds, labels, warmup=1)
    sb = b.executor.make_graphed_train_step(feeds, labels, warmup=1)
    for _ in range(3):
        sa()
        sb()
    torch.cuda.synchronize()
    for n in a.executor.parameter_names():
        torch.testing.assert_close(a.executor.get_parameter(n), b.executor.get_parameter(n), rtol=1e-5, atol=1e-6)


def test_wgrad_stream_matches_single_stream():
    """Weight-gradient GEMMs on the side stream (ExecConfig.wgrad_stream)
    train like the single-stream backward, eagerly and inside a captured
    hipGraph (residual gradients shared with a dW GEMM's input are not
    accumulated in place)."""
    torch.manual_seed(0)
    a, feeds, labels = _model()
    b, _, _ = _model()
    dev = a.executor.cfg.device
    feeds = {k: v.to(dev) for k, v in feeds.items()}
    labels = labels.to(dev)
    a.executor.cfg.wgrad_stream = True
    b.executor.cfg.wgrad_stream = False
    for _ in range(3):
        a.executor.train_step(feeds, labels)
        b.executor.train_step(feeds, labels)
    torch.cuda.synchronize()
    assert getattr(a.executor, "_wg", None) is not None, "side stream never used"
    assert not a.executor._wg[1], "side stream not joined at the end of the backward pass"
    for n in a.executor.parameter_names():
        torch.testing.assert_close(a.executor.get_parameter(n), b.executor.get_parameter(n), rtol=2e-2, atol=2e-3)
    sa = a.executor.make_graphed_train_step(feeds, labels, warmup=1)
    sb = b.executor.make_graphed_train_step(feeds, labels, warmup=1)
    for _ in range(3):
        sa()
        sb()
    torch.cuda.synchronize()
    for n in a.executor.parameter_names():
        torch.testing.assert_close(a.executor.get_parameter(n), b.executor.get_parameter(n), rtol=2e-2, atol=2e-3)


def test_sync_debug_mode_trains_like_default():
    """ExecConfig.sync_debug (FF_SYNC_DEBUG=1): a device synchronisation after
    every operator, faults attributed to the operator; same numbers."""
    torch.manual_seed(0)
    a, feeds, labels = _model()
    b, _, _ = _model()
    dev = a.executor.cfg.device
    feeds = {k: v.to(dev) for k, v in feeds.items()}
    labels = labels.to(dev)
    a.executor.cfg.sync_debug = True
    for _ in range(2):
        a.executor.train_step(feeds, labels)
        b.executor.train_step(feeds, labels)
    torch.cuda.synchronize()
    for n in a.executor.parameter_names():
        torch.testing.assert_close(a.executor.get_parameter(n), b.executor.get_parameter(n), rtol=1e-5, atol=1e-6)
