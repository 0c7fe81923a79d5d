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
