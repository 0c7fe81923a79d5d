"""An fp32 model trains on the GPU through the native kernels only: every
Linear / BatchMatmul GEMM on the exact-fp32 MFMA kernel and every
convolution (grouped ones included) on the fp32 implicit GEMM
(igemm32.hip) -- torch.mm / torch.matmul / F.conv2d are never called with
GPU tensors -- and one SGD step matches the CPU fp32 executor.

Parity: the reference trains fp32 end to end (linear_kernels.cu:124-131,
conv_2d_kernels.cu:279 with groups, examples/python/native/*)."""
import pytest
import torch
import torch.nn.functional as F

from flexflow_train_amd import kernels as K
from flexflow_train_amd.core import ActiMode, DataType, FFConfig, FFModel, LossType, MetricsType, SGDOptimizer

pytestmark = pytest.mark.gpu


def _net(m):
    x = m.create_tensor([4, 16, 10, 10], DataType.DT_FLOAT, name="img")
    t = m.conv2d(x, 32, 3, 3, 1, 1, 1, 1, ActiMode.AC_MODE_RELU, name="c1")
    t = m.conv2d(t, 32, 3, 3, 2, 2, 1, 1, ActiMode.AC_MODE_RELU, groups=8, name="gconv")   # 4 channels per group
    t = m.conv2d(t, 24, 1, 1, 1, 1, 0, 0, name="pw")
    t = m.dense(m.flat(t, name="flat"), 40, ActiMode.AC_MODE_RELU, name="fc1")
    t = m.dense(t, 6, name="out")
    m.softmax(t, name="sm")
    g = torch.Generator().manual_seed(5)
    return {"img": torch.randn(4, 16, 10, 10, generator=g)}, torch.randint(0, 6, (4,), generator=g)


def _build(device):
    cfg = FFConfig()
    cfg.compute_dtype = "float32"
    if device == "cpu":
        cfg.cpu_only = True
    m = FFModel(cfg)
    feeds, labels = _net(m)
    m.compile(optimizer=SGDOptimizer(m, lr=0.05), loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY,
              metrics=[MetricsType.METRICS_ACCURACY])
    return m, feeds, labels


def test_fp32_model_uses_native_kernels_only(monkeypatch):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    m, feeds, labels = _build("cuda")
    ex = m.executor
    assert ex.cfg.compute_dtype == torch.float32
    g = torch.Generator().manual_seed(0)
    init = {}
    for n in sorted(ex.parameter_names()):
        init[n] = torch.randn(ex.get_parameter(n).shape, generator=g) * 0.2
        ex.set_parameter(n, init[n])

    def refuse(name, fn):
        def wrapped(*args, **kw):
            if any(isinstance(a, torch.Tensor) and a.is_cuda for a in args):
                raise AssertionError(f"{name} called with GPU tensors on the fp32 path")
            return fn(*args, **kw)
        return wrapped

    for name in ("mm", "addmm", "matmul", "bmm"):
        monkeypatch.setattr(torch, name, refuse(f"torch.{name}", getattr(torch, name)))
    monkeypatch.setattr(F, "conv2d", refuse("F.conv2d", F.conv2d))
    monkeypatch.setattr(torch.Tensor, "__matmul__", refuse("Tensor.__matmul__", torch.Tensor.__matmul__))
    n_g, n_c = K.STATS["gemm_f32"], K.STATS["conv32_fwd"]
    dev = ex.cfg.device
    ex.train_step({k: v.to(dev) for k, v in feeds.items()}, labels.to(dev))
    torch.cuda.synchronize()
    monkeypatch.undo()
    assert K.STATS["gemm_f32"] > n_g and K.STATS["conv32_fwd"] >= n_c + 3
    gpu = {n: ex.get_parameter(n).cpu() for n in sorted(ex.parameter_names())}

    # the CPU fp32 executor from the same weights
    from flexflow_train_amd.parallel.comm import DistContext
    from flexflow_train_amd.runtime.executor import ExecConfig, Executor
    from flexflow_train_amd.runtime.optimizer import SGDConfig

    cpu = Executor(m.pcg, DistContext(0, 1, torch.device("cpu")), ExecConfig(compute_dtype=torch.float32),
                   loss_type="sparse_categorical_crossentropy", optimizer=SGDConfig(lr=0.05),
                   valid_classes=m.valid_classes)
    cpu.init_parameters()
    for n, t in init.items():
        cpu.set_parameter(n, t)
    cpu.train_step(feeds, labels)
    for n in gpu:
        torch.testing.assert_close(gpu[n], cpu.get_parameter(n), rtol=1e-4, atol=1e-5, msg=lambda s: f"{n}: {s}")
