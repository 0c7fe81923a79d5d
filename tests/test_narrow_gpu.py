"""Narrow-output Linear kernels (elementwise.hip narrow_*: N <= 8, the DLRM
sigmoid head) and the one-pass MSE loss + metrics kernel, against plain
PyTorch fp32 references of the same ops."""
import pytest
import torch

pytestmark = pytest.mark.gpu

ACTS = {"none": lambda t: t, "relu": torch.relu, "sigmoid": torch.sigmoid,
        "gelu": lambda t: torch.nn.functional.gelu(t, approximate="tanh")}


def _rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12)).item()


@pytest.mark.parametrize("N", [1, 3, 8])
@pytest.mark.parametrize("act", ["none", "sigmoid", "relu", "gelu"])
def test_narrow_linear_matches_fp32(N, act):
    from flexflow_train_amd import kernels as K
    torch.manual_seed(N)
    M, Kd = 1000, 1024
    x = torch.randn(M, Kd, device="cuda").bfloat16()
    w = (torch.randn(Kd, N, device="cuda") * 0.03).bfloat16()
    b = torch.randn(N, device="cuda")
    pre = torch.empty(M, N, device="cuda", dtype=torch.bfloat16) if act != "none" else None
    y = K.narrow_linear_fwd(x, w, bias=b, act=act, pre=pre)
    xf, wf = x.float().requires_grad_(True), w.float().requires_grad_(True)
    bf = b.clone().requires_grad_(True)
    yr = ACTS[act](xf @ wf + bf)
    assert _rel(y, yr) < 5e-3
    dy = torch.randn(M, N, device="cuda").bfloat16()
    yr.backward(dy.float())
    dw = torch.full((Kd, N), 7.0, device="cuda")            # beta = 0 overwrites
    db = torch.ones(N, device="cuda")                        # accumulates
    dx = K.narrow_linear_bwd(x, w, dy, pre=pre, act=act, dw=dw, wbeta=0.0, db=db)
    assert _rel(dx, xf.grad) < 5e-3
    assert _rel(dw, wf.grad) < 5e-3
    # db of a 1-wide head is ONE sum of 1000 random-sign terms, each from the
    # bf16-rounded pre-activation: a cancelling sum, looser bound
    assert _rel(db - 1.0, bf.grad) < 2e-2
    # accumulate forms: dW += , dX +=
    dw2 = dw.clone()
    acc = torch.randn(M, Kd, device="cuda").bfloat16()
    acc0 = acc.float().clone()
    K.narrow_linear_bwd(x, w, dy, pre=pre, act=act, dw=dw2, wbeta=1.0, dx=acc, dx_beta=1.0)
    assert _rel(dw2, 2 * wf.grad) < 5e-3
    # one bf16 rounding of (old + g W^T), computed in fp32
    assert _rel(acc.float(), acc0 + xf.grad) < 5e-3


def test_mse_full_metrics():
    from flexflow_train_amd import kernels as K
    torch.manual_seed(0)
    p = torch.rand(1024, 3, device="cuda").bfloat16()
    y = torch.rand(1024, 3, device="cuda")
    m = torch.zeros(6, device="cuda")
    g = torch.empty_like(p)
    K.mse_full(p, y, g, m, 2.0 / p.numel(), 3, 1024)
    d = p.float() - y
    torch.testing.assert_close(g.float(), (d * 2.0 / p.numel()), rtol=1e-2, atol=1e-5)
    torch.testing.assert_close(m[3], (d * d).sum(), rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(m[4], d.abs().sum(), rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(m[0], (d * d).sum() / 3, rtol=1e-4, atol=1e-4)
    assert m[2].item() == 1024.0 and m[1].item() == 0.0


def test_dlrm_head_runs_native():
    """A sigmoid 1-wide head + MSE on the GPU: the narrow kernels and the
    fused MSE run, torch's sigmoid / mm do not (STATS counters)."""
    from flexflow_train_amd import kernels as K
    from flexflow_train_amd.core import ActiMode, DataType, FFConfig, FFModel, LossType, MetricsType, SGDOptimizer
    m = FFModel(FFConfig())
    x = m.create_tensor([256, 64], DataType.DT_FLOAT, name="x")
    t = m.dense(x, 128, ActiMode.AC_MODE_RELU, name="fc")
    m.dense(t, 1, ActiMode.AC_MODE_SIGMOID, name="head")
    m.compile(optimizer=SGDOptimizer(m, lr=0.1), loss_type=LossType.LOSS_MEAN_SQUARED_ERROR_AVG_REDUCE,
              metrics=[MetricsType.METRICS_MEAN_SQUARED_ERROR])
    ex = m.executor
    before = dict(K.STATS)
    feeds = {"x": torch.randn(256, 64)}
    labels = torch.rand(256, 1)
    for _ in range(3):
        ex.train_step(feeds, labels)
    torch.cuda.synchronize()
    assert K.STATS["narrow_linear"] > before.get("narrow_linear", 0)
    assert K.STATS["mse"] > before.get("mse", 0)
    pm = ex.perf_metrics()
    assert pm.mse_loss > 0


def test_zero_fill_kernel():
    from flexflow_train_amd import kernels as K
    for n, dt in ((1, torch.bfloat16), (1000003, torch.float32), (4096, torch.bfloat16)):
        t = torch.randn(n, device="cuda").to(dt)
        K.zero_(t)
        assert int((t != 0).sum()) == 0
