"""GPU numerics of the exact-fp32 MFMA kernels (csrc/kernels/igemm32.hip):
fp32 GEMMs (every transpose, fused bias / activation / pre-activation /
beta) and grouped / fp32 convolutions (forward, data gradient, weight
gradient), each against a float64 PyTorch reference of the same op.

fp32 inputs must agree to 1e-5 relative Frobenius error (the kernel is a
k-ordered fp32 fmaf chain: the expected error is ~1e-7 sqrt(K)); bf16 inputs
(grouped ResNeXt convolutions) are compared with the reference evaluated on
the same bf16-rounded values, so only the fp32 accumulation and the final
bf16 rounding differ (2^-9 relative per element)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

dev = "cuda"


def _k():
    from flexflow_train_amd import kernels as K
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    K.ext()
    return K


def rel(a, b):
    a = a.double().cpu()
    b = b.double().cpu()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


@pytest.mark.parametrize("ta", [False, True])
@pytest.mark.parametrize("tb", [False, True])
@pytest.mark.parametrize("M,N,Kd", [(256, 192, 320), (97, 33, 70), (1000, 8, 1)])
def test_gemm_f32_transposes(ta, tb, M, N, Kd):
    K = _k()
    g = torch.Generator().manual_seed(M + N + Kd)
    A = torch.randn(M, Kd, generator=g, dtype=torch.float64)
    B = torch.randn(Kd, N, generator=g, dtype=torch.float64)
    a = (A.t().contiguous() if ta else A).float().to(dev)
    b = (B.t().contiguous() if tb else B).float().to(dev)
    n0 = K.STATS["gemm_f32"]
    c = K.gemm_f32(a, b, trans_a=ta, trans_b=tb)
    torch.cuda.synchronize()
    assert K.STATS["gemm_f32"] == n0 + 1
    assert rel(c, A @ B) < 1e-5


@pytest.mark.parametrize("act", ["none", "relu", "sigmoid", "tanh", "gelu"])
def test_gemm_f32_epilogue(act):
    K = _k()
    g = torch.Generator().manual_seed(7)
    A = torch.randn(130, 96, generator=g, dtype=torch.float64)
    B = torch.randn(96, 72, generator=g, dtype=torch.float64)
    bias = torch.randn(72, generator=g, dtype=torch.float64)
    C0 = torch.randn(130, 72, generator=g, dtype=torch.float64)
    pre = torch.empty(130, 72, device=dev)
    out = K.gemm_f32(A.float().to(dev), B.float().to(dev), bias=bias.float().to(dev), act=act, pre=pre, alpha=0.5)
    u = 0.5 * (A @ B) + bias
    ref = {"none": lambda t: t, "relu": torch.relu, "sigmoid": torch.sigmoid, "tanh": torch.tanh,
           "gelu": lambda t: F.gelu(t, approximate="tanh")}[act](u)
    assert rel(pre, u) < 1e-5
    assert rel(out, ref) < 1e-5
    # accumulate form: C = AB + beta C (the input-gradient / weight-gradient += of the Linear backward)
    c = C0.float().to(dev)
    K.gemm_f32(A.float().to(dev), B.float().to(dev), out=c, beta=1.0)
    assert rel(c, A @ B + C0) < 1e-5


def _conv_ref(x, w, b, stride, pad, dil, groups):
    return F.conv2d(x, w, b, stride=stride, padding=pad, dilation=dil, groups=groups)


CASES = [
    # N, C, H, W, K, R, S, stride, pad, dil, groups
    (2, 16, 9, 11, 24, 3, 3, (1, 1), (1, 1), (1, 1), 1),
    (2, 12, 10, 10, 20, 3, 3, (2, 2), (1, 1), (1, 1), 1),
    (2, 64, 8, 8, 64, 3, 3, (1, 1), (1, 1), (1, 1), 32),     # ResNeXt: 2 channels per group
    (2, 128, 7, 7, 128, 3, 3, (2, 2), (1, 1), (1, 1), 32),   # 4 channels per group, strided
    (1, 96, 6, 6, 96, 3, 3, (1, 1), (2, 2), (2, 2), 3),      # dilated, 32 per group
    (3, 8, 5, 7, 16, 1, 1, (1, 1), (0, 0), (1, 1), 2),
    (2, 6, 9, 9, 9, 5, 3, (1, 2), (2, 1), (1, 1), 3),         # odd channels per group
]


@pytest.mark.parametrize("case", CASES, ids=[f"c{i}" for i in range(len(CASES))])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_conv32(case, dtype):
    K = _k()
    N, C, H, W, Ko, R, S, stride, pad, dil, groups = case
    g = torch.Generator().manual_seed(hash(case) % 1000)
    x = torch.randn(N, C, H, W, generator=g, dtype=torch.float64)
    w = torch.randn(Ko, C // groups, R, S, generator=g, dtype=torch.float64) * 0.3
    b = torch.randn(Ko, generator=g, dtype=torch.float64)
    if dtype == torch.bfloat16:   # reference on the same rounded values
        x, w, b = (t.to(torch.bfloat16).double() for t in (x, w, b))
    xr = x.requires_grad_(True)
    wr = w.clone().requires_grad_(True)
    y_ref = _conv_ref(xr, wr, b, stride, pad, dil, groups)
    dy = torch.randn(y_ref.shape, generator=g, dtype=torch.float64)
    if dtype == torch.bfloat16:
        dy = dy.to(torch.bfloat16).double()
    y_ref.backward(dy)

    xd = x.detach().to(dtype).to(dev).contiguous(memory_format=torch.channels_last)
    wd = w.detach().permute(0, 2, 3, 1).contiguous().to(dtype).to(dev)   # [K][R][S][C/groups]
    y = K.conv32_fwd(xd, wd, b.to(dtype).to(dev), stride, pad, dil, groups=groups)
    dyd = dy.to(dtype).to(dev).contiguous(memory_format=torch.channels_last)
    dx = K.conv32_dgrad(dyd, wd, tuple(x.shape), stride, pad, dil, groups=groups)
    dw = torch.zeros(wd.numel(), device=dev, dtype=torch.float32)
    K.conv32_wgrad(xd, dyd, dw, R, S, stride, pad, dil, groups=groups)
    torch.cuda.synchronize()
    dw_l = dw.view(Ko, R, S, C // groups).permute(0, 3, 1, 2)
    tol = 1e-5 if dtype == torch.float32 else 5e-3
    assert rel(y, y_ref.detach()) < tol
    assert rel(dx, xr.grad) < tol
    # the weight gradient accumulates in fp32 whatever the input dtype
    assert rel(dw_l, wr.grad) < (1e-5 if dtype == torch.float32 else 1e-5 * 10)


def test_conv32_accumulates():
    """dx += and dw += forms (gradient accumulation into existing buffers)."""
    K = _k()
    g = torch.Generator().manual_seed(3)
    x = torch.randn(2, 64, 6, 6, generator=g)
    w = torch.randn(64, 2, 3, 3, generator=g)
    dy = torch.randn(2, 64, 6, 6, generator=g)
    xd = x.to(dev).contiguous(memory_format=torch.channels_last)
    wd = w.permute(0, 2, 3, 1).contiguous().to(dev)
    dyd = dy.to(dev).contiguous(memory_format=torch.channels_last)
    base = torch.randn(x.shape, generator=g)
    dx = base.to(dev).contiguous(memory_format=torch.channels_last)
    K.conv32_dgrad(dyd, wd, tuple(x.shape), (1, 1), (1, 1), groups=32, out=dx, beta=1.0)
    w0 = torch.randn(wd.numel(), generator=g)
    dw = w0.clone().to(dev)
    K.conv32_wgrad(xd, dyd, dw, 3, 3, (1, 1), (1, 1), groups=32)
    xr = x.double().requires_grad_(True)
    wr = w.double().requires_grad_(True)
    F.conv2d(xr, wr, None, padding=1, groups=32).backward(dy.double())
    assert rel(dx, xr.grad + base.double()) < 1e-5
    assert rel(dw.view(64, 3, 3, 2).permute(0, 3, 1, 2), wr.grad + w0.view(64, 3, 3, 2).permute(0, 3, 1, 2)) < 1e-5
