"""bf16 grouped convolutions on the MFMA implicit-GEMM kernels (conv.hip
group_plan: super-groups of whole groups as block-diagonal dense convs,
blockIdx.z = super-group) against fp64 torch ``F.conv2d(groups=g)`` on the
same bf16-rounded inputs, at the output-rounding level (relative Frobenius
5e-3 for bf16 outputs, 1e-5 for the fp32 weight gradient).

Parity: lib/kernels/src/cuda/ops/conv_2d_kernels.cu:194-196 (group count,
tensor-op math), :279 / :346 / :362; ResNeXt-50 is an AE workload
(scripts/osdi22ae/resnext-50.sh)."""
import pytest
import torch
import torch.nn.functional as F

from flexflow_train_amd import kernels as K

pytestmark = pytest.mark.gpu

DEV = "cuda"

# (N, C, H, W, K, R, S, stride, pad, groups)
CASES = [
    (2, 128, 9, 9, 128, 3, 3, 1, 1, 32),     # ResNeXt-50 32x4d layer 1: 4 channels per group
    (2, 256, 10, 10, 256, 3, 3, 2, 1, 32),   # layer 2 entry: 8 per group, stride 2
    (2, 512, 7, 7, 512, 3, 3, 1, 1, 32),     # 16 per group
    (2, 1024, 5, 5, 1024, 3, 3, 1, 1, 32),   # 32 per group: 2 groups per 64-wide super-group
    (2, 64, 8, 8, 128, 3, 3, 1, 1, 2),       # Cg 32 -> Kg 64
    (2, 256, 6, 6, 256, 3, 3, 1, 1, 2),      # Cg 128: one group per super-group
    (2, 64, 8, 8, 64, 3, 3, 1, 1, 64),       # depthwise
    (1, 96, 7, 9, 48, 1, 3, 1, (0, 1), 4),   # non-square kernel, Cg 24 -> Kg 12 (all 4 groups in one super-group)
]


def _relerr(a, ref):
    a, ref = a.double().cpu(), ref.double().cpu()
    return ((a - ref).norm() / ref.norm().clamp_min(1e-30)).item()


def _nhwc(t):
    return t.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)


def _case(case, seed):
    N, C, H, W, Ko, R, S, st, pd, groups = case
    pd = pd if isinstance(pd, tuple) else (pd, pd)
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(N, C, H, W, generator=g).to(torch.bfloat16)
    w = (torch.randn(Ko, C // groups, R, S, generator=g) / (R * S * C / groups) ** 0.5).to(torch.bfloat16)
    b = (0.1 * torch.randn(Ko, generator=g)).to(torch.bfloat16)
    return x, w, b, (st, st), pd, groups


@pytest.mark.parametrize("case", CASES)
def test_grouped_fwd_stats(case):
    x, w, b, st, pd, groups = _case(case, 0)
    Ko = w.shape[0]
    ref = torch.relu(F.conv2d(x.double(), w.double(), b.double(), stride=st, padding=pd, groups=groups))
    stats = torch.zeros(2 * Ko, device=DEV)
    wp = w.permute(0, 2, 3, 1).contiguous().to(DEV)           # [K][R][S][C/groups]
    n0 = K.STATS["conv2d_grouped_fwd"]
    y, wexp = K.conv2d_grouped_fwd(_nhwc(x.to(DEV)), wp, b.to(DEV), st, pd, groups=groups, act="relu", stats=stats)
    assert K.STATS["conv2d_grouped_fwd"] == n0 + 1
    assert y.shape == ref.shape and y.is_contiguous(memory_format=torch.channels_last)
    assert _relerr(y, ref) < 5e-3
    yd = y.double().cpu()
    assert _relerr(stats[:Ko], yd.sum((0, 2, 3))) < 1e-5
    assert _relerr(stats[Ko:], (yd * yd).sum((0, 2, 3))) < 1e-5


@pytest.mark.parametrize("case", CASES)
def test_grouped_dgrad_wgrad(case):
    x, w, b, st, pd, groups = _case(case, 1)
    Ko, Cg, R, S = w.shape
    xr = x.double().requires_grad_(True)
    wr = w.double().requires_grad_(True)
    yr = F.conv2d(xr, wr, stride=st, padding=pd, groups=groups)
    dy = torch.randn(yr.shape, generator=torch.Generator().manual_seed(7)).to(torch.bfloat16)
    yr.backward(dy.double())
    wp = w.permute(0, 2, 3, 1).contiguous().to(DEV)
    wexp = K.conv2d_grouped_expand(wp, tuple(x.shape), st, pd, groups=groups)
    dyd = _nhwc(dy.to(DEV))
    dx = K.conv2d_grouped_dgrad(dyd, wexp, tuple(wp.shape), tuple(x.shape), st, pd, groups=groups)
    assert _relerr(dx, xr.grad) < 5e-3
    acc = dx.clone(memory_format=torch.channels_last)
    K.conv2d_grouped_dgrad(dyd, wexp, tuple(wp.shape), tuple(x.shape), st, pd, groups=groups, out=acc, beta=1.0)
    assert _relerr(acc, 2 * xr.grad) < 5e-3
    dw = torch.full((Ko * R * S * Cg,), 0.5, device=DEV)
    K.conv2d_grouped_wgrad(_nhwc(x.to(DEV)), dyd, dw, R, S, st, pd, groups=groups)
    dw_ref = wr.grad.permute(0, 2, 3, 1).contiguous()
    assert _relerr(dw.view_as(dw_ref).double().cpu() - 0.5, dw_ref) < 1e-5


def test_grouped_op_path_and_fused_stats():
    """Conv2DOp takes the grouped MFMA path for bf16 (no igemm32), with the
    BatchNorm statistics epilogue and the accumulated input gradient."""
    from flexflow_train_amd.ops import conv as CV
    from flexflow_train_amd.ops.base import OpContext

    x, w, b, st, pd, groups = _case((4, 128, 14, 14, 128, 3, 3, 1, 1, 32), 3)
    Ko, Cg, R, S = w.shape
    ctx = OpContext("CONV2D", {"kernel_h": 3, "kernel_w": 3, "stride_h": 1, "stride_w": 1, "padding_h": 1,
                               "padding_w": 1, "groups": groups}, "g", device=torch.device(DEV),
                    compute_dtype=torch.bfloat16)
    ctx.extra["emit_bn_stats"] = True
    op = CV.Conv2DOp()
    Wl = w.permute(0, 2, 3, 1).contiguous().to(DEV).reshape(Ko, Cg, R, S)   # logical-shaped piece, physical data
    n32 = K.STATS["conv32_fwd"]
    (y,), saved = op.forward(ctx, [_nhwc(x.to(DEV))], [Wl])
    assert saved[0] == "hipg" and K.STATS["conv32_fwd"] == n32
    ref = F.conv2d(x.double(), w.double(), padding=1, groups=groups)
    assert _relerr(y, ref) < 5e-3
    assert _relerr(y._ff_bn_stats[:Ko], y.double().cpu().sum((0, 2, 3))) < 1e-5
    dy = torch.randn(ref.shape, generator=torch.Generator().manual_seed(5)).to(torch.bfloat16)
    base = torch.randn(x.shape, generator=torch.Generator().manual_seed(6)).to(torch.bfloat16)
    ctx.extra["grad_acc"] = [_nhwc(base.to(DEV))]
    dW = torch.zeros(Ko * Cg * R * S, device=DEV)
    (dx,) = op.backward(ctx, saved, [_nhwc(dy.to(DEV))], [dW], [True])
    xr = x.double().requires_grad_(True)
    wr = w.double().requires_grad_(True)
    F.conv2d(xr, wr, padding=1, groups=groups).backward(dy.double())
    assert _relerr(dx, xr.grad + base.double()) < 5e-3
    assert _relerr(dW.view(Ko, R, S, Cg).double().cpu(), wr.grad.permute(0, 2, 3, 1)) < 1e-5
