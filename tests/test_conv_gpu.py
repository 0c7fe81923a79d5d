"""GPU numerics of the NHWC convolution / BatchNorm / pooling HIP kernels
(csrc/kernels/conv.hip, bnpool.hip) against PyTorch fp32 references of the
same ops, and a CNN model step on the HIP path against the CPU fp32 executor."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from flexflow_train_amd import kernels as K

pytestmark = pytest.mark.gpu

DEV = "cuda"

# (N, C, H, W, K, R, S, stride, pad)
CONV_CASES = [
    (2, 16, 9, 9, 24, 3, 3, 1, 1),
    (2, 16, 9, 9, 24, 3, 3, 2, 1),
    (3, 64, 14, 14, 64, 1, 1, 1, 0),      # BN=64 tile
    (2, 32, 15, 15, 192, 1, 1, 2, 0),     # 128 + 64 N tiles, strided 1x1
    (2, 8, 23, 23, 64, 7, 7, 2, 3),       # stem-like
    (4, 128, 7, 7, 256, 3, 3, 1, 1),
    (1, 40, 5, 6, 16, 3, 2, 1, 0),        # non-square kernel, odd sizes
]


def _rand_nhwc(shape, scale=1.0):
    return (torch.randn(shape, device=DEV) * scale).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)


def _relerr(a, ref):
    """Relative Frobenius error against an fp64 reference (on the CPU)."""
    a, ref = a.double().cpu(), ref.double().cpu()
    return ((a - ref).norm() / ref.norm().clamp_min(1e-30)).item()


@pytest.mark.parametrize("case", CONV_CASES)
def test_conv_fwd_and_stats(case):
    torch.manual_seed(0)
    N, C, H, W, Ko, R, S, st, pd = case
    x = _rand_nhwc((N, C, H, W))
    w = (torch.randn(Ko, R, S, C, device=DEV) * (1.0 / (R * S * C) ** 0.5)).to(torch.bfloat16).contiguous()
    b = (torch.randn(Ko, device=DEV) * 0.1).to(torch.bfloat16)
    stats = torch.zeros(2 * Ko, device=DEV)
    y = K.conv2d_fwd(x, w, b, (st, st), (pd, pd), act="relu", stats=stats)
    # fp64 reference on the same bf16 inputs: the bound is the bf16 output
    # rounding (relative RMS ~1.1e-3), so a 1 % error in one tile phase fails
    ref = torch.relu(F.conv2d(x.double().cpu(), w.double().cpu().permute(0, 3, 1, 2), b.double().cpu(), stride=st,
                              padding=pd))
    assert y.shape == ref.shape and y.is_contiguous(memory_format=torch.channels_last)
    assert _relerr(y, ref) < 5e-3
    yd = y.double().cpu()
    assert _relerr(stats[:Ko], yd.sum((0, 2, 3))) < 1e-5
    assert _relerr(stats[Ko:], (yd * yd).sum((0, 2, 3))) < 1e-5


@pytest.mark.parametrize("case", CONV_CASES)
def test_conv_dgrad_wgrad(case):
    torch.manual_seed(1)
    N, C, H, W, Ko, R, S, st, pd = case
    x = _rand_nhwc((N, C, H, W))
    w = (torch.randn(Ko, R, S, C, device=DEV) * (1.0 / (R * S * C) ** 0.5)).to(torch.bfloat16).contiguous()
    xr = x.double().cpu().requires_grad_(True)
    wr = w.double().cpu().permute(0, 3, 1, 2).contiguous().requires_grad_(True)
    yr = F.conv2d(xr, wr, stride=st, padding=pd)
    dy = _rand_nhwc(yr.shape)
    yr.backward(dy.double().cpu())
    dx = K.conv2d_dgrad(dy, w, tuple(x.shape), (st, st), (pd, pd))
    assert _relerr(dx, xr.grad) < 5e-3
    # accumulate form
    acc = dx.clone(memory_format=torch.channels_last)
    K.conv2d_dgrad(dy, w, tuple(x.shape), (st, st), (pd, pd), out=acc, beta=1.0)
    assert _relerr(acc, 2 * xr.grad) < 5e-3
    dw_ref = wr.grad.permute(0, 2, 3, 1).contiguous()  # -> [K, R, S, C]
    for splits in (0, 1, 3, 8, 64):   # the tuned degrees (ops/conv._wgrad), 64: two-pass slab reduce
        dw = torch.full((Ko * R * S * C,), 0.5, device=DEV)
        K.conv2d_wgrad(x, dy, dw, R, S, (st, st), (pd, pd), splits=splits)
        assert _relerr(dw.view_as(dw_ref).double().cpu() - 0.5, dw_ref) < 1e-5


@pytest.mark.parametrize("C,relu,residual", [(64, True, False), (24, False, False), (256, True, True), (8, True, False)])
def test_batchnorm_fwd_bwd(C, relu, residual):
    torch.manual_seed(2)
    N, H, W = 4, 7, 9
    x = _rand_nhwc((N, C, H, W), 2.0) + 0.5
    x = x.contiguous(memory_format=torch.channels_last)
    res = _rand_nhwc((N, C, H, W)) if residual else None
    g = (1 + 0.1 * torch.randn(C, device=DEV)).to(torch.bfloat16)
    b = (0.1 * torch.randn(C, device=DEV)).to(torch.bfloat16)
    stats = torch.zeros(2 * C, device=DEV)
    K.bn_stats(x, stats)
    rm, rv = torch.zeros(C, device=DEV), torch.ones(C, device=DEV)
    scale, shift, mean, rstd = K.bn_finalize(stats, g, b, x.numel() // C, 1e-5, 0.1, rm, rv)
    y = K.bn_apply(x, scale, shift, relu, residual=res)

    xr = x.float().requires_grad_(True)
    gr = g.float().requires_grad_(True)
    br = b.float().requires_grad_(True)
    rr = res.float().requires_grad_(True) if residual else None
    rm2, rv2 = torch.zeros(C, device=DEV), torch.ones(C, device=DEV)
    yr = F.batch_norm(xr, rm2, rv2, gr, br, training=True, momentum=0.1, eps=1e-5)
    if residual:
        yr = yr + rr
    if relu:
        yr = torch.relu(yr)
    torch.testing.assert_close(y.float(), yr.detach(), rtol=2e-2, atol=3e-2)
    torch.testing.assert_close(rm, rm2, rtol=1e-3, atol=1e-4)
    torch.testing.assert_close(rv, rv2, rtol=1e-3, atol=1e-4)

    dy = _rand_nhwc(yr.shape)
    yr.backward(dy.float())
    dg = torch.zeros(C, device=DEV)
    db = torch.zeros(C, device=DEV)
    dx, dres = K.bn_bwd(dy, x, y, mean, rstd, g, relu, dgamma=dg, dbeta=db, want_masked=residual)
    torch.testing.assert_close(dx.float(), xr.grad, rtol=3e-2, atol=5e-2)
    torch.testing.assert_close(dg, gr.grad, rtol=2e-2, atol=0.5)
    torch.testing.assert_close(db, br.grad, rtol=2e-2, atol=0.5)
    if residual:
        torch.testing.assert_close(dres.float(), rr.grad, rtol=1e-2, atol=1e-2)
    if relu and not residual:
        # ReLU mask recomputed from x with the forward's scale / shift: same result, y unread
        ss = torch.stack([scale, shift]).reshape(-1)
        dg2, db2 = torch.zeros(C, device=DEV), torch.zeros(C, device=DEV)
        dx2, _ = K.bn_bwd(dy, x, None, mean, rstd, g, True, dgamma=dg2, dbeta=db2, scale_shift=ss)
        torch.testing.assert_close(dx2.float(), dx.float(), rtol=1e-2, atol=1e-2)
        torch.testing.assert_close(dg2, dg, rtol=1e-3, atol=1e-2)
        torch.testing.assert_close(db2, db, rtol=1e-3, atol=1e-2)


@pytest.mark.parametrize("C,Ko,R,relu", [(64, 64, 3, True), (128, 256, 1, True), (200, 72, 3, False),
                                          (2048, 512, 1, True)])
def test_dgrad_bn_sums(C, Ko, R, relu):
    """A BN(+ReLU) -> conv pair: the dgrad epilogue's BN backward sums
    (conv.hip, ConvBnBwd) give the same BN backward as bn_bwd's own
    reduction pass."""
    torch.manual_seed(4)
    N, H, W = 3, 9, 11
    xb = _rand_nhwc((N, C, H, W), 2.0) + 0.3
    g = (1 + 0.1 * torch.randn(C, device=DEV)).to(torch.bfloat16)
    b = (0.1 * torch.randn(C, device=DEV)).to(torch.bfloat16)
    stats = torch.zeros(2 * C, device=DEV)
    K.bn_stats(xb, stats)
    scale, shift, mean, rstd = K.bn_finalize(stats, g, b, xb.numel() // C, 1e-5, 0.0, None, None)
    ss = torch.as_strided(scale, (2 * C,), (1,)) if relu else None
    w = (torch.randn(Ko, R, R, C, device=DEV) / (R * R * C) ** 0.5).to(torch.bfloat16).contiguous()
    pad = (R // 2, R // 2)
    dyc = _rand_nhwc((N, Ko, H, W))
    n0 = K.STATS["conv2d_dgrad_bn"]
    dx = K.conv2d_dgrad(dyc, w, tuple(xb.shape), (1, 1), pad, bn=(xb, mean, rstd, ss))
    assert K.STATS["conv2d_dgrad_bn"] == n0 + 1
    torch.testing.assert_close(dx.float(), K.conv2d_dgrad(dyc, w, tuple(xb.shape), (1, 1), pad).float(),
                               rtol=0, atol=0)
    sums, src = dx._ff_bn_sums
    assert src is xb
    # fp32 reference of the sums from the stored gradient
    xf = xb.float()
    gm = dx.float() * ((xf * scale.view(1, -1, 1, 1) + shift.view(1, -1, 1, 1)) > 0).float() if relu else dx.float()
    xhat = (xf - mean.view(1, -1, 1, 1)) * rstd.view(1, -1, 1, 1)
    torch.testing.assert_close(sums[:C], gm.sum((0, 2, 3)), rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(sums[C:], (gm * xhat).sum((0, 2, 3)), rtol=1e-4, atol=1e-3)
    outs = []
    for pre in (None, sums):
        dg, db = torch.zeros(C, device=DEV), torch.zeros(C, device=DEV)
        d, _ = K.bn_bwd(dx, xb, None, mean, rstd, g, relu, dgamma=dg, dbeta=db, scale_shift=ss, pre_sums=pre)
        outs.append((d.float(), dg, db))
    torch.testing.assert_close(outs[1][0], outs[0][0], rtol=1e-2, atol=1e-2)
    torch.testing.assert_close(outs[1][1], outs[0][1], rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(outs[1][2], outs[0][2], rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("k,s,p,avg", [((3, 3), (2, 2), (1, 1), False), ((2, 2), (2, 2), (0, 0), False),
                                       ((3, 3), (1, 1), (1, 1), True), ((7, 7), (1, 1), (0, 0), True),
                                       ((3, 3), (2, 2), (0, 0), True)])
def test_pool2d(k, s, p, avg):
    torch.manual_seed(3)
    x = _rand_nhwc((2, 24, 14, 14))
    y, arg = K.pool2d_fwd(x, k, s, p, avg)
    xr = x.float().cpu().contiguous().requires_grad_(True)  # fp32 CPU reference
    yr = F.avg_pool2d(xr, k, s, p, count_include_pad=False) if avg else F.max_pool2d(xr, k, s, p)
    torch.testing.assert_close(y.float().cpu(), yr.detach(), rtol=1e-2, atol=1e-2)
    dy = _rand_nhwc(yr.shape)
    yr.backward(dy.float().cpu())
    dx = K.pool2d_bwd(dy, arg, tuple(x.shape), k, s, p, avg)
    torch.testing.assert_close(dx.float().cpu(), xr.grad, rtol=2e-2, atol=2e-2)


def test_resnet_gpu_step_matches_cpu_fp32():
    """Tiny ResNet through the executor: the HIP conv/BN/pool path (with the
    conv->BN statistics and BN+add+ReLU fusions) against the CPU fp32 path."""
    from flexflow_train_amd import models as Z
    from flexflow_train_amd.core import FFConfig, FFModel, LossType, MetricsType, SGDOptimizer
    from flexflow_train_amd.parallel.comm import DistContext
    from flexflow_train_amd.runtime.executor import ExecConfig, Executor
    from flexflow_train_amd.runtime.optimizer import SGDConfig

    m = FFModel(FFConfig())
    inputs, out, mcfg = Z.build("resnet50", m, batch_size=32, image_size=32, num_classes=16)
    m.compile(optimizer=SGDOptimizer(m, lr=0.01), loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY,
              metrics=[MetricsType.METRICS_SPARSE_CATEGORICAL_CROSSENTROPY])
    ex = m.executor
    feeds, labels = Z.synthetic("resnet50", mcfg, inputs, np.random.default_rng(0))
    feeds = {k: torch.as_tensor(v) for k, v in feeds.items()}
    labels = torch.as_tensor(labels)
    assert any(s.ctx is not None and s.ctx.extra.get("residual_relu") for s in ex.steps)
    params = {n: ex.get_parameter(n).cpu() for n in ex.parameter_names()}
    before = dict(K.STATS)
    ex.zero_metrics()
    ex.forward({k: v.to(ex.cfg.device) for k, v in feeds.items()})
    ex.compute_loss(labels.to(ex.cfg.device))
    gpu_loss = ex.perf_metrics().loss
    gpu_env = {k: v.detach().float().cpu() for k, v in ex._env.items() if torch.is_tensor(v) and v.is_floating_point()}
    for name in ("conv2d_fwd", "bn_apply", "pool2d_fwd"):
        assert K.STATS[name] > before.get(name, 0), f"{name} did not run on the HIP path"

    cpu = Executor(m.pcg, DistContext(0, 1, torch.device("cpu")), ExecConfig(compute_dtype=torch.float32),
                   loss_type="sparse_categorical_crossentropy", optimizer=SGDConfig(),
                   valid_classes=m.valid_classes)
    cpu.init_parameters()
    for n, t in params.items():
        cpu.set_parameter(n, t)
    cpu.zero_metrics()
    cpu.forward(feeds)
    cpu.compute_loss(labels)
    ref = cpu.perf_metrics().loss
    # layer by layer through the first stage (before bf16 rounding flips get
    # amplified): every fused conv / BN(+add+ReLU) / pool output matches fp32
    checked = 0
    for s in ex.steps[:24]:
        for o in s.outputs:
            if o in gpu_env and torch.is_tensor(cpu._env.get(o)):
                a, b = gpu_env[o], cpu._env[o].float()
                assert (a - b).abs().max().item() < 3e-2 * b.abs().max().item() + 1e-2, s.name
                checked += 1
    assert checked >= 12
    # the loss after 53 batch-statistics layers: a random-init ResNet amplifies
    # single-ulp bf16 differences ~30x (GPU run-to-run spread from atomic
    # summation order alone is ~5%), so only a loose end-to-end bound
    assert abs(ref - gpu_loss) < 0.12 * abs(ref)

    # a full GPU training step runs the backward kernels and keeps the loss finite
    before = dict(K.STATS)
    for _ in range(3):
        ex.train_step({k: v.to(ex.cfg.device) for k, v in feeds.items()}, labels.to(ex.cfg.device))
    torch.cuda.synchronize()
    for name in ("conv2d_dgrad", "conv2d_wgrad", "bn_bwd", "pool2d_bwd"):
        assert K.STATS[name] > before.get(name, 0), f"{name} did not run on the HIP path"
    assert np.isfinite(ex.perf_metrics().loss)


@pytest.mark.parametrize("mode", ["native", "gemm"])
@pytest.mark.parametrize("C,Ko,acc,st", [(64, 256, False, 1), (256, 64, True, 1), (64, 128, False, 2),
                                         (128, 64, True, 2)])
def test_pointwise_conv_paths(mode, C, Ko, acc, st):
    """1x1 convolutions: the implicit-GEMM kernels and the hand-written GEMM
    path (ops/conv.py picks per shape at stride 1) both match fp32 — forward with the
    BN statistics, dgrad (fresh or accumulated) and the accumulated wgrad."""
    from flexflow_train_amd.ops import conv as CV
    from flexflow_train_amd.ops.base import OpContext

    old = CV._MODE
    CV._MODE, CV._CHOICE = mode, {}
    try:
        N, H = 4, 14
        x = _rand_nhwc((N, C, H, H))
        W = (torch.randn(Ko, 1, 1, C, device="cuda") * 0.1).to(torch.bfloat16)   # physical [K, R, S, C]
        ctx = OpContext("CONV2D", {"kernel_h": 1, "kernel_w": 1, "stride_h": st, "stride_w": st}, "c",
                        device=torch.device("cuda"),
                        compute_dtype=torch.bfloat16)
        ctx.extra["emit_bn_stats"] = True
        op = CV.Conv2DOp()
        Wl = W.view(Ko, 1, 1, C).reshape(Ko, C, 1, 1)  # logical-shaped piece over the physical data
        (y,), saved = op.forward(ctx, [x], [Wl])
        ref = F.conv2d(x.float(), W.float().permute(0, 3, 1, 2), stride=st)
        torch.testing.assert_close(y.float(), ref, rtol=2e-2, atol=2e-2)
        sts = y._ff_bn_stats
        torch.testing.assert_close(sts[:Ko], y.float().sum((0, 2, 3)), rtol=1e-3, atol=1e-1)
        dy = _rand_nhwc(tuple(y.shape))
        dW = torch.full((Ko * C,), 0.5, device="cuda")
        if acc:
            base = _rand_nhwc(tuple(x.shape))
            ctx.extra["grad_acc"] = [base.clone()]
        (dx,) = op.backward(ctx, saved, [dy], [dW], [True])
        xr = x.float().requires_grad_(True)
        wr = W.float().permute(0, 3, 1, 2).contiguous().requires_grad_(True)
        F.conv2d(xr, wr, stride=st).backward(dy.float())
        want_dx = xr.grad + (base.float() if acc else 0)
        torch.testing.assert_close(dx.float(), want_dx, rtol=2e-2, atol=5e-2)
        torch.testing.assert_close(dW.view(Ko, C), wr.grad.view(Ko, C) + 0.5, rtol=1e-2, atol=5e-2)
        # strided 1x1 convolutions always run the implicit-GEMM kernels (no
        # gather copy): only unit-stride ones have a per-shape choice
        assert set(CV._CHOICE.values()) == ({mode} if st == 1 else set())
    finally:
        CV._MODE, CV._CHOICE = old, {}


@pytest.mark.parametrize("layout", ["nchw", "nhwc"])
@pytest.mark.parametrize("C,Cp", [(3, 8), (5, 16), (8, 8)])
def test_pad_channels_nhwc(layout, C, Cp):
    """One-pass channel padding (conv.hip pad_channels_kernel) from either
    layout into a channels_last tensor with zero pad channels."""
    x = torch.randn(3, C, 17, 11, device=DEV).to(torch.bfloat16)
    if layout == "nhwc":
        x = x.contiguous(memory_format=torch.channels_last)
    y = K.pad_channels_nhwc(x, Cp)
    assert y.shape == (3, Cp, 17, 11) and y.is_contiguous(memory_format=torch.channels_last)
    assert torch.equal(y[:, :C], x)
    assert not y[:, C:].any()
