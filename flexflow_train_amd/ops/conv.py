"""CONV2D and POOL2D operators.

Parity: lib/kernels/src/cuda/ops/conv_2d_kernels.cu (cuDNN conv with
autotuned algorithms, fused bias + activation, :8-391) and
pool_2d_kernels.cu (:103 forward, :123 backward).  Channel parallelism
follows op-attrs conv_2d.cc: an input-channel shard produces partial sums
(bias on replica 0 only), an output-channel shard is expressed by the weight
piece.

MI355X path (csrc/kernels/conv.hip, bnpool.hip): activations stay NHWC
(torch channels_last, logical shape NCHW) end to end; the weight is stored
physically as [K][R][S][C] (``to_physical``) so the implicit-GEMM kernels
read both operands in 16-byte channel chunks.  Forward fuses bias +
activation and, when the executor pairs the conv with a following
BatchNorm (``emit_bn_stats``), the per-channel statistics that BN needs.
Backward = dgrad implicit GEMM + split-K wgrad accumulating in fp32 straight
into the flat gradient buffer.  Inputs with fewer than 8 channels (the RGB
stem) are zero-padded to 8.  bf16 grouped convolutions (ResNeXt) run on the
same MFMA kernels as block-diagonal super-group convs (conv.hip
group_plan); fp32 models on igemm32.hip; CPU tensors through PyTorch (the
weight is viewed back to OIHW).
"""
from __future__ import annotations

import os

import torch
import torch.nn.functional as F

from .. import kernels as K
from . import gemm as G
from .base import OpImpl, acc_grad, register

_ACTS = {"none": lambda t: t, "relu": torch.relu, "sigmoid": torch.sigmoid, "tanh": torch.tanh,
         "gelu": lambda t: F.gelu(t, approximate="tanh")}

# FF_CONV_BN_BWD=1: a BatchNorm(+ReLU) feeding a stride-1 convolution takes its
# backward sums from that conv's dgrad epilogue (conv.hip ConvBnBwd) instead of
# its own reduction pass.  Off by default: on ResNet-50 the epilogue's extra
# BN-input read and per-tile partial rows cost the dgrad kernels more than the
# skipped bn_reduce passes save (+3.2 / -2.9 ms per 5 steps,
# profiles/r5/ab_conv_bn_bwd_r5.txt)
_CONV_BN_BWD = os.environ.get("FF_CONV_BN_BWD", "0") == "1"


def _geom(ctx):
    # an H-sharded input (attribute parallelism) arrives with its halo rows
    # and border padding attached (parallel/halo.py): no H padding here
    ph = 0 if ctx.extra.get("halo") is not None else int(ctx.a("padding_h", 0))
    return ((int(ctx.a("stride_h", 1)), int(ctx.a("stride_w", 1))),
            (ph, int(ctx.a("padding_w", 0))),
            int(ctx.a("groups", 1)), ctx.a("activation", "none"))


_CHOICE = {}


def _pick(key, cands):
    """Per-shape choice between the implicit-GEMM kernels and a library GEMM
    (1x1 stride-1 convolutions are plain GEMMs over NHWC pixels): each
    candidate runs once untimed, then the faster of two timed repeats wins —
    outside graph capture; under capture the native kernel is used."""
    c = _CHOICE.get(key)
    if c is None:
        if len(cands) == 1 or torch.cuda.is_current_stream_capturing() or _MODE != "auto":
            c = "gemm" if (_MODE == "gemm" and "gemm" in cands) else "native"
        else:
            # eager clock (these convolutions run for hundreds of microseconds);
            # candidates interleaved over three passes, best of each kept, so a
            # clock or power transient during one candidate's turn does not
            # decide the pick (one-shot picks flipped run to run: 7 wgrads per
            # ResNet-50 step moved between the two paths, profiles/r5/g35_*)
            from .gemm import _time
            times = {name: float("inf") for name in cands}
            for _ in range(3):
                for name, fn in cands.items():
                    times[name] = min(times[name], _time(fn, iters=3, rounds=1))
            c = min(times, key=times.get)
        _CHOICE[key] = c
    return c


_MODE = os.environ.get("FF_CONV1X1", "auto")   # auto | native | gemm
_WGRAD_SPLITS: dict = {}
# opt-in: on ResNet-50 (512 / GPU) the tuned degrees matched the heuristic
# (9714-9729 vs 9706-9709 img/s, profiles/r6/g44_wgrad_splits.txt)
_WGRAD_TUNE = os.environ.get("FF_CONV_WGRAD_TUNE", "0") == "1"


def _wgrad(xin, dy, dw, R, S, stride, pad):
    """Native weight gradient with its split-K degree picked per shape: the
    kernel's heuristic (~2048 workgroups, >= 8 K-tiles per split) against
    explicit degrees, timed once outside graph capture on a scratch buffer
    (candidates interleaved over two passes, best of each); under capture an
    untuned shape keeps the heuristic."""
    key = (tuple(xin.shape), int(dy.shape[1]), R, S, tuple(stride), tuple(pad))
    sp = _WGRAD_SPLITS.get(key)
    if sp is None:
        sp = 0
        if _WGRAD_TUNE and not torch.cuda.is_current_stream_capturing():
            from .gemm import _time
            N, _, P, Q = dy.shape
            nk = (N * P * Q + 63) // 64
            wbytes = dw.numel() * 4
            cands = [0] + [c for c in (1, 2, 4, 8, 16, 32, 64) if nk // c >= 4 and c * wbytes <= (512 << 20)]
            tmp = torch.zeros_like(dw)
            times = {c: float("inf") for c in cands}
            for _ in range(2):
                for c in cands:
                    times[c] = min(times[c], _time(lambda c_=c: K.conv2d_wgrad(xin, dy, tmp, R, S, stride, pad,
                                                                             splits=c_), iters=3, rounds=1))
            sp = min(times, key=times.get)
            del tmp
        _WGRAD_SPLITS[key] = sp
    K.conv2d_wgrad(xin, dy, dw, R, S, stride, pad, splits=sp)


def _pointwise(R, S, stride, pad, groups) -> bool:
    """1x1, unit-stride, unpadded, ungrouped: a GEMM over the NHWC pixels
    (views, no copies).  Strided 1x1 convolutions stay on the implicit-GEMM
    kernels, which read the sampled pixels in place instead of gathering them
    with a torch copy (and scattering dgrad into a zeroed buffer)."""
    return R == 1 and S == 1 and tuple(pad) == (0, 0) and groups == 1 and tuple(stride) == (1, 1)


def _sub(x: torch.Tensor, stride) -> torch.Tensor:
    """The pixels a strided 1x1 convolution reads, packed (channels_last)."""
    if tuple(stride) == (1, 1):
        return x
    return x[:, :, ::stride[0], ::stride[1]].contiguous(memory_format=torch.channels_last)


def _rows(t: torch.Tensor) -> torch.Tensor:
    """channels_last [N, C, H, W] -> its [N*H*W, C] row-major view (no copy)."""
    return t.permute(0, 2, 3, 1).reshape(-1, t.shape[1])


def _oihw(W: torch.Tensor) -> torch.Tensor:
    """Logical-shaped [K, C, R, S] piece holding physical [K, R, S, C] data -> OIHW view."""
    Kc, C, R, S = W.shape
    return W.reshape(Kc, R, S, C).permute(0, 3, 1, 2)


@register("CONV2D")
class Conv2DOp(OpImpl):
    def to_physical(self, attrs, index, piece):
        if index != 0:
            return piece
        return piece.permute(0, 2, 3, 1).contiguous()

    def to_logical(self, attrs, index, piece):
        if index != 0:
            return piece
        return _oihw(piece).contiguous()

    @staticmethod
    def _native(x, W, groups, act):
        return (x.is_cuda and x.dtype == torch.bfloat16 and groups == 1 and W.shape[0] % 8 == 0
                and (x.shape[1] % 8 == 0 or x.shape[1] < 8) and act in ("none", "relu", "sigmoid", "tanh")
                and K.use_hip(x))

    @staticmethod
    def _native_grouped(x, W, groups, act):
        """bf16 grouped convolutions (ResNeXt) on the MFMA implicit-GEMM
        kernels: super-groups of whole groups whose channel counts are
        multiples of 8 (conv.hip group_plan)."""
        if not (groups > 1 and x.is_cuda and x.dtype == torch.bfloat16 and act in ("none", "relu", "sigmoid", "tanh")
                and K.use_hip(x)):
            return False
        C, Kc = x.shape[1], W.shape[0]
        if C % groups or Kc % groups:
            return False
        cg, kg = C // groups, Kc // groups
        return any(groups % g == 0 and (g * cg) % 8 == 0 and (g * kg) % 8 == 0 for g in range(1, groups + 1))

    @staticmethod
    def _native32(x, act):
        """fp32 models and grouped convolutions (ResNeXt): the exact-fp32 MFMA
        implicit GEMM (igemm32.hip), any channel count per group."""
        return (x.is_cuda and x.dtype in (torch.float32, torch.bfloat16)
                and act in ("none", "relu", "sigmoid", "tanh") and K.use_hip(x))

    def forward(self, ctx, inputs, weights):
        x = inputs[0]
        halo = ctx.extra.get("halo")
        if halo is not None:
            x = halo.extend(x)
        W = weights[0]
        b = weights[1] if len(weights) > 1 and ctx.sum_index == 0 else None
        stride, pad, groups, act = _geom(ctx)
        Kc, C, R, S = W.shape
        if self._native(x, W, groups, act):
            wp = W.reshape(Kc, R, S, C)
            if wp.dtype != torch.bfloat16:
                wp = wp.to(torch.bfloat16)
            if C % 8:  # RGB stem: zero-pad channels to a multiple of 8 (input and weight), one pass each
                Cp = (C + 7) // 8 * 8
                xin = K.pad_channels_nhwc(x, Cp)
                wp = K.pad_channels_nhwc(wp.permute(0, 3, 1, 2), Cp).permute(0, 2, 3, 1)
            else:
                xin = K.nhwc(x)
            stats = None
            if ctx.extra.get("emit_bn_stats"):
                stats = torch.empty(2 * Kc, device=x.device, dtype=torch.float32)
            bias = None if b is None else b.to(torch.bfloat16).contiguous()
            if _pointwise(R, S, stride, pad, groups) and C % 8 == 0:
                def via_gemm(st=stats):
                    xs = _sub(xin, stride)
                    # hand-written GEMMs only (no library kernel for convolutions)
                    y2 = G.matmul(_rows(xs), wp.view(Kc, C), trans_b=True, bias=bias, act=act, native_only=True)
                    yv = y2.view(xs.shape[0], xs.shape[2], xs.shape[3], Kc).permute(0, 3, 1, 2)
                    if st is not None:
                        K.bn_stats(yv, st, overwrite=True)
                    return yv
                key = ("fwd", tuple(xin.shape), Kc, tuple(stride), act, bias is not None, stats is not None)
                scratch = None if stats is None else torch.empty_like(stats)
                choice = _pick(key, {"native": lambda: K.conv2d_fwd(xin, wp, bias, stride, pad, act=act,
                                                                   stats=scratch),
                                     "gemm": lambda: via_gemm(scratch)})
                y = via_gemm() if choice == "gemm" else K.conv2d_fwd(xin, wp, bias, stride, pad, act=act, stats=stats)
            else:
                y = K.conv2d_fwd(xin, wp, bias, stride, pad, act=act, stats=stats)
            if stats is not None:
                y._ff_bn_stats = stats
            bnsrc = None
            if (_CONV_BN_BWD and ctx.training and ctx.extra.get("emit_bn_bwd_sums") and halo is None
                    and tuple(stride) == (1, 1) and C % 8 == 0):
                bnsrc = getattr(x, "_ff_bn_bwd", None)   # set by the producing BatchNorm
            return [y], ("hip", xin, wp, y if act != "none" else None, tuple(x.shape), bnsrc)
        if self._native_grouped(x, W, groups, act):
            wp = W.reshape(Kc, R, S, C)   # physical [K][R][S][C/groups]
            wp = (wp if wp.dtype == torch.bfloat16 else wp.to(torch.bfloat16)).contiguous()
            xin = K.nhwc(x)
            stats = None
            if ctx.extra.get("emit_bn_stats"):
                stats = torch.empty(2 * Kc, device=x.device, dtype=torch.float32)
            bias = None if b is None else b.to(torch.bfloat16).contiguous()
            y, wexp = K.conv2d_grouped_fwd(xin, wp, bias, stride, pad, groups=groups, act=act, stats=stats)
            if stats is not None:
                y._ff_bn_stats = stats
            return [y], ("hipg", xin, wexp, y if act != "none" else None, tuple(x.shape), groups, tuple(wp.shape))
        if self._native32(x, act):
            wp = W.reshape(Kc, R, S, C)   # physical [K][R][S][C/groups]
            if wp.dtype != x.dtype:
                wp = wp.to(x.dtype)
            wp = wp.contiguous()
            xin = x.contiguous(memory_format=torch.channels_last)
            bias = None if b is None else b.to(x.dtype).contiguous()
            y = K.conv32_fwd(xin, wp, bias, stride, pad, groups=groups, act=act)
            return [y], ("hip32", xin, wp, y if act != "none" else None, tuple(x.shape), groups)
        # library path (CPU): the autograd graph recorded here is replayed in
        # backward — no forward recomputation
        xi = x.detach().requires_grad_(ctx.training and x.is_floating_point())
        Wr = W.detach().requires_grad_(ctx.training)
        with torch.enable_grad():
            xw = xi.contiguous(memory_format=torch.channels_last) if xi.is_cuda else xi
            u = F.conv2d(xw, _oihw(Wr).to(x.dtype), None, stride=stride, padding=pad, groups=groups)
            if ctx.training:
                u.retain_grad()
            y = _ACTS[act](u + b.to(u.dtype).view(1, -1, 1, 1) if b is not None else u)
        return [y.detach()], ("torch", xi, Wr, u, y)

    def backward(self, ctx, saved, grad_outputs, weight_grads, need_input_grad):
        halo = ctx.extra.get("halo")
        gx = self._backward(ctx, saved, grad_outputs, weight_grads, need_input_grad)
        if halo is not None and need_input_grad[0]:
            # every band takes part in the halo return, with or without a gradient
            return [halo.fold(gx[0])]
        return gx

    def _backward(self, ctx, saved, grad_outputs, weight_grads, need_input_grad):
        stride, pad, groups, act = _geom(ctx)
        if saved[0] == "torch":
            _, xi, Wr, u, y = saved
            torch.autograd.backward([y], [grad_outputs[0].to(y.dtype)])
            if weight_grads[0] is not None and Wr.grad is not None:
                acc_grad(weight_grads[0], Wr.grad)
            if len(weight_grads) > 1 and weight_grads[1] is not None:
                # every partial-sum replica computes the (identical) bias gradient
                acc_grad(weight_grads[1], u.grad.float().sum((0, 2, 3)))
            return [xi.grad if (xi.requires_grad and need_input_grad[0]) else None]

        if saved[0] == "hip32":
            return self._backward32(ctx, saved, grad_outputs, weight_grads, need_input_grad, stride, pad, act)
        if saved[0] == "hipg":
            return self._backward_grouped(ctx, saved, grad_outputs, weight_grads, need_input_grad, stride, pad, act)
        _, xin, wp, y, xshape, bnsrc = saved
        Kc, R, S, Cp = wp.shape
        dy = K.nhwc(grad_outputs[0].to(torch.bfloat16))
        if act != "none":
            if act == "relu":
                dy = torch.where(y > 0, dy, torch.zeros((), device=dy.device, dtype=dy.dtype))
            else:
                yf = y.float().detach()
                if act == "sigmoid":
                    d = yf * (1 - yf)
                elif act == "tanh":
                    d = 1 - yf * yf
                else:
                    raise NotImplementedError("conv2d: gelu backward needs the pre-activation")
                dy = (dy.float() * d).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        if len(weight_grads) > 1 and weight_grads[1] is not None:
            d2 = dy.permute(0, 2, 3, 1).reshape(-1, Kc)  # channels_last -> [pixels, K] view
            K.colsum_act(d2, None, "none", weight_grads[1], write_dx=False)
        dW = weight_grads[0]
        if dW is not None:
            if Cp == xshape[1] and _pointwise(R, S, stride, pad, 1):
                key = ("wgrad", tuple(xin.shape), Kc, tuple(stride))
                if key not in _CHOICE:
                    tmp = torch.zeros_like(dW.view(-1))
                    _pick(key, {"native": lambda: _wgrad(xin, dy, tmp, R, S, stride, pad),
                                "gemm": lambda: G.matmul(_rows(dy), _rows(_sub(xin, stride)), trans_a=True,
                                                         out=tmp.view(Kc, Cp), beta=1.0, native_only=True)})
                if _CHOICE[key] == "gemm":
                    G.matmul(_rows(dy), _rows(_sub(xin, stride)), trans_a=True, out=dW.view(Kc, Cp), beta=1.0,
                             native_only=True)
                else:
                    _wgrad(xin, dy, dW.view(-1), R, S, stride, pad)
            elif Cp == xshape[1]:
                _wgrad(xin, dy, dW.view(-1), R, S, stride, pad)
            else:  # padded stem: wgrad into a padded buffer, keep the real channels
                tmp = torch.zeros(Kc * R * S * Cp, device=dy.device, dtype=torch.float32)
                _wgrad(xin, dy, tmp, R, S, stride, pad)
                dW.view(Kc, R, S, xshape[1]).add_(tmp.view(Kc, R, S, Cp)[..., :xshape[1]])
        if not need_input_grad[0]:
            return [None]
        if Cp != xshape[1]:
            dx = K.conv2d_dgrad(dy, wp, (xshape[0], Cp, xshape[2], xshape[3]), stride, pad)
            return [dx[:, :xshape[1]]]
        acc = ctx.extra.get("grad_acc", [None])[0]
        use_acc = (acc is not None and ctx.extra.get("halo") is None and acc.is_cuda and acc.dtype == torch.bfloat16 and tuple(acc.shape) == tuple(xshape)
                   and acc.is_contiguous(memory_format=torch.channels_last))
        fuse_bn = bnsrc is not None and not use_acc
        if _pointwise(R, S, stride, pad, 1):
            def dgrad_gemm(out):
                if tuple(stride) == (1, 1):
                    if out is not None:
                        G.matmul(_rows(dy), wp.view(Kc, Cp), out=_rows(out), beta=1.0, native_only=True)
                        return out
                    dx2 = G.matmul(_rows(dy), wp.view(Kc, Cp), native_only=True)
                    return dx2.view(xshape[0], xshape[2], xshape[3], Cp).permute(0, 3, 1, 2)
                # strided: the gradient lands on the sampled pixels only
                ds = G.matmul(_rows(dy), wp.view(Kc, Cp), native_only=True).view(dy.shape[0], dy.shape[2],
                                                                                  dy.shape[3], Cp)
                if out is None:
                    out = torch.empty(tuple(xshape), device=dy.device, dtype=dy.dtype,
                                      memory_format=torch.channels_last).zero_()
                    out[:, :, ::stride[0], ::stride[1]] = ds.permute(0, 3, 1, 2)
                else:
                    out[:, :, ::stride[0], ::stride[1]] += ds.permute(0, 3, 1, 2)
                return out
            key = ("dgrad", tuple(xshape), Kc, tuple(stride), use_acc)
            if key not in _CHOICE:
                tmp = acc.clone() if use_acc else None
                _pick(key, {"native": lambda: K.conv2d_dgrad(dy, wp, xshape, stride, pad, out=tmp,
                                                             beta=1.0 if use_acc else 0.0),
                            "gemm": lambda: dgrad_gemm(tmp)})
            if _CHOICE[key] == "gemm":
                return [dgrad_gemm(acc if use_acc else None)]
        if fuse_bn:
            # the producing BN's backward sums come out of this dgrad's epilogue
            return [K.conv2d_dgrad(dy, wp, xshape, stride, pad, bn=bnsrc)]
        if use_acc:
            K.conv2d_dgrad(dy, wp, xshape, stride, pad, out=acc, beta=1.0)
            return [acc]
        return [K.conv2d_dgrad(dy, wp, xshape, stride, pad)]


    @staticmethod
    def _backward_grouped(ctx, saved, grad_outputs, weight_grads, need_input_grad, stride, pad, act):
        _, xin, wexp, y, xshape, groups, wshape = saved
        Kc, R, S, Cg = wshape
        dy = K.nhwc(grad_outputs[0].to(torch.bfloat16))
        if act == "relu":
            dy = torch.where(y > 0, dy, torch.zeros((), device=dy.device, dtype=dy.dtype))
        elif act in ("sigmoid", "tanh"):
            yf = y.float()
            d = yf * (1 - yf) if act == "sigmoid" else 1 - yf * yf
            dy = (dy.float() * d).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        if len(weight_grads) > 1 and weight_grads[1] is not None:
            K.colsum_act(dy.permute(0, 2, 3, 1).reshape(-1, Kc), None, "none", weight_grads[1], write_dx=False)
        dW = weight_grads[0]
        if dW is not None:
            if dW.dtype == torch.float32 and dW.is_contiguous():
                K.conv2d_grouped_wgrad(xin, dy, dW.view(-1), R, S, stride, pad, groups=groups)
            else:
                tmp = torch.zeros(dW.numel(), device=dy.device, dtype=torch.float32)
                K.conv2d_grouped_wgrad(xin, dy, tmp, R, S, stride, pad, groups=groups)
                acc_grad(dW, tmp.view(dW.shape))
        if not need_input_grad[0]:
            return [None]
        acc = ctx.extra.get("grad_acc", [None])[0]
        if (acc is not None and ctx.extra.get("halo") is None and acc.is_cuda and acc.dtype == torch.bfloat16
                and tuple(acc.shape) == tuple(xshape) and acc.is_contiguous(memory_format=torch.channels_last)):
            K.conv2d_grouped_dgrad(dy, wexp, wshape, xshape, stride, pad, groups=groups, out=acc, beta=1.0)
            return [acc]
        return [K.conv2d_grouped_dgrad(dy, wexp, wshape, xshape, stride, pad, groups=groups)]

    @staticmethod
    def _backward32(ctx, saved, grad_outputs, weight_grads, need_input_grad, stride, pad, act):
        _, xin, wp, y, xshape, groups = saved
        Kc, R, S, Cg = wp.shape
        dy = grad_outputs[0].to(xin.dtype).contiguous(memory_format=torch.channels_last)
        if act == "relu":
            dy = torch.where(y > 0, dy, torch.zeros((), device=dy.device, dtype=dy.dtype))
        elif act in ("sigmoid", "tanh"):
            yf = y.float()
            d = yf * (1 - yf) if act == "sigmoid" else 1 - yf * yf
            dy = (dy.float() * d).to(xin.dtype).contiguous(memory_format=torch.channels_last)
        if len(weight_grads) > 1 and weight_grads[1] is not None:
            d2 = dy.permute(0, 2, 3, 1).reshape(-1, Kc)
            if Kc % 8 == 0:
                K.colsum_act(d2, None, "none", weight_grads[1], write_dx=False)
            else:
                acc_grad(weight_grads[1], d2.float().sum(0))
        dW = weight_grads[0]
        if dW is not None:
            if dW.dtype == torch.float32 and dW.is_contiguous():
                K.conv32_wgrad(xin, dy, dW.view(-1), R, S, stride, pad, groups=groups)
            else:
                tmp = torch.zeros(dW.numel(), device=dy.device, dtype=torch.float32)
                K.conv32_wgrad(xin, dy, tmp, R, S, stride, pad, groups=groups)
                acc_grad(dW, tmp.view(dW.shape))
        if not need_input_grad[0]:
            return [None]
        acc = ctx.extra.get("grad_acc", [None])[0]
        if (acc is not None and ctx.extra.get("halo") is None and acc.is_cuda and acc.dtype == xin.dtype
                and tuple(acc.shape) == tuple(xshape) and acc.is_contiguous(memory_format=torch.channels_last)):
            K.conv32_dgrad(dy, wp, xshape, stride, pad, groups=groups, out=acc, beta=1.0)
            return [acc]
        return [K.conv32_dgrad(dy, wp, xshape, stride, pad, groups=groups)]


@register("POOL2D")
class Pool2DOp(OpImpl):
    @staticmethod
    def _geom(ctx):
        k = (int(ctx.a("kernel_h")), int(ctx.a("kernel_w")))
        s = (int(ctx.a("stride_h", 1)), int(ctx.a("stride_w", 1)))
        p = (int(ctx.a("padding_h", 0)), int(ctx.a("padding_w", 0)))
        return k, s, p, ctx.a("pool_type", "max") != "max", ctx.a("activation", "none")

    def forward(self, ctx, inputs, weights):
        x = inputs[0]
        k, s, p, avg, act = self._geom(ctx)
        halo = ctx.extra.get("halo")
        if halo is not None:
            return self._halo_forward(ctx, halo, x, k, s, p, avg, act)
        if (x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 4 and x.shape[1] % 8 == 0 and act == "none"
                and k[0] * k[1] <= 256 and K.use_hip(x)):
            xin = K.nhwc(x)
            y, arg = K.pool2d_fwd(xin, k, s, p, avg, count_pad=False, need_argmax=ctx.training)
            return [y], ("hip", tuple(x.shape), arg)
        with torch.no_grad():
            y = self._torch(x, k, s, p, avg, act)
        return [y], ("torch", x)

    @staticmethod
    def _torch(x, k, s, p, avg, act):
        y = F.avg_pool2d(x, k, s, p, count_include_pad=False) if avg else F.max_pool2d(x, k, s, p)
        return _ACTS[act](y)

    @staticmethod
    def _banded(xe, me, k, s, p, avg, act):
        """Pool an H band with its halo / border rows attached (``me`` marks
        the real rows: the average excludes the border, as count_pad=False)."""
        ph, pw = 0, p[1]
        if avg:
            num = F.avg_pool2d(xe, k, s, (ph, pw), count_include_pad=True)
            den = F.avg_pool2d(me, k, s, (ph, pw), count_include_pad=True)
            y = num / den.clamp_min(1e-12)
        else:
            y = F.max_pool2d(xe, k, s, (ph, pw))
        return _ACTS[act](y)

    def _halo_forward(self, ctx, halo, x, k, s, p, avg, act):
        # the border rows: -inf for max pooling, zeros (and a zero mask) for average
        halo.pad_value = 0.0 if avg else float("-inf")
        xe = halo.extend(x)
        me = None
        if avg:   # real rows 1, border rows 0 (known locally: no exchange)
            _, _, _, _, pad_top, pad_bot = halo.plan.rows[halo.index]
            me = torch.ones((1, 1, xe.shape[2], xe.shape[3]), dtype=xe.dtype, device=xe.device)
            me[:, :, :pad_top] = 0
            if pad_bot:
                me[:, :, xe.shape[2] - pad_bot:] = 0
        with torch.no_grad():
            y = self._banded(xe, me, k, s, p, avg, act)
        return [y.to(x.dtype)], ("halo", xe, me)

    def backward(self, ctx, saved, grad_outputs, weight_grads, need_input_grad):
        k, s, p, avg, act = self._geom(ctx)
        if saved[0] == "halo":
            _, xe, me = saved
            xg = xe.detach().requires_grad_(True)
            with torch.enable_grad():
                y = self._banded(xg, me, k, s, p, avg, act)
            y.backward(grad_outputs[0].to(y.dtype))
            return [ctx.extra["halo"].fold(xg.grad)] if need_input_grad[0] else [None]
        if not need_input_grad[0]:
            return [None]
        if saved[0] == "hip":
            _, xshape, arg = saved
            dy = K.nhwc(grad_outputs[0].to(torch.bfloat16))
            return [K.pool2d_bwd(dy, arg, xshape, k, s, p, avg, count_pad=False)]
        x = saved[1].detach().requires_grad_(True)
        with torch.enable_grad():
            y = self._torch(x, k, s, p, avg, act)
        y.backward(grad_outputs[0].to(y.dtype))
        return [x.grad]
