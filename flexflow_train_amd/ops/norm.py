"""LAYERNORM (optionally fused with the residual add) and BATCHNORM.

Parity: lib/kernels/src/cuda/ops/layer_norm_kernels.cu, batch_norm_kernels.cu
(cuDNN training-mode BN with running stats and optional fused ReLU).

``FUSED_ADD_LAYERNORM`` is produced by the executor's fusion pass from
EW_ADD -> LAYERNORM (the post-LN transformer block): one HIP kernel reads
both operands once and writes y, the pre-norm sum and the row statistics.
"""
from __future__ import annotations

import math

import torch

from .. import kernels as K
from .base import OpImpl, acc_grad, register


def _bn_sums_from_conv() -> bool:
    from . import conv
    return conv._CONV_BN_BWD


def _ln_axes_are_trailing(ctx, x):
    axes = sorted(int(a) % x.dim() for a in ctx.a("axes", [-1]))
    return axes == list(range(x.dim() - len(axes), x.dim())), len(axes)


class _LayerNormBase(OpImpl):
    fused_add = False

    def forward(self, ctx, inputs, weights):
        x = inputs[0]
        res = inputs[1] if self.fused_add else None
        eps = float(ctx.a("eps", 1e-5))
        gamma = weights[0] if len(weights) > 0 else None
        beta = weights[1] if len(weights) > 1 else None
        trailing, nax = _ln_axes_are_trailing(ctx, x)
        N = int(math.prod(x.shape[x.dim() - nax:]))
        if (x.is_cuda and trailing and N % 8 == 0 and x.dtype in (torch.bfloat16, torch.float32) and K.available()):
            xc = x.contiguous()
            rc = res.contiguous() if res is not None else None
            g = gamma.reshape(-1) if gamma is not None else None
            b = beta.reshape(-1) if beta is not None else None
            y, s, mean, rstd = K.layernorm_fwd(xc.view(-1, N), g, b, eps,
                                               residual=rc.view(-1, N) if rc is not None else None)
            outs = [y.view(x.shape)]
            if ctx.extra.get("emit_sum"):
                outs.append(s.view(x.shape))
            return outs, ("hip", s, mean, rstd, gamma, N)
        xs = x + res if res is not None else x
        shape = x.shape[x.dim() - nax:] if trailing else None
        if not trailing:
            raise NotImplementedError("LAYERNORM over non-trailing axes")
        with torch.no_grad():
            y = torch.nn.functional.layer_norm(xs.float(), shape, gamma.float() if gamma is not None else None,
                                               beta.float() if beta is not None else None, eps).to(x.dtype)
        outs = [y]
        if ctx.extra.get("emit_sum"):
            outs.append(xs)
        return outs, ("torch", xs, gamma, beta, shape, eps)

    def backward(self, ctx, saved, grad_outputs, weight_grads, need_input_grad):
        dy = grad_outputs[0]
        dsum_in = grad_outputs[1] if len(grad_outputs) > 1 else None   # other consumers of the sum
        dg = weight_grads[0] if len(weight_grads) > 0 else None
        db = weight_grads[1] if len(weight_grads) > 1 else None
        target = ctx.extra.pop("dsum_target", None)
        if saved[0] == "hip":
            _, s, mean, rstd, gamma, N = saved
            dres = None
            if dsum_in is not None:
                dres = dsum_in.contiguous().view(-1, N)
                if dres.dtype != dy.dtype:
                    dres = dres.to(dy.dtype)
            dsum = None
            if target is not None and target[0] is not None and target[0].dtype == torch.float32 \
                    and target[0].is_contiguous() and target[0].numel() == N:
                dsum = target[0].reshape(-1)
            dx = K.layernorm_bwd(dy.contiguous().view(-1, N), s, mean, rstd,
                                 gamma.reshape(-1) if gamma is not None else None,
                                 dg.reshape(-1) if dg is not None else None,
                                 db.reshape(-1) if db is not None else None,
                                 dres=dres, dsum=dsum).view(dy.shape)
            if dsum is not None:
                target[1].extra["db_done"] = True
        else:
            _, xs, gamma, beta, shape, eps = saved
            xf = xs.detach().float().requires_grad_(True)
            gf = gamma.detach().float().requires_grad_(dg is not None) if gamma is not None else None
            bf = beta.detach().float().requires_grad_(db is not None) if beta is not None else None
            with torch.enable_grad():
                y = torch.nn.functional.layer_norm(xf, shape, gf, bf, eps)
            y.backward(dy.float())
            dx = xf.grad.to(dy.dtype)
            if dsum_in is not None:
                dx = dx + dsum_in.to(dx.dtype)
            if dg is not None:
                acc_grad(dg, gf.grad)
            if db is not None:
                acc_grad(db, bf.grad)
        if self.fused_add:
            return [dx, dx]
        return [dx]


@register("LAYERNORM")
class LayerNormOp(_LayerNormBase):
    fused_add = False


@register("FUSED_ADD_LAYERNORM")
class FusedAddLayerNormOp(_LayerNormBase):
    fused_add = True


@register("BATCHNORM")
class BatchNormOp(OpImpl):
    """Training-mode batch norm over the sample + spatial dims, running stats
    kept in the op's persistent state (ctx.extra['state']).

    GPU (bnpool.hip): per-channel statistics come from the producing
    convolution's epilogue when the executor paired them (``_ff_bn_stats`` on
    the input tensor) or from one reduction pass; apply = one fused pass
    (scale/shift [+ residual] [ReLU]); backward = one reduction + one apply
    pass.  ``ctx.extra['residual_relu']`` (set by the executor's
    BATCHNORM -> EW_ADD -> RELU fusion) makes the op compute
    relu(bn(x) + residual) and return the residual's gradient too.
    """

    @staticmethod
    def _state(ctx, C, dev):
        state = ctx.extra.setdefault("state", {})
        if "running_mean" not in state or state["running_mean"].device != dev:
            state["running_mean"] = torch.zeros(C, device=dev, dtype=torch.float32)
            state["running_var"] = torch.ones(C, device=dev, dtype=torch.float32)
        return state

    def forward(self, ctx, inputs, weights):
        x = inputs[0]
        fused = bool(ctx.extra.get("residual_relu"))
        res = inputs[1] if fused else None
        relu = True if fused else bool(ctx.a("relu", False))
        C = x.shape[1]
        state = self._state(ctx, C, x.device)
        g = weights[0] if weights else None
        b = weights[1] if len(weights) > 1 else None
        eps = float(ctx.a("eps", 1e-5))
        mom = float(ctx.a("momentum", 0.1))
        if (x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 4 and C % 8 == 0 and K.use_hip(x)
                and (res is None or (res.dtype == x.dtype and res.shape == x.shape))):
            stats_in = getattr(x, "_ff_bn_stats", None)
            xin = K.nhwc(x)
            if ctx.training:
                stats = stats_in
                if stats is None:
                    stats = torch.empty(2 * C, device=x.device, dtype=torch.float32)
                    K.bn_stats(xin, stats, overwrite=True)
                scale, shift, mean, rstd = K.bn_finalize(stats, g, b, xin.numel() // C, eps, mom,
                                                         state["running_mean"], state["running_var"])
            else:
                rstd = torch.rsqrt(state["running_var"] + eps)
                mean = state["running_mean"]
                gf = g.float() if g is not None else torch.ones_like(rstd)
                bf = b.float() if b is not None else torch.zeros_like(rstd)
                scale = (gf * rstd).contiguous()
                shift = (bf - mean * gf * rstd).contiguous()
            y = K.bn_apply(xin, scale, shift, relu, residual=None if res is None else K.nhwc(res))
            ss = None
            if relu and not fused and ctx.training:
                # backward recomputes the ReLU mask from x (scale / shift are
                # rows 0 and 1 of bn_finalize's [4, C] buffer): y is not kept
                assert shift.data_ptr() == scale.data_ptr() + 4 * C
                ss = torch.as_strided(scale, (2 * C,), (1,))
            if (ctx.training and not fused and ctx.extra.get("bn_sums_from_conv") and _bn_sums_from_conv()
                    and (ss is not None or not relu)):
                # the consuming conv's dgrad reduces this BN's backward sums (conv.hip)
                y._ff_bn_bwd = (xin, mean, rstd, ss)
            return [y], ("hip", xin, y if (relu and ss is None) else None, mean, rstd, g, relu, fused, ss)
        train = ctx.training
        xf = x.float()
        y = torch.nn.functional.batch_norm(
            xf, state["running_mean"], state["running_var"],
            g.float() if g is not None else None, b.float() if b is not None else None,
            training=train, momentum=mom if train else 0.0, eps=eps)
        if res is not None:
            y = y + res.float()
        if relu:
            y = torch.relu(y)
        return [y.to(x.dtype)], ("torch", x, res, g, b, relu)

    def backward(self, ctx, saved, grad_outputs, weight_grads, need_input_grad):
        dy = grad_outputs[0]
        dg = weight_grads[0] if weight_grads else None
        db = weight_grads[1] if len(weight_grads) > 1 else None
        if saved[0] == "hip":
            _, xin, y, mean, rstd, g, relu, fused, ss = saved
            dyn = K.nhwc(dy.to(torch.bfloat16))
            pre = getattr(dyn, "_ff_bn_sums", None)
            pre = pre[0] if pre is not None and pre[1] is xin and not fused else None
            dx, dres = K.bn_bwd(dyn, xin, y, mean, rstd, g, relu, dgamma=dg, dbeta=db, want_masked=fused,
                                scale_shift=ss, pre_sums=pre)
            return [dx, dres] if fused else [dx]
        _, x, res, g, b, relu = saved
        eps = float(ctx.a("eps", 1e-5))
        xi = x.detach().float().requires_grad_(True)
        gr = g.detach().float().requires_grad_(True) if g is not None else None
        br = b.detach().float().requires_grad_(True) if b is not None else None
        rr = res.detach().float().requires_grad_(True) if res is not None else None
        with torch.enable_grad():
            y = torch.nn.functional.batch_norm(xi, None, None, gr, br, training=True, eps=eps)
            if rr is not None:
                y = y + rr
            if relu:
                y = torch.relu(y)
        y.backward(dy.float())
        if dg is not None and gr is not None:
            acc_grad(dg, gr.grad)
        if db is not None and br is not None:
            acc_grad(db, br.grad)
        outs = [xi.grad.to(x.dtype)]
        if rr is not None:
            outs.append(rr.grad.to(res.dtype))
        return outs
