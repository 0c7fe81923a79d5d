"""LINEAR and BATCHMATMUL operators.

Parity: lib/local-execution/src/ops/linear.cc + lib/kernels/src/cuda/ops/
linear_kernels.cu (forward GEMM + bias + activation, backward activation
grad in place, dW += X dY^T, db += sum dY, dX += W dY — gradients accumulate,
:109-327); batch_matmul_kernels.cu.  The local-execution bug
`in_dim = shape[0] + 1` (linear.cc:99-101) is not reproduced.

Parallel semantics (op-attrs linear.cc:73-140): a row-parallel shard
(input last dim sharded -> output partial sums) adds the bias only on the
partial-sum replica 0, so the Reduction that follows sums it once.
"""
from __future__ import annotations

import os

import torch

from .. import kernels as K
from .base import OpContext, OpImpl, acc_grad, register
from .gemm import matmul, wgrad_matmul

_ACT_T = {
    "none": lambda t: t,
    "relu": torch.relu,
    "sigmoid": torch.sigmoid,
    "tanh": torch.tanh,
    "gelu": lambda t: torch.nn.functional.gelu(t, approximate="tanh"),
}


@register("LINEAR")
class LinearOp(OpImpl):
    def forward(self, ctx: OpContext, inputs, weights):
        x = inputs[0]
        W = weights[0]
        b = weights[1] if len(weights) > 1 and ctx.sum_index == 0 else None
        act = ctx.a("activation", "none")
        lead = x.shape[:-1]
        x2 = x.reshape(-1, x.shape[-1])
        if not x2.is_contiguous():
            x2 = x2.contiguous()
        if x2.is_cuda and W.shape[1] <= 8 and K.narrow_ok(x2, W if W.dtype == x2.dtype else W.to(x2.dtype)):
            # narrow head (N <= 8, e.g. DLRM's sigmoid output): GEMV-shaped
            # kernel with bias + activation fused (elementwise.hip narrow_*)
            Wc = W if W.dtype == x2.dtype else W.to(x2.dtype)
            pre = torch.empty(x2.shape[0], W.shape[1], device=x2.device, dtype=x2.dtype) if act != "none" else None
            y = K.narrow_linear_fwd(x2, Wc, bias=b, act=act, pre=pre)
        elif x2.is_cuda and x2.dtype in (torch.bfloat16, torch.float32):
            # bf16: the autotuned MFMA GEMMs; fp32: the exact-fp32 MFMA kernel
            # (igemm32.hip) -- no library GEMM either way
            Wc = W if W.dtype == x2.dtype else W.to(x2.dtype)
            pre = torch.empty(x2.shape[0], W.shape[1], device=x2.device, dtype=x2.dtype) if act != "none" else None
            y = matmul(x2, Wc, bias=b, act=act, pre=pre)
        else:
            u = x2 @ W.to(x2.dtype)
            if b is not None:
                u = u + b.to(u.dtype)
            pre = u if act != "none" else None
            y = _ACT_T[act](u)
        return [y.reshape(*lead, W.shape[1])], (x2, pre, W)

    def backward(self, ctx, saved, grad_outputs, weight_grads, need_input_grad):
        x2, pre, W = saved
        dy = grad_outputs[0]
        act = ctx.a("activation", "none")
        dy2 = dy.reshape(-1, dy.shape[-1])
        if not dy2.is_contiguous():
            dy2 = dy2.contiguous()
        has_bias = len(weight_grads) > 1
        # every partial-sum replica computes the (identical) bias gradient so the
        # stored copies stay in sync; only replica 0 adds the bias in forward
        db = weight_grads[1] if has_bias else None
        dW = weight_grads[0]
        if ctx.extra.pop("db_done", False):
            db = None   # accumulated by the consuming add+LayerNorm's backward (layernorm_bwd dsum)
        if ctx.extra.pop("grad_is_preact", False):
            # the consumer's dX GEMM already applied act' and accumulated db (gemmp epilogue)
            act = "none"
            db = None
        Wb = W if W.dtype == torch.bfloat16 else None
        if (dy2.is_cuda and dy2.dtype == torch.bfloat16 and W.shape[1] <= 8 and Wb is not None
                and K.narrow_ok(x2, Wb) and (pre is None or pre.dtype == torch.bfloat16)
                and (dW is None or dW.dtype in (torch.float32, torch.bfloat16))):
            # narrow head: weight / bias / input gradients with act' fused, no
            # separate activation-gradient or column-sum pass
            ctx.extra.pop("dact", None)
            acc = ctx.extra.get("grad_acc", [None])[0] if need_input_grad[0] else None
            acc_ok = acc is not None and acc.is_cuda and acc.dtype == torch.bfloat16 and acc.is_contiguous()
            dx = K.narrow_linear_bwd(x2, Wb, dy2, pre=pre, act=act, dw=dW,
                                     wbeta=ctx.extra.get("wgrad_beta", [1.0])[0], db=db,
                                     dx=acc.view(-1, W.shape[0]) if acc_ok else None, dx_beta=1.0 if acc_ok else 0.0,
                                     need_dx=bool(need_input_grad[0]))
            if acc_ok:
                return [acc]
            return [dx.reshape(*dy.shape[:-1], W.shape[0]) if dx is not None else None]
        if (dy2.is_cuda and dy2.dtype in (torch.bfloat16, torch.float32) and K.available() and dy2.shape[1] % 8 == 0
                and (pre is None or pre.dtype == dy2.dtype)):
            if act != "none":
                g = K.colsum_act(dy2, pre, act, db, write_dx=True)
            else:
                g = dy2
                if db is not None:
                    K.colsum_act(dy2, None, "none", db, write_dx=False)
        else:
            if act != "none":
                p = pre.float().detach().requires_grad_(True)
                y = _ACT_T[act](p)
                y.backward(dy2.float())
                g = p.grad.to(dy2.dtype)
            else:
                g = dy2
            if db is not None:
                acc_grad(db, g.float().sum(0))
        if dW is not None:
            if dW.is_cuda and g.dtype == torch.bfloat16:
                wgrad_matmul(ctx, x2, g, dW, ctx.extra.get("wgrad_beta", [1.0])[0])
            elif dW.is_cuda and g.dtype == torch.float32 and x2.dtype == torch.float32 and dW.dtype == torch.float32:
                matmul(x2, g, trans_a=True, out=dW, beta=ctx.extra.get("wgrad_beta", [1.0])[0])
            else:
                acc_grad(dW, x2.float().t() @ g.float())
        dx = None
        dact = ctx.extra.pop("dact", None)
        if need_input_grad[0] and dact is not None and g.is_cuda and g.dtype == torch.bfloat16:
            act_p, pre_p, db_p, pctx = dact
            pre2 = pre_p.reshape(-1, W.shape[0])
            ok = (W.dtype == torch.bfloat16 and pre2.dtype == torch.bfloat16 and pre2.is_contiguous()
                  and pre2.shape[0] == g.shape[0] and (db_p is None or (db_p.dtype == torch.float32
                                                                      and db_p.is_contiguous()))
                  and K.gemmp_supported(g, W, False, True))
            if ok and _dact_fused_wins(g, W, pre2, act_p, db_p is not None):
                dx = K.gemmp(g, W, trans_b=True, act=act_p, aux=pre2, act_bwd=True,
                             dbias=db_p.reshape(-1) if db_p is not None else None,
                             variant=_dact_variant(act_p, g.shape[0], W.shape[0]))
                pctx.extra["grad_is_preact"] = True
                return [dx.reshape(*dy.shape[:-1], W.shape[0])]
        if need_input_grad[0]:
            acc = ctx.extra.get("grad_acc", [None])[0]
            if acc is not None and acc.is_cuda and acc.dtype == g.dtype and acc.is_contiguous():
                matmul(g, W, trans_b=True, out=acc.view(-1, W.shape[0]), beta=1.0)
                return [acc]
            dx = matmul(g, W if W.dtype == g.dtype else W.to(g.dtype), trans_b=True) if g.is_cuda else (g @ W.to(g.dtype).t())
            dx = dx.reshape(*dy.shape[:-1], W.shape[0])
        return [dx]


_DACT_CHOICE = {}
_DACT_TIMES = {}


def _dact_variant(act: str, M: int = 1 << 30, N: int = 1 << 30) -> int:
    """The fused activation-gradient GEMM runs on the 64x64-tile MLP kernel
    (gemms.hip) when 256x256 tiles cannot fill the chip, else on gemmt (one
    wave per SIMD, 128x128 wave tiles, operands staged by LDS-DMA) for the
    activations it instantiates, else on gemmp."""
    from .gemm import _GT_DMA, _GT_VARIANT, _small_mn
    if _small_mn(M, N) and os.environ.get("FF_GEMMS", "1") != "0":
        return 8
    if not _GT_VARIANT or act not in ("relu", "gelu"):
        return 0
    return 6 if _GT_DMA else _GT_VARIANT   # both operands by LDS-DMA (the dact GEMM is NT)


def _dact_fused_wins(g, W, pre, act, has_bias) -> bool:
    """Measure once per shape (outside graph capture): the fused input-gradient
    GEMM with the activation-gradient + bias-gradient epilogue (gemmp) against
    the autotuned plain GEMM followed by the producer's colsum_act pass."""
    key = (tuple(g.shape), tuple(W.shape), act, has_bias)
    hit = _DACT_CHOICE.get(key)
    if hit is not None:
        return hit
    if torch.cuda.is_current_stream_capturing():
        return False
    from .gemm import _time_all
    db = torch.zeros(W.shape[0], device=g.device, dtype=torch.float32)
    dx = matmul(g, W, trans_b=True)   # settles the autotuner's pick first
    t = _time_all({
        "fused": lambda: K.gemmp(g, W, trans_b=True, act=act, aux=pre, act_bwd=True,
                                 dbias=db if has_bias else None, variant=_dact_variant(act, g.shape[0], W.shape[0])),
        "plain": lambda: (matmul(g, W, trans_b=True),
                          K.colsum_act(dx, pre, act, db if has_bias else None, write_dx=True))})
    fused, plain = t["fused"], t["plain"]
    _DACT_CHOICE[key] = fused < plain
    _DACT_TIMES[key] = (fused, plain)
    return _DACT_CHOICE[key]


def dact_report() -> str:
    """One line per input-gradient GEMM that could fuse the activation
    gradient: fused (gemmt / gemmp epilogue) vs plain GEMM + colsum_act, ms."""
    return "\n".join(f"dact g{list(k[0])} W{list(k[1])} act={k[2]} bias={int(k[3])} -> "
                     f"{'fused' if _DACT_CHOICE.get(k) else 'plain'}  fused:{f:.3f} plain:{p:.3f}"
                     for k, (f, p) in _DACT_TIMES.items())


def _bmm(a, b, trans_a=False, trans_b=False):
    """Batched product on the hand-written 64x64-tile kernel (gemms.hip,
    one launch for the whole batch) when the shapes allow, else torch."""
    if K.bmm_supported(a, b, trans_a, trans_b):
        return K.bmm(a, b, trans_a, trans_b)
    if a.is_cuda and a.dtype == torch.float32 and b.dtype == torch.float32 and K.use_hip(a, b):
        return K.bmm_f32(a, b, trans_a, trans_b)   # exact-fp32 MFMA (igemm32.hip)
    return torch.matmul(a.transpose(-1, -2) if trans_a else a, b.transpose(-1, -2) if trans_b else b)


@register("BATCHMATMUL", "MATMUL")
class BatchMatmulOp(OpImpl):
    """Parity: batch_matmul_kernels.cu:66-123 (forward, dA = dC B^T, dB = A^T dC)."""

    def forward(self, ctx, inputs, weights):
        a, b = inputs
        if a.dim() == b.dim() and a.dim() >= 3 and a.shape[:-2] == b.shape[:-2]:
            return [_bmm(a.contiguous(), b.contiguous())], (a, b)
        return [torch.matmul(a, b)], (a, b)

    def backward(self, ctx, saved, grad_outputs, weight_grads, need_input_grad):
        a, b = saved
        d = grad_outputs[0]
        if a.dim() == b.dim() and a.dim() >= 3 and a.shape[:-2] == b.shape[:-2]:
            d = d.contiguous()
            da = _bmm(d, b.contiguous(), trans_b=True) if need_input_grad[0] else None
            db = _bmm(a.contiguous(), d, trans_a=True) if need_input_grad[1] else None
            return [da, db]
        da = torch.matmul(d, b.transpose(-1, -2)) if need_input_grad[0] else None
        db = torch.matmul(a.transpose(-1, -2), d) if need_input_grad[1] else None
        return [da, db]
