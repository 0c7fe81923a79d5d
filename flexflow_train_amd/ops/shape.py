"""Shape / data-movement operators: RESHAPE, FLAT, TRANSPOSE, REVERSE,
CONCAT, SPLIT, GATHER, REDUCE_*, MEAN, TOPK, BROADCAST, SQUEEZE/UNSQUEEZE,
SLICE, PAD.

Parity: lib/kernels/src/cuda/ops/{reshape,flat,transpose,reverse,concat,
split,gather,reduce,topk}_kernels.cu.  Operating on local pieces: attribute
sizes that refer to partitioned dims are rescaled by the executor
(ctx.output_shapes carries the local output shape).
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

from .base import register
from .generic import AutogradOp


@register("RESHAPE")
class ReshapeOp(AutogradOp):
    def compute(self, ctx, inputs, weights):
        return [inputs[0].reshape(ctx.output_shapes[0])]


@register("FLAT")
class FlatOp(AutogradOp):
    def compute(self, ctx, inputs, weights):
        return [inputs[0].reshape(ctx.output_shapes[0])]


@register("TRANSPOSE")
class TransposeOp(AutogradOp):
    def compute(self, ctx, inputs, weights):
        perm = [int(p) % inputs[0].dim() for p in ctx.a("perm")]
        return [inputs[0].permute(*perm).contiguous()]


@register("REVERSE")
class ReverseOp(AutogradOp):
    def compute(self, ctx, inputs, weights):
        return [torch.flip(inputs[0], [int(ctx.a("axis"))])]


@register("CONCAT")
class ConcatOp(AutogradOp):
    def compute(self, ctx, inputs, weights):
        return [torch.cat(inputs, dim=int(ctx.a("axis")))]


@register("SPLIT")
class SplitOp(AutogradOp):
    def compute(self, ctx, inputs, weights):
        axis = int(ctx.a("axis")) % inputs[0].dim()
        sizes = [s[axis] for s in ctx.output_shapes]
        return [t.contiguous() for t in torch.split(inputs[0], sizes, dim=axis)]


@register("GATHER")
class GatherOp(AutogradOp):
    def compute(self, ctx, inputs, weights):
        return [torch.gather(inputs[0], int(ctx.a("dim")), inputs[1].long())]


_REDUCE = {
    "REDUCE_SUM": lambda x, ax, k: x.sum(ax, keepdim=k),
    "REDUCE_MEAN": lambda x, ax, k: x.mean(ax, keepdim=k),
    "MEAN": lambda x, ax, k: x.mean(ax, keepdim=k),
    "REDUCE_MAX": lambda x, ax, k: x.amax(ax, keepdim=k),
    "REDUCE_MIN": lambda x, ax, k: x.amin(ax, keepdim=k),
    "REDUCE_PROD": lambda x, ax, k: x.prod(ax[0], keepdim=k) if len(ax) == 1 else x.flatten().prod(),
    "REDUCE_ARGMAX": lambda x, ax, k: x.argmax(ax[0], keepdim=k),
    "REDUCE_ARGMIN": lambda x, ax, k: x.argmin(ax[0], keepdim=k),
}


@register(*_REDUCE.keys())
class ReduceOp(AutogradOp):
    def compute(self, ctx, inputs, weights):
        x = inputs[0]
        axes = tuple(int(a) % x.dim() for a in ctx.a("axes"))
        r = _REDUCE[ctx.op_type](x, axes, bool(ctx.a("keepdims", False)))
        if ctx.op_type in ("REDUCE_MEAN", "MEAN") and ctx.extra.get("mean_scale"):
            # a partitioned reduced axis: local mean * (local/global) -> partial sum of the global mean
            r = r * ctx.extra["mean_scale"]
        return [r]


@register("TOPK")
class TopKOp(AutogradOp):
    def compute(self, ctx, inputs, weights):
        v, i = torch.topk(inputs[0], int(ctx.a("k")), dim=-1, sorted=bool(ctx.a("sorted", True)))
        return [v, i.to(torch.int32)]


@register("BROADCAST")
class BroadcastOp(AutogradOp):
    def compute(self, ctx, inputs, weights):
        return [inputs[0].expand(ctx.output_shapes[0]).contiguous()]


@register("SQUEEZE", "UNSQUEEZE")
class SqueezeOp(AutogradOp):
    def compute(self, ctx, inputs, weights):
        return [inputs[0].reshape(ctx.output_shapes[0])]


@register("SLICE")
class SliceOp(AutogradOp):
    def compute(self, ctx, inputs, weights):
        x = inputs[0]
        idx = [slice(None)] * x.dim()
        for a, s, e in zip(ctx.a("axes"), ctx.a("starts"), ctx.a("ends")):
            idx[int(a) % x.dim()] = slice(int(s), int(e))
        return [x[tuple(idx)].contiguous()]


@register("PAD")
class PadOp(AutogradOp):
    def compute(self, ctx, inputs, weights):
        x = inputs[0]
        pads = [int(p) for p in ctx.a("pads")]
        tp = []
        for d in reversed(range(x.dim())):
            tp += [pads[2 * d], pads[2 * d + 1]]
        return [F.pad(x, tp)]


# ---------------------------------------------------------------------------
# HIP paths (csrc/kernels/tensorops.hip) for the data-movement operators; the
# autograd-recompute implementations above remain the CPU path.
from .. import kernels as K  # noqa: E402


def _hip(*ts) -> bool:
    return K.tensorop_ok(*ts) and all(t.dim() <= 6 for t in ts)


def _expand(t, shape):
    """Materialise a broadcast of ``t`` (same rank, 1s on broadcast dims) to ``shape``."""
    st = K._bcast_strides(list(t.shape), list(shape))
    y = torch.empty(list(shape), device=t.device, dtype=t.dtype)
    K.ext().permute_nd(K._dt(t), t.data_ptr(), y.data_ptr(), list(shape), st, K._stream())
    return y


@register("TRANSPOSE")
class HipTransposeOp(TransposeOp):
    def forward(self, ctx, inputs, weights):
        x = inputs[0]
        perm = [int(p) % x.dim() for p in ctx.a("perm")]
        if _hip(x):
            return [K.permute(x, perm)], ("hip", perm)
        return super().forward(ctx, inputs, weights)

    def backward(self, ctx, saved, grad_outputs, weight_grads, need_input_grad):
        if saved[0] == "hip":
            inv = [0] * len(saved[1])
            for i, p in enumerate(saved[1]):
                inv[p] = i
            return [K.permute(grad_outputs[0].contiguous(), inv)]
        return super().backward(ctx, saved, grad_outputs, weight_grads, need_input_grad)


@register("REVERSE")
class HipReverseOp(ReverseOp):
    def forward(self, ctx, inputs, weights):
        x = inputs[0]
        if _hip(x):
            return [K.reverse(x, int(ctx.a("axis")))], ("hip",)
        return super().forward(ctx, inputs, weights)

    def backward(self, ctx, saved, grad_outputs, weight_grads, need_input_grad):
        if saved[0] == "hip":
            return [K.reverse(grad_outputs[0].contiguous(), int(ctx.a("axis")))]
        return super().backward(ctx, saved, grad_outputs, weight_grads, need_input_grad)


@register("CONCAT")
class HipConcatOp(ConcatOp):
    def forward(self, ctx, inputs, weights):
        if _hip(*inputs) and len({t.dtype for t in inputs}) == 1:
            axis = int(ctx.a("axis")) % inputs[0].dim()
            return [K.concat(list(inputs), axis)], ("hip", axis, [int(t.shape[axis]) for t in inputs])
        return super().forward(ctx, inputs, weights)

    def backward(self, ctx, saved, grad_outputs, weight_grads, need_input_grad):
        if saved[0] == "hip":
            _, axis, sizes = saved
            parts = K.split(grad_outputs[0].contiguous(), sizes, axis)
            return [p if need else None for p, need in zip(parts, need_input_grad)]
        return super().backward(ctx, saved, grad_outputs, weight_grads, need_input_grad)


@register("SPLIT")
class HipSplitOp(SplitOp):
    def forward(self, ctx, inputs, weights):
        x = inputs[0]
        if _hip(x):
            axis = int(ctx.a("axis")) % x.dim()
            sizes = [int(s[axis]) for s in ctx.output_shapes]
            return K.split(x, sizes, axis), ("hip", axis, sizes, x.dtype)
        return super().forward(ctx, inputs, weights)

    def backward(self, ctx, saved, grad_outputs, weight_grads, need_input_grad):
        if saved[0] == "hip":
            _, axis, sizes, dt = saved
            gs = []
            for g, shp in zip(grad_outputs, ctx.output_shapes):
                gs.append(g.contiguous().to(dt) if g is not None else torch.zeros(shp, device=ctx.device, dtype=dt))
            return [K.concat(gs, axis)]
        return super().backward(ctx, saved, grad_outputs, weight_grads, need_input_grad)


@register("GATHER")
class HipGatherOp(GatherOp):
    def forward(self, ctx, inputs, weights):
        x, idx = inputs
        if _hip(x) and idx.is_cuda and idx.dtype in (torch.int32, torch.int64):
            dim = int(ctx.a("dim")) % x.dim()
            idx = idx.contiguous()
            return [K.gather(x, idx, dim)], ("hip", idx, dim, tuple(x.shape), x.dtype)
        return super().forward(ctx, inputs, weights)

    def backward(self, ctx, saved, grad_outputs, weight_grads, need_input_grad):
        if saved[0] == "hip":
            _, idx, dim, xs, dt = saved
            return [K.scatter_add(grad_outputs[0].contiguous().to(dt), idx, dim, list(xs)).to(dt), None]
        return super().backward(ctx, saved, grad_outputs, weight_grads, need_input_grad)


_HIP_REDUCE = {"REDUCE_SUM": "sum", "REDUCE_MEAN": "mean", "MEAN": "mean", "REDUCE_MAX": "max",
               "REDUCE_MIN": "min"}


@register(*_REDUCE.keys())
class HipReduceOp(ReduceOp):
    def forward(self, ctx, inputs, weights):
        x = inputs[0]
        axes = sorted({int(a) % x.dim() for a in ctx.a("axes")})
        contiguous_axes = axes and axes == list(range(axes[0], axes[-1] + 1))
        if ctx.op_type in _HIP_REDUCE and _hip(x) and contiguous_axes and not ctx.extra.get("mean_scale"):
            kind = _HIP_REDUCE[ctx.op_type]
            r = K.reduce_contig(x, axes[0], axes[-1], kind)
            keep_shape = [1 if i in axes else s for i, s in enumerate(x.shape)]
            out = r.reshape(keep_shape) if bool(ctx.a("keepdims", False)) else r
            return [out], ("hip", x if kind in ("max", "min") else None, r, kind, keep_shape, tuple(x.shape))
        return super().forward(ctx, inputs, weights)

    def backward(self, ctx, saved, grad_outputs, weight_grads, need_input_grad):
        if saved[0] == "hip":
            _, x, r, kind, keep_shape, xs = saved
            g = grad_outputs[0].contiguous().to(r.dtype).reshape(keep_shape)
            dx = _expand(g, xs)
            if kind == "mean":
                red = 1
                for a, b in zip(keep_shape, xs):
                    red *= b // a
                dx = K.unary(dx, "SCALAR_MULTIPLY", 1.0 / red)
            elif kind in ("max", "min"):
                mask = K.binary(x, _expand(r.reshape(keep_shape), xs), "EW_EQUAL")
                dx = K.binary(dx, mask, "EW_MUL")
            return [dx]
        return super().backward(ctx, saved, grad_outputs, weight_grads, need_input_grad)


@register("TOPK")
class HipTopKOp(TopKOp):
    def forward(self, ctx, inputs, weights):
        x = inputs[0]
        k = int(ctx.a("k"))
        if _hip(x) and k <= x.shape[-1]:
            v, i = K.topk(x.contiguous(), k)
            return [v, i.to(torch.int32)], ("hip", i, tuple(x.shape))
        return super().forward(ctx, inputs, weights)

    def backward(self, ctx, saved, grad_outputs, weight_grads, need_input_grad):
        if saved[0] == "hip":
            _, idx, xs = saved
            g = grad_outputs[0]
            if g is None:
                return [None]
            return [K.scatter_add(g.contiguous(), idx, len(xs) - 1, list(xs)).to(g.dtype)]
        return super().backward(ctx, saved, grad_outputs, weight_grads, need_input_grad)
