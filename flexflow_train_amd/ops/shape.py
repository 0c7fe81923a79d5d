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
