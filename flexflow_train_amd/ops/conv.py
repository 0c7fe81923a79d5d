"""CONV2D and POOL2D operators.

Parity: lib/kernels/src/cuda/ops/conv_2d_kernels.cu (cuDNN conv with
autotuned algorithms, fused bias + activation, :8-391) and
pool_2d_kernels.cu.  Channel parallelism follows op-attrs conv_2d.cc: an
input-channel shard produces partial sums (bias on replica 0 only), an
output-channel shard is expressed by the weight piece.

MI355X path: bf16 convolution through PyTorch-ROCm (MIOpen, channels-last
NHWC so MIOpen picks its implicit-GEMM MFMA solvers), bias + activation
applied in the same expression so MIOpen's fusion can take them.  A
hand-written implicit-GEMM MFMA convolution is future work.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from .base import register
from .generic import AutogradOp

_ACTS = {"none": lambda t: t, "relu": torch.relu, "sigmoid": torch.sigmoid, "tanh": torch.tanh,
         "gelu": lambda t: F.gelu(t, approximate="tanh")}


@register("CONV2D")
class Conv2DOp(AutogradOp):
    def compute(self, ctx, inputs, weights):
        x = inputs[0]
        W = weights[0]
        b = weights[1] if len(weights) > 1 and ctx.sum_index == 0 else None
        if x.is_cuda:
            x = x.contiguous(memory_format=torch.channels_last)
        y = F.conv2d(x, W.to(x.dtype), b.to(x.dtype) if b is not None else None,
                     stride=(int(ctx.a("stride_h", 1)), int(ctx.a("stride_w", 1))),
                     padding=(int(ctx.a("padding_h", 0)), int(ctx.a("padding_w", 0))),
                     groups=int(ctx.a("groups", 1)))
        return [_ACTS[ctx.a("activation", "none")](y)]


@register("POOL2D")
class Pool2DOp(AutogradOp):
    def compute(self, ctx, inputs, weights):
        x = inputs[0]
        k = (int(ctx.a("kernel_h")), int(ctx.a("kernel_w")))
        s = (int(ctx.a("stride_h", 1)), int(ctx.a("stride_w", 1)))
        p = (int(ctx.a("padding_h", 0)), int(ctx.a("padding_w", 0)))
        if ctx.a("pool_type", "max") == "max":
            y = F.max_pool2d(x, k, s, p)
        else:
            y = F.avg_pool2d(x, k, s, p, count_include_pad=False)
        return [_ACTS[ctx.a("activation", "none")](y)]
