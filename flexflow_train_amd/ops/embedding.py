"""EMBEDDING operator (lookup; SUM/AVG bags).

Parity: lib/kernels/src/cuda/embedding_kernels.cu + local-execution
ops/embedding.cc.  Out-channel (parameter) parallelism: the local weight
piece holds a slice of the output channels, the output piece is the matching
channel slice (op-attrs embedding.cc:63-112).
"""
from __future__ import annotations

import torch

from .. import kernels as K
from .base import OpImpl, acc_grad, register


@register("EMBEDDING")
class EmbeddingOp(OpImpl):
    def forward(self, ctx, inputs, weights):
        idx = inputs[0]
        W = weights[0]
        aggr = ctx.a("aggr", "none")
        if idx.dtype not in (torch.int32, torch.int64):
            idx = idx.long()
        if (W.is_cuda and K.available() and W.dtype in (torch.bfloat16, torch.float32) and W.shape[1] % 8 == 0):
            out = K.embedding_fwd(idx.contiguous(), W.contiguous(), aggr)
        else:
            # out-of-range ids read a zero row (as the HIP kernel does) and
            # get no gradient (both backward paths drop them)
            li = idx.long()
            ok = (li >= 0) & (li < W.shape[0])
            e = torch.nn.functional.embedding(li.clamp(0, W.shape[0] - 1), W) * ok.unsqueeze(-1).to(W.dtype)
            if aggr == "sum":
                e = e.sum(-2)
            elif aggr == "avg":
                e = e.mean(-2)
            out = e
        return [out], (idx, W.shape)

    def backward(self, ctx, saved, grad_outputs, weight_grads, need_input_grad):
        idx, wshape = saved
        dW = weight_grads[0]
        if dW is None:
            return [None]
        g = grad_outputs[0]
        aggr = ctx.a("aggr", "none")
        if ctx.extra.get("track_rows"):
            # row-sparse update (executor): the optimizer touches only these
            # rows; the list is consumed by the update or by zero_gradients
            ctx.extra.setdefault("touched_rows", []).append(idx.reshape(-1))
        if g.is_cuda and K.available() and wshape[1] % 8 == 0 and dW.is_contiguous():
            K.embedding_bwd(idx.contiguous(), g.contiguous(), dW, aggr)
        else:
            D = wshape[1]
            if aggr == "none":
                flat_i = idx.reshape(-1).long()
                flat_g = g.reshape(-1, D).float()
            else:
                L = idx.shape[-1]
                flat_i = idx.reshape(-1).long()
                gg = g.reshape(-1, 1, D).float().expand(-1, L, D)
                if aggr == "avg":
                    gg = gg / L
                flat_g = gg.reshape(-1, D)
            ok = (flat_i >= 0) & (flat_i < wshape[0])
            full = torch.zeros(wshape, dtype=torch.float32, device=g.device)
            full.index_add_(0, flat_i[ok], flat_g[ok])
            acc_grad(dW, full)
        return [None]
