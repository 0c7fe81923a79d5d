"""Generic operator base: the forward is a PyTorch expression; the backward
recomputes it under autograd.  Used for the long tail of operators (shape
manipulation, reductions, pooling, convolution on CPU, ...) that are not on
the hot path of the benchmark models.  Hot operators (Linear, attention,
LayerNorm, embedding, softmax-CE, optimizers) have hand-written HIP paths.

Parity: the remaining lib/kernels ops (reshape/flat/transpose/reverse/
concat/split/gather/reduce/topk/cast/dropout/pool/batch_norm, lib/kernels/src/
cuda/ops/*.cu) and their local-execution task wrappers.
"""
from __future__ import annotations

from typing import List

import torch

from .base import OpContext, OpImpl, acc_grad


def _is_float(t):
    return t is not None and t.is_floating_point()


class AutogradOp(OpImpl):
    """Subclasses implement ``compute(ctx, inputs, weights) -> list``."""

    save_outputs = False

    def compute(self, ctx: OpContext, inputs: List[torch.Tensor], weights: List[torch.Tensor]):
        raise NotImplementedError

    def forward(self, ctx, inputs, weights):
        with torch.no_grad():
            outs = self.compute(ctx, inputs, weights)
        return outs, (inputs, weights)

    def backward(self, ctx, saved, grad_outputs, weight_grads, need_input_grad):
        inputs, weights = saved
        ins = [x.detach().requires_grad_(bool(need_input_grad[i]) and _is_float(x)) if x is not None else None
               for i, x in enumerate(inputs)]
        ws = [w.detach().requires_grad_(weight_grads[i] is not None and _is_float(w))
              for i, w in enumerate(weights)]
        with torch.enable_grad():
            outs = self.compute(ctx, ins, ws)
        pairs = [(o, g) for o, g in zip(outs, grad_outputs) if g is not None and o.requires_grad]
        if pairs:
            torch.autograd.backward([p[0] for p in pairs], [p[1].to(p[0].dtype) for p in pairs])
        for i, w in enumerate(ws):
            if weight_grads[i] is not None and w.grad is not None:
                acc_grad(weight_grads[i], w.grad)
        return [x.grad if (x is not None and x.requires_grad) else None for x in ins]
