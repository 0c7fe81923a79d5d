"""Element-wise unary / binary / scalar operators, dropout, cast, softmax.

Parity: lib/kernels/src/cuda/ops/element_unary_kernels.cu,
element_binary_kernels.cu (broadcasting, backward reduces over broadcast
dims), dropout_kernels.cu, cast_kernels.cu, softmax_kernels.cu.  The
reference's ELEMENTUNARY_BWD_TASK_ID -> binary-bwd mapping bug
(task_signature_impl.cc:52-54) is not reproduced.

Activations run through the HIP activation kernels on GPU (16-byte vector
loads, regenerated dropout masks); broadcasting binaries use PyTorch-ROCm's
element-wise library kernels (not on a hot path of the benchmark models).
"""
from __future__ import annotations

import torch

from .. import kernels as K
from .base import OpImpl, register
from .generic import AutogradOp

_HIP_ACTS = {"RELU": "relu", "SIGMOID": "sigmoid", "TANH": "tanh", "GELU": "gelu", "ELU": "elu", "EXP": "exp"}


def _torch_unary(op, ctx, x):
    F = torch.nn.functional
    if op == "RELU":
        return torch.relu(x)
    if op == "SIGMOID":
        return torch.sigmoid(x)
    if op == "TANH":
        return torch.tanh(x)
    if op == "GELU":
        return F.gelu(x, approximate="tanh" if ctx.a("approximate", "tanh") == "tanh" else "none")
    if op == "ELU":
        return F.elu(x, alpha=float(ctx.a("alpha", 1.0)))
    if op == "LEAKYRELU":
        return F.leaky_relu(x, float(ctx.a("alpha", 0.01)))
    if op == "EXP":
        return torch.exp(x)
    if op == "LOG":
        return torch.log(x)
    if op == "SQRT":
        return torch.sqrt(x)
    if op == "RSQRT":
        return torch.rsqrt(x)
    if op == "SIN":
        return torch.sin(x)
    if op == "COS":
        return torch.cos(x)
    if op == "POW":
        return torch.pow(x, float(ctx.a("exponent")))
    if op == "CEIL":
        return torch.ceil(x)
    if op == "ROUND":
        return torch.round(x)
    if op == "LOGICAL_NOT":
        return torch.logical_not(x)
    if op in ("IDENTITY", "NOOP"):
        return x.clone() if torch.is_grad_enabled() else x
    s = float(ctx.a("scalar", 0.0))
    if op == "SCALAR_MULTIPLY":
        return x * s
    if op == "SCALAR_ADD":
        return x + s
    if op == "SCALAR_SUB":
        return x - s
    if op == "SCALAR_TRUE_DIV":
        return x / s
    if op == "SCALAR_FLOOR_DIV":
        return torch.floor_divide(x, s)
    raise NotImplementedError(op)


_INPLACE_ACT = {"RELU": torch.relu_, "SIGMOID": torch.sigmoid_, "TANH": torch.tanh_, "EXP": torch.exp_}


def _act_grad_from_output(op, y, dy):
    yf = y.float()
    if op == "RELU":
        d = (yf > 0).float()
    elif op == "SIGMOID":
        d = yf * (1 - yf)
    elif op == "TANH":
        d = 1 - yf * yf
    else:  # EXP
        d = yf
    return (dy.float() * d).to(dy.dtype)


@register("RELU", "SIGMOID", "TANH", "GELU", "ELU", "EXP")
class ActivationOp(OpImpl):
    def forward(self, ctx, inputs, weights):
        x = inputs[0]
        if ctx.extra.get("inplace_ok") and ctx.op_type in _INPLACE_ACT:
            # --enable-inplace-optimizations: the output overwrites the input,
            # the backward runs from the output
            with torch.no_grad():
                y = _INPLACE_ACT[ctx.op_type](x)
            return [y], ("out", y)
        if (x.is_cuda and x.dtype in (torch.bfloat16, torch.float32) and x.numel() % 8 == 0
                and x.is_contiguous() and K.available()
                and not (ctx.op_type == "GELU" and ctx.a("approximate", "tanh") != "tanh")):
            y, _ = K.bias_act_fwd(x.view(-1, x.shape[-1] if x.shape[-1] % 8 == 0 else 8), None,
                                  _HIP_ACTS[ctx.op_type], float(ctx.a("alpha", 1.0)))
            return [y.view(x.shape)], ("hip", x)
        with torch.no_grad():
            y = _torch_unary(ctx.op_type, ctx, x)
        return [y], ("torch", x)

    def backward(self, ctx, saved, grad_outputs, weight_grads, need_input_grad):
        kind, x = saved
        dy = grad_outputs[0]
        if kind == "out":
            return [_act_grad_from_output(ctx.op_type, x, dy)]
        if kind == "hip" and dy.is_contiguous():
            return [K.act_bwd(dy, x, _HIP_ACTS[ctx.op_type], float(ctx.a("alpha", 1.0)))]
        xf = x.detach().float().requires_grad_(True)
        with torch.enable_grad():
            y = _torch_unary(ctx.op_type, ctx, xf)
        y.backward(dy.float())
        return [xf.grad.to(dy.dtype)]


@register("LEAKYRELU", "LOG", "SQRT", "RSQRT", "SIN", "COS", "POW", "CEIL", "ROUND", "LOGICAL_NOT", "IDENTITY",
          "NOOP", "SCALAR_MULTIPLY", "SCALAR_ADD", "SCALAR_SUB", "SCALAR_TRUE_DIV", "SCALAR_FLOOR_DIV")
class UnaryOp(AutogradOp):
    """Scalar / math unary ops: HIP unary kernel on GPU (tensorops.hip),
    autograd recompute elsewhere (CPU, LOGICAL_NOT, FLOOR_DIV)."""

    @staticmethod
    def _scalar(ctx):
        op = ctx.op_type
        if op == "POW":
            return float(ctx.a("exponent"))
        if op == "LEAKYRELU":
            return float(ctx.a("alpha", 0.01))
        return float(ctx.a("scalar", 0.0))

    def compute(self, ctx, inputs, weights):
        return [_torch_unary(ctx.op_type, ctx, inputs[0])]

    _INPLACE = {"SCALAR_MULTIPLY": torch.Tensor.mul_, "SCALAR_ADD": torch.Tensor.add_,
                "SCALAR_SUB": torch.Tensor.sub_, "SCALAR_TRUE_DIV": torch.Tensor.div_}

    def forward(self, ctx, inputs, weights):
        x = inputs[0]
        if ctx.extra.get("inplace_ok") and ctx.op_type in self._INPLACE:
            s = self._scalar(ctx)
            with torch.no_grad():
                y = self._INPLACE[ctx.op_type](x, s)
            return [y], ("inplace", s)
        if ctx.op_type in K.UNARY_CODES and K.tensorop_ok(x):
            s = self._scalar(ctx)
            return [K.unary(x, ctx.op_type, s)], ("hip", x, s)
        return super().forward(ctx, inputs, weights)

    def backward(self, ctx, saved, grad_outputs, weight_grads, need_input_grad):
        if saved[0] == "inplace":
            s, g = saved[1], grad_outputs[0]
            if not need_input_grad[0]:
                return [None]
            if ctx.op_type == "SCALAR_MULTIPLY":
                return [g * s]
            return [g / s if ctx.op_type == "SCALAR_TRUE_DIV" else g]
        if saved[0] == "hip":
            _, x, s = saved
            g = grad_outputs[0]
            return [K.unary(x, ctx.op_type, s, dy=g.contiguous().to(x.dtype)) if need_input_grad[0] else None]
        return super().backward(ctx, saved, grad_outputs, weight_grads, need_input_grad)


def _unbroadcast(g, shape):
    while g.dim() > len(shape):
        g = g.sum(0)
    for i, s in enumerate(shape):
        if s == 1 and g.shape[i] != 1:
            g = g.sum(i, keepdim=True)
    return g


@register("EW_ADD", "EW_SUB", "EW_MUL", "EW_DIV", "EW_MAX", "EW_MIN", "EW_EQUAL", "EW_GREATER", "EW_LESS")
class BinaryOp(OpImpl):
    def forward(self, ctx, inputs, weights):
        a, b = inputs
        op = ctx.op_type
        if op in K.BINARY_CODES and a.dtype == b.dtype and K.tensorop_ok(a, b) and a.dim() <= 6 and b.dim() <= 6:
            y = K.binary(a, b, op)
            keep = (a, b) if op in ("EW_MUL", "EW_DIV", "EW_MAX", "EW_MIN") else (None, None)
            return [y], ("hip", keep, tuple(a.shape), tuple(b.shape))
        with torch.no_grad():
            if op == "EW_ADD":
                y = a + b
            elif op == "EW_SUB":
                y = a - b
            elif op == "EW_MUL":
                y = a * b
            elif op == "EW_DIV":
                y = a / b
            elif op == "EW_MAX":
                y = torch.maximum(a, b)
            elif op == "EW_MIN":
                y = torch.minimum(a, b)
            elif op == "EW_EQUAL":
                y = a == b
            elif op == "EW_GREATER":
                y = a > b
            else:
                y = a < b
        keep = (a, b) if op in ("EW_MUL", "EW_DIV", "EW_MAX", "EW_MIN") else (None, None)
        return [y], (keep, a.shape, b.shape)

    def backward(self, ctx, saved, grad_outputs, weight_grads, need_input_grad):
        if saved[0] == "hip":
            _, (a, b), sa, sb = saved
            g = grad_outputs[0].contiguous()
            if a is not None and g.dtype != a.dtype:
                g = g.to(a.dtype)
            return [K.binary_grad(g, a, b, ctx.op_type, 0, sa, sb) if need_input_grad[0] else None,
                    K.binary_grad(g, a, b, ctx.op_type, 1, sa, sb) if need_input_grad[1] else None]
        (a, b), sa, sb = saved
        g = grad_outputs[0]
        op = ctx.op_type
        if op == "EW_ADD":
            ga, gb = g, g
        elif op == "EW_SUB":
            ga, gb = g, -g
        elif op == "EW_MUL":
            ga, gb = g * b, g * a
        elif op == "EW_DIV":
            ga, gb = g / b, -g * a / (b * b)
        elif op in ("EW_MAX", "EW_MIN"):
            m = (a >= b) if op == "EW_MAX" else (a <= b)
            ga, gb = g * m, g * (~m)
        else:
            return [None, None]
        ra = _unbroadcast(ga, sa).reshape(sa) if need_input_grad[0] else None
        rb = _unbroadcast(gb, sb).reshape(sb) if need_input_grad[1] else None
        return [ra, rb]


@register("DROPOUT")
class DropoutOp(OpImpl):
    def forward(self, ctx, inputs, weights):
        x = inputs[0]
        p = float(ctx.a("rate", 0.5))
        if not ctx.training or p <= 0.0:
            return [x], None
        seed = (int(ctx.a("seed", 0)) * 1000003 + ctx.seed * 7919 + ctx.step * 104729) & ((1 << 63) - 1)
        if x.is_cuda and x.is_contiguous() and x.numel() % 8 == 0 and K.available():
            return [K.dropout(x, p, seed)], ("hip", seed, p)
        gen = torch.Generator(device=x.device).manual_seed(seed)
        mask = (torch.rand(x.shape, generator=gen, device=x.device) >= p).to(x.dtype) / (1.0 - p)
        return [x * mask], ("torch", mask, p)

    def backward(self, ctx, saved, grad_outputs, weight_grads, need_input_grad):
        g = grad_outputs[0]
        if saved is None:
            return [g]
        if saved[0] == "hip":
            # the mask is a pure function of (seed, index): regenerate it
            return [K.dropout(g.contiguous(), saved[2], saved[1])]
        return [g * saved[1]]


@register("CAST")
class CastOp(AutogradOp):
    _MAP = {"float": torch.float32, "double": torch.float64, "half": torch.float16, "bfloat16": torch.bfloat16,
            "int32": torch.int32, "int64": torch.int64, "bool": torch.bool}

    def compute(self, ctx, inputs, weights):
        return [inputs[0].to(self._MAP[ctx.a("dtype")])]


@register("SOFTMAX")
class SoftmaxOp(OpImpl):
    def forward(self, ctx, inputs, weights):
        x = inputs[0]
        dim = int(ctx.a("dim", -1)) % x.dim()
        if (x.is_cuda and dim == x.dim() - 1 and x.is_contiguous() and x.dtype in (torch.bfloat16, torch.float32)
                and K.available()):
            y = K.softmax_fwd(x.view(-1, x.shape[-1])).view(x.shape)
        else:
            y = torch.softmax(x.float(), dim).to(x.dtype)
        return [y], (y, dim)

    def backward(self, ctx, saved, grad_outputs, weight_grads, need_input_grad):
        y, dim = saved
        g = grad_outputs[0]
        if ctx.extra.get("identity_backward"):
            # the reference's softmax backward (softmax_kernels.cu:63-72): a copy
            return [g.clone()]
        if g.is_cuda and dim == y.dim() - 1 and g.is_contiguous() and K.available():
            return [K.softmax_bwd(g.view(-1, g.shape[-1]), y.view(-1, y.shape[-1])).view(g.shape)]
        yf = y.float()
        gf = g.float()
        return [(yf * (gf - (gf * yf).sum(dim, keepdim=True))).to(g.dtype)]
