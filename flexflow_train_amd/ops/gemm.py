"""GEMM dispatch: hand-written MFMA GEMM (fused epilogues) vs hipBLASLt.

The MFMA kernel (csrc/kernels/gemm.hip) fuses bias / activation /
pre-activation store / fp32-accumulate epilogues; hipBLASLt (through
torch.mm / addmm) is the plain library GEMM.  ``FF_GEMM`` selects:

* ``auto`` (default): time both once per (shape, layout, epilogue) signature
  outside graph capture and keep the faster — "measure, don't guess";
* ``hip``: always the MFMA kernel; ``blas``: always hipBLASLt.

On CPU everything is a torch matmul in the compute dtype.
"""
from __future__ import annotations

import os
from typing import Dict, Optional, Tuple

import torch

from .. import kernels as K

_MODE = os.environ.get("FF_GEMM", "auto")
_CHOICE: Dict[Tuple, str] = {}
_ACT = {
    "none": lambda t: t,
    "relu": torch.relu,
    "sigmoid": torch.sigmoid,
    "tanh": torch.tanh,
    "gelu": lambda t: torch.nn.functional.gelu(t, approximate="tanh"),
}


def set_mode(mode: str):
    global _MODE
    assert mode in ("auto", "hip", "blas")
    _MODE = mode
    _CHOICE.clear()


def choices() -> Dict[Tuple, str]:
    return dict(_CHOICE)


def _hip_ok(a, b, trans_a, trans_b) -> bool:
    if a.dtype != torch.bfloat16 or b.dtype != torch.bfloat16 or not K.available():
        return False
    M, Kd = (a.shape[1], a.shape[0]) if trans_a else a.shape
    N = b.shape[0] if trans_b else b.shape[1]
    if a.stride(0) % 8 or b.stride(0) % 8:
        return False
    if (not trans_a and Kd % 8) or (trans_a and M % 8) or (not trans_b and N % 8) or (trans_b and Kd % 8):
        return False
    return a.data_ptr() % 16 == 0 and b.data_ptr() % 16 == 0


def _blas(a, b, trans_a, trans_b, bias, act, out, beta, pre):
    A = a.t() if trans_a else a
    B = b.t() if trans_b else b
    if not A.is_cuda:
        r = A.float() @ B.float() if (out is not None and out.dtype == torch.float32) else A @ B
        if bias is not None:
            r = r + bias.to(r.dtype)
        if pre is not None:
            pre.copy_(r)
        r = _ACT[act](r)
        if out is not None:
            if beta:
                out.mul_(beta).add_(r.to(out.dtype))
            else:
                out.copy_(r)
            return out
        return r
    if out is not None and out.dtype == torch.float32:
        if not beta and bias is None and act == "none" and pre is None:
            return torch.mm(A, B, out_dtype=torch.float32, out=out)   # weight grads: written in place
        r = torch.mm(A, B, out_dtype=torch.float32)
        if bias is not None:
            r += bias.float()
        if pre is not None:
            pre.copy_(r)
        r = _ACT[act](r)
        if beta:
            out.mul_(beta).add_(r)
        else:
            out.copy_(r)
        return out
    if act != "none":
        # hipBLASLt GEMM (+ bias epilogue) writes the pre-activation directly,
        # the activation runs in the HIP element-wise kernel (16 B / lane).
        u = pre if pre is not None else torch.empty(A.shape[0], B.shape[1], device=A.device, dtype=A.dtype)
        if bias is not None:
            torch.addmm(bias, A, B, out=u)
        else:
            torch.mm(A, B, out=u)
        y, _ = K.bias_act_fwd(u, None, act)
        if out is not None:
            out.copy_(y)
            return out
        return y
    if out is not None:
        if not beta and bias is None and out.dtype == A.dtype:
            return torch.mm(A, B, out=out)                           # written in place (e.g. bf16 dW)
        if beta == 1.0 and bias is None and out.dtype == A.dtype:
            return out.addmm_(A, B)                                  # in-place gradient accumulation
        r = torch.addmm(bias, A, B) if bias is not None else A @ B
        if beta:
            out.mul_(beta).add_(r)
        else:
            out.copy_(r)
        return out
    if bias is not None:
        return torch.addmm(bias, A, B)
    return A @ B


def _hip(a, b, trans_a, trans_b, bias, act, out, beta, pre):
    return K.gemm(a, b, trans_a=trans_a, trans_b=trans_b, bias=bias, act=act, beta=beta, out=out, pre=pre)


def _time(fn, iters=3) -> float:
    fn()
    s = torch.cuda.Event(enable_timing=True)
    e = torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters


def matmul(a: torch.Tensor, b: torch.Tensor, trans_a=False, trans_b=False, bias: Optional[torch.Tensor] = None,
           act: str = "none", out: Optional[torch.Tensor] = None, beta: float = 0.0,
           pre: Optional[torch.Tensor] = None) -> torch.Tensor:
    """C = act(op(a) @ op(b) + bias) (+ beta * out).  2-D operands."""
    if not a.is_cuda:
        return _blas(a, b, trans_a, trans_b, bias, act, out, beta, pre)
    hip_ok = _hip_ok(a, b, trans_a, trans_b) and (out is None or out.stride(1) == 1)
    if not hip_ok or _MODE == "blas":
        return _blas(a, b, trans_a, trans_b, bias, act, out, beta, pre)
    if _MODE == "hip":
        return _hip(a, b, trans_a, trans_b, bias, act, out, beta, pre)
    key = (tuple(a.shape), tuple(b.shape), trans_a, trans_b, bias is not None, act,
           None if out is None else out.dtype, bool(beta), pre is not None)
    choice = _CHOICE.get(key)
    if choice is None:
        if torch.cuda.is_current_stream_capturing():
            choice = "hip"
        else:
            scratch = None if out is None else out.clone()
            pscratch = None if pre is None else pre.clone()
            t_hip = _time(lambda: _hip(a, b, trans_a, trans_b, bias, act, scratch, beta, pscratch))
            t_blas = _time(lambda: _blas(a, b, trans_a, trans_b, bias, act, scratch, beta, pscratch))
            choice = "hip" if t_hip <= t_blas else "blas"
        _CHOICE[key] = choice
    if choice == "hip":
        return _hip(a, b, trans_a, trans_b, bias, act, out, beta, pre)
    return _blas(a, b, trans_a, trans_b, bias, act, out, beta, pre)
