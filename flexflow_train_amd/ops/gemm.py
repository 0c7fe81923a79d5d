"""GEMM dispatch: hand-written MFMA GEMM (fused epilogues) vs hipBLASLt.

The MFMA kernel (csrc/kernels/gemm.hip) fuses bias / activation /
pre-activation store / fp32-accumulate epilogues; hipBLASLt (through
torch.mm / addmm) is the plain library GEMM.  ``FF_GEMM`` selects:

* ``auto`` (default): time every candidate once per (shape, layout,
  epilogue) signature outside graph capture and keep the fastest — "measure,
  don't guess".  Candidates: hipBLASLt through torch.mm (its heuristic's first
  pick), hipBLASLt called directly with each of its top ``FF_GEMM_LT_ALGOS``
  (default 4) heuristic candidates (``lt:i``, csrc/kernels/blaslt.hip, bias
  in the library epilogue), the 128² register-staged MFMA kernel, the
  256² LDS-DMA kernel (csrc/kernels/gemm256.hip) and the phase-pipelined
  persistent 256² kernel (``p:s``, csrc/kernels/gemmp.hip, fused bias /
  activation / pre-activation epilogue) and the one-wave-per-SIMD 128x128
  wave-tile kernel (``t:s``, csrc/kernels/gemmt.hip, same epilogues; ``u:s``
  is the same kernel with B staged by LDS-DMA, ``w:s`` with both) and, for
  products whose 256x256 tiles cannot fill the chip, the 64x64-tile MLP
  kernel (``s:s``, csrc/kernels/gemms.hip, same epilogues) at several
  split-K degrees (the long-K weight-gradient GEMMs are where split-K
  and gemmt win); the 256² LDS-DMA kernel only with FF_GEMM256=1;
* ``hip``: always the MFMA kernel; ``blas``: always hipBLASLt.

On CPU everything is a torch matmul in the compute dtype.
"""
from __future__ import annotations

import os
from typing import Any, Callable, Dict, List, Optional, Tuple

import torch

from .. import kernels as K

_MODE = os.environ.get("FF_GEMM", "auto")
_CHOICE: Dict[Tuple, str] = {}
_TIMES: Dict[Tuple, Dict[str, float]] = {}   # autotuner measurements (ms), for reports
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


def report() -> str:
    """One line per tuned GEMM signature: shape, transposes, epilogue, the
    candidates' times (ms) and the pick."""
    lines = []
    for key, ch in _CHOICE.items():
        (ash, bsh, ta, tb, bias, act, odt, beta, pre) = key[:9]
        t = _TIMES.get(key, {})
        best = sorted(t.items(), key=lambda kv: kv[1])[:4]
        lines.append(f"a{list(ash)} b{list(bsh)} ta={int(ta)} tb={int(tb)} bias={int(bias)} act={act} "
                     f"out={str(odt).replace('torch.', '')} beta={int(beta)} pre={int(pre)} -> {ch}  "
                     + " ".join(f"{k}:{v:.3f}" for k, v in best))
    return "\n".join(lines)


def _hip_ok(a, b, trans_a, trans_b) -> bool:
    if a.dtype != torch.bfloat16 or b.dtype != torch.bfloat16 or not K.available():
        return False
    M, Kd = (a.shape[1], a.shape[0]) if trans_a else a.shape
    N = b.shape[0] if trans_b else b.shape[1]
    if a.stride(0) % 8 or b.stride(0) % 8:
        return False
    if (not trans_a and Kd % 8) or (trans_a and M % 8) or (not trans_b and N % 8) or (trans_b and Kd % 8):
        return False
    if N % 4:  # the output rows are written in 8 / 16-byte pieces
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
        if u.shape[-1] % 8 == 0:
            y, _ = K.bias_act_fwd(u, None, act)
        else:  # narrow heads (e.g. DLRM's 1-wide output) miss the 16-byte vector path
            y = _ACT[act](u)
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


def _f32(a, b, trans_a, trans_b, bias, act, out, beta, pre):
    """fp32 operands: the exact-fp32 MFMA kernel (csrc/kernels/igemm32.hip),
    the counterpart of the reference's fp32 cublasGemmEx
    (linear_kernels.cu:124-131).  No library GEMM on this path."""
    a = a if a.stride(1) == 1 else a.contiguous()
    b = b if b.stride(1) == 1 else b.contiguous()
    if bias is not None and bias.dtype != torch.float32:
        bias = bias.float()
    if bias is not None:
        bias = bias.contiguous()
    if out is not None and out.stride(1) != 1:
        r = K.gemm_f32(a, b, trans_a, trans_b, bias=bias, act=act)
        if beta:
            out.mul_(beta).add_(r.to(out.dtype))
        else:
            out.copy_(r)
        return out
    if pre is not None and pre.dtype != (out.dtype if out is not None else torch.float32):
        p32 = torch.empty(pre.shape, device=pre.device, dtype=torch.float32)
        r = K.gemm_f32(a, b, trans_a, trans_b, bias=bias, act=act, alpha=1.0, beta=beta, out=out, pre=p32)
        pre.copy_(p32)
        return r
    return K.gemm_f32(a, b, trans_a, trans_b, bias=bias, act=act, beta=beta, out=out, pre=pre)


def _hip(a, b, trans_a, trans_b, bias, act, out, beta, pre, splits=1):
    return K.gemm(a, b, trans_a=trans_a, trans_b=trans_b, bias=bias, act=act, beta=beta, out=out, pre=pre,
                  splits=splits)


def _hip_splits(M: int, N: int, Kd: int) -> List[int]:
    """Split-K degrees for the 128x128-tile kernel when its grid leaves most
    of the 256 CUs idle (small-batch MLPs: a 1024x1024 output is 64 tiles):
    the degrees that bring the grid to about one or two workgroups per CU,
    keeping >= 2 K-tiles of 64 per split."""
    tiles = ((M + 127) // 128) * ((N + 127) // 128)
    if tiles >= 192 or N % 4:
        return []
    return sorted({s for s in (2, 4, 8, 16) if s * tiles <= 640 and Kd // 64 >= 2 * s})


def _hip256(a, b, trans_a, trans_b, bias, act, out, beta, pre, splits=1):
    return K.gemm256(a, b, trans_a=trans_a, trans_b=trans_b, bias=bias, act=act, beta=beta, out=out, pre=pre,
                     splits=splits)


def _gp(a, b, trans_a, trans_b, bias, act, out, beta, pre, splits=1):
    return K.gemmp(a, b, trans_a=trans_a, trans_b=trans_b, bias=bias, act=act, beta=beta, out=out, pre=pre,
                   splits=splits)


# gemmp.hip family variants of the one-wave-per-SIMD kernel (gemmt.hip): 3 =
# both operands staged through registers ("t:" candidates), 4 = B by LDS-DMA
# ("u:", 4-8 % faster on most forward / input-gradient shapes), 6 = both by
# LDS-DMA ("w:": forward GEMMs at hipBLASLt parity, weight gradients 7-10 %
# past register staging; profiles/gemm_ab_gemmt_dma_r3.jsonl,
# gemm_ab_gemmt_dma2_r3.jsonl, gemm_ab_gemmt_dma2_dw_r3.jsonl); 0 disables all
# three
_GT_VARIANT = int(os.environ.get("FF_GEMMT_VARIANT", "3"))
_GT_DMA = _GT_VARIANT != 0 and os.environ.get("FF_GEMMT_DMA", "1") != "0"
_GT_RS = _GT_VARIANT != 0 and os.environ.get("FF_GEMMT_RS", "1") != "0"
_GT_PERS = _GT_VARIANT != 0 and os.environ.get("FF_GEMMT_PERS", "1") != "0"


def _gt(a, b, trans_a, trans_b, bias, act, out, beta, pre, splits=1, variant=None):
    return K.gemmp(a, b, trans_a=trans_a, trans_b=trans_b, bias=bias, act=act, beta=beta, out=out, pre=pre,
                   splits=splits, variant=_GT_VARIANT if variant is None else variant)


def _gs(a, b, trans_a, trans_b, bias, act, out, beta, pre, splits=1):
    """64x64-tile MLP GEMM (csrc/kernels/gemms.hip, gemmp variant 8)."""
    return K.gemmp(a, b, trans_a=trans_a, trans_b=trans_b, bias=bias, act=act, beta=beta, out=out, pre=pre,
                   splits=splits, variant=8)


def _gs_splits(M: int, N: int, Kd: int) -> List[int]:
    """Split-K degrees that bring a 64x64-tile grid to about one or two
    workgroups per CU (plain epilogue only; >= 2 K-tiles per split)."""
    tiles = ((M + 63) // 64) * ((N + 63) // 64)
    return sorted({s for s in (2, 4, 8, 16) if tiles * s <= 640 and Kd // 64 >= 2 * s})


def _small_mn(M: int, N: int) -> bool:
    """Products whose 256x256 tiles cannot fill the chip (DLRM's MLPs)."""
    return ((M + 255) // 256) * ((N + 255) // 256) < 64


def _gt_ok(bias, act, out, beta, pre) -> bool:
    """gemmt instantiates the activation epilogues for none / relu / gelu."""
    return _gp_ok(bias, act, out, beta, pre) and act in ("none", "relu", "gelu")


def _gp_ok(bias, act, out, beta, pre) -> bool:
    """Epilogues gemmp implements: plain (alpha/beta, bf16 or fp32 out) or
    bias/activation/pre-activation into a fresh bf16 output."""
    if bias is None and act == "none" and pre is None:
        return True
    return not beta and (out is None or out.dtype == torch.bfloat16) and act in ("none", "relu", "sigmoid", "tanh",
                                                                                   "gelu")


def _lt(a, b, trans_a, trans_b, bias, act, out, beta, pre, algo=0):
    """hipBLASLt called directly with the ``algo``-th heuristic candidate
    (torch.mm always takes the first); bias in the GEMM epilogue, the
    activation in the HIP element-wise kernel."""
    M = a.shape[1] if trans_a else a.shape[0]
    N = b.shape[0] if trans_b else b.shape[1]
    if act != "none":
        u = pre if pre is not None else torch.empty(M, N, device=a.device, dtype=torch.bfloat16)
        K.blaslt_matmul(a, b, trans_a, trans_b, u, 0.0, bias, algo)
        y = K.bias_act_fwd(u, None, act)[0] if N % 8 == 0 else _ACT[act](u)
        if out is not None:
            out.copy_(y)
            return out
        return y
    if out is None:
        out = torch.empty(M, N, device=a.device, dtype=torch.bfloat16)
        beta = 0.0
    return K.blaslt_matmul(a, b, trans_a, trans_b, out, beta, bias, algo)


_LT_MAX = 0 if os.environ.get("FF_LIBRARY_GEMM", "1") == "0" else int(os.environ.get("FF_GEMM_LT_ALGOS", "4"))


def _lt_candidates(a, b, trans_a, trans_b, bias, act, out, beta, pre):
    if _LT_MAX <= 0 or not hasattr(K.ext(), "blaslt_num_algos"):
        return {}
    if bias is not None and (bias.dtype != torch.bfloat16 or (out is not None and out.dtype != torch.bfloat16)):
        return {}
    if act != "none" and out is not None and out.dtype != torch.bfloat16:
        return {}
    target = pre if act != "none" else out
    n = K.blaslt_num_algos(a, b, trans_a, trans_b, target, beta if act == "none" else 0.0, bias is not None)
    return {f"lt:{i}": (lambda i_: (lambda *args: _lt(*args, algo=i_)))(i) for i in range(min(n, _LT_MAX))}


def _candidates(a, b, trans_a, trans_b, bias, act, pre, out=None, beta=0.0):
    """name -> callable(a, b, ta, tb, bias, act, out, beta, pre) tried by the autotuner."""
    c = {"hip": _hip} if _LIB_OFF else {"hip": _hip, "blas": _blas}
    M_, Kd_ = (a.shape[1], a.shape[0]) if trans_a else (a.shape[0], a.shape[1])
    N_ = b.shape[0] if trans_b else b.shape[1]
    for s in _hip_splits(M_, N_, Kd_):
        c[f"hip:{s}"] = (lambda s_: (lambda *args: _hip(*args, splits=s_)))(s)
    c.update(_lt_candidates(a, b, trans_a, trans_b, bias, act, out, beta, pre))
    if os.environ.get("FF_GEMM256", "0") != "0" and K.gemm256_supported(a, b, trans_a, trans_b):
        M, Kd = (a.shape[1], a.shape[0]) if trans_a else (a.shape[0], a.shape[1])
        N = b.shape[0] if trans_b else b.shape[1]
        plain = bias is None and act == "none" and pre is None
        splits = {1}
        if plain:
            d = K.default_splits(M, N, Kd)
            splits |= {s for s in (d // 2, d, d * 2) if 1 <= s <= max(1, Kd // 512)}
        for s in sorted(splits):
            c[f"hip256:{s}"] = (lambda s_: (lambda *args: _hip256(*args, splits=s_)))(s)
    if os.environ.get("FF_GEMMP", "1") != "0" and K.gemmp_supported(a, b, trans_a, trans_b) and _gp_ok(
            bias, act, out, beta, pre):
        M, Kd = (a.shape[1], a.shape[0]) if trans_a else (a.shape[0], a.shape[1])
        N = b.shape[0] if trans_b else b.shape[1]
        splits, tsplits = {1}, {1}
        tiles = ((M + 255) // 256) * ((N + 255) // 256)
        # split-K only where the output tiles leave CUs idle: past two waves of
        # workgroups a split only adds its fp32 partial slab (GPT-3's logits
        # GEMM at split 2: 13 GB of partials for nothing)
        if bias is None and act == "none" and pre is None and tiles < 512:
            # powers of two around the grid-filling degree (gemmp: K-tiles must
            # split evenly); gemmt also takes uneven splits, so it adds the
            # degrees that fill one or two waves of workgroups exactly
            d = K.default_splits(M, N, Kd)
            pow2 = {s for s in (2, 4, 8, 16, 32) if d / 3 <= s <= 2 * d and s <= max(1, Kd // 512)}
            splits |= {s for s in pow2 if (Kd // 64) % s == 0}
            tsplits |= pow2 | {s for s in (round(256 / tiles), round(512 / tiles)) if 2 <= s <= max(1, Kd // 512)}
        if trans_b and not trans_a and bias is None and act == "none" and pre is None \
                and os.environ.get("FF_GEMMN", "1") != "0":
            c["n:1"] = lambda *args: _gt(*args, splits=1, variant=9)
        if trans_b and not trans_a and act == "none" and pre is None and Kd // 64 >= 2 \
                and (out is None or out.dtype == torch.bfloat16) and os.environ.get("FF_GEMMPP", "1") != "0":
            # eight-wave ping-pong A B^T kernel (gemmpp.hip, variant 11): plain,
            # accumulate (beta) and bias epilogues
            c["y:1"] = lambda *args: _gt(*args, splits=1, variant=11)
        if _small_mn(M, N) and os.environ.get("FF_GEMMS", "1") != "0":
            c["s:1"] = _gs
            if bias is None and act == "none" and pre is None:
                for s in _gs_splits(M, N, Kd):
                    c[f"s:{s}"] = (lambda s_: (lambda *args: _gs(*args, splits=s_)))(s)
        for s in sorted(splits):
            c[f"p:{s}"] = (lambda s_: (lambda *args: _gp(*args, splits=s_)))(s)
        for s in sorted(tsplits):
            if _GT_VARIANT and _gt_ok(bias, act, out, beta, pre):
                c[f"t:{s}"] = (lambda s_: (lambda *args: _gt(*args, splits=s_)))(s)
                if _GT_DMA:
                    c[f"u:{s}"] = (lambda s_: (lambda *args: _gt(*args, splits=s_, variant=4)))(s)
                    c[f"w:{s}"] = (lambda s_: (lambda *args: _gt(*args, splits=s_, variant=6)))(s)
                if _GT_PERS and (Kd // 64) % s == 0 and Kd // 64 // s >= 2:
                    # persistent form (variant 5): one workgroup per CU walks its
                    # tiles, the next tile's loads in flight under this tile's
                    # epilogue -- for the epilogue-heavy K = 1024 forwards
                    c[f"v:{s}"] = (lambda s_: (lambda *args: _gt(*args, splits=s_, variant=5)))(s)
                if _GT_RS and not (trans_a and trans_b):
                    # the padded-image kernel with register staging (variant 10):
                    # 1-11 % ahead of "w" on the weight-gradient and long-K
                    # input-gradient shapes, behind it on the K = 1024 forwards
                    # (profiles/r5/ab_gemmt_kk_rs_r5.txt) -- timed, not assumed
                    c[f"x:{s}"] = (lambda s_: (lambda *args: _gt(*args, splits=s_, variant=10)))(s)
    return c


_TRACE = os.environ.get("FF_AUTOTUNE_TRACE", "0") == "1"
_SLEEP_PER_MS: Dict[int, float] = {}   # device -> torch.cuda._sleep cycles per millisecond


def _gpu_busy(ms: float):
    """Enqueue ~``ms`` of device-side busy wait on the current stream, so the
    host can queue the calls being timed behind it and the device then runs
    them back to back (no host launch gaps inside the timed interval)."""
    dev = torch.cuda.current_device()
    rate = _SLEEP_PER_MS.get(dev)
    if rate is None:
        cyc = 1_000_000
        torch.cuda._sleep(cyc)   # first call: module load
        s = torch.cuda.Event(enable_timing=True)
        e = torch.cuda.Event(enable_timing=True)
        s.record()
        torch.cuda._sleep(cyc)
        e.record()
        e.synchronize()
        rate = _SLEEP_PER_MS[dev] = cyc / max(1e-3, s.elapsed_time(e))
    torch.cuda._sleep(max(1, int(ms * rate)))


def _time_queued(fn, iters: int, rounds: int = 2) -> float:
    """Mean device time per call of ``fn``: ``iters`` calls queued behind a
    device busy-wait and bracketed by events.  Eager back-to-back calls of a
    10-20 us GEMM time the host launch path (pybind + Python), which the
    training step -- itself one hipGraph -- never pays; this clock sees only
    the kernels, without capturing anything.  It replaces round 3's clock
    that replayed each candidate from a captured hipGraph: one such replay
    (torch's in-place hipBLASLt accumulate, captured inside the smoke step's
    backward) never completed, while the same capture / replay outside a
    training step completes (docs/PERF.md 'Autotuner clock').  If the host
    needed longer to queue the calls than the busy-wait lasted, the round is
    repeated with a longer wait."""
    import time as _time_mod
    fn()
    best = float("inf")
    busy = 1.0
    r = 0
    while r < rounds:
        s = torch.cuda.Event(enable_timing=True)
        e = torch.cuda.Event(enable_timing=True)
        _gpu_busy(busy)
        t0 = _time_mod.perf_counter()
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        host_ms = (_time_mod.perf_counter() - t0) * 1e3
        e.synchronize()
        if host_ms > 0.8 * busy and busy < 64:
            busy = max(2 * busy, 2 * host_ms)   # the queue may have drained: redo this round
            continue
        best = min(best, s.elapsed_time(e) / iters)
        r += 1
    return best


def _time_all(fns: Dict[str, Callable[[], Any]], iters=5) -> Dict[str, float]:
    """Time every candidate the same way: eagerly, and when the fastest one
    is under ~50 us per call (where eager back-to-back issue is launch-bound)
    all of them again with the queued clock (``_time_queued``) -- one clock
    for the comparison."""
    times = {name: _time(fn, iters=iters) for name, fn in fns.items()}
    if times and min(times.values()) < 0.05 and not torch.cuda.is_current_stream_capturing():
        out = {}
        for name, fn in fns.items():
            if _TRACE:
                import sys
                print(f"[autotune] queued clock: {name}", file=sys.stderr, flush=True)
            out[name] = _time_queued(fn, max(iters, 10))
        times = out
    return times


def _time(fn, iters=5, rounds=2) -> float:
    """min over rounds of the mean time of ``iters`` back-to-back calls."""
    fn()
    best = float("inf")
    for _ in range(rounds):
        s = torch.cuda.Event(enable_timing=True)
        e = torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        e.synchronize()
        best = min(best, s.elapsed_time(e) / iters)
    return best


# a library GEMM (hipBLASLt / torch.mm) is taken only when it beats the
# fastest hand-written candidate by more than this fraction AND by more than
# _LIB_MIN_MS per call: within timing noise, and on the microsecond GEMMs of
# small MLPs, the MFMA kernel runs (FF_GEMM_LIB_MARGIN / FF_GEMM_LIB_MIN_MS;
# 0 / 0 = the fastest outright)
_LIB_MARGIN = float(os.environ.get("FF_GEMM_LIB_MARGIN", "0.03"))
# FF_LIBRARY_GEMM=0: hand-written kernels only -- rocBLAS / hipBLASLt are
# neither timed nor picked wherever a native candidate takes the shape
_LIB_OFF = os.environ.get("FF_LIBRARY_GEMM", "1") == "0"
if _LIB_OFF:
    _LIB_MARGIN = 1.0
_LIB_MIN_MS = float(os.environ.get("FF_GEMM_LIB_MIN_MS", "0.004"))


def _is_library(name: str) -> bool:
    return name == "blas" or name.startswith("lt:")


def _pick_fastest(times: Dict[str, float]) -> str:
    best = min(times, key=times.get)
    if not _is_library(best):
        return best
    native = {k: v for k, v in times.items() if not _is_library(k)}
    if native:
        nb = min(native, key=native.get)
        if times[best] >= native[nb] * (1.0 - _LIB_MARGIN) or native[nb] - times[best] < _LIB_MIN_MS:
            return nb
    return best


def matmul(a: torch.Tensor, b: torch.Tensor, trans_a=False, trans_b=False, bias: Optional[torch.Tensor] = None,
           act: str = "none", out: Optional[torch.Tensor] = None, beta: float = 0.0,
           pre: Optional[torch.Tensor] = None, native_only: bool = False) -> torch.Tensor:
    """C = act(op(a) @ op(b) + bias) (+ beta * out).  2-D operands.
    ``native_only``: hand-written kernels only (no library candidate)."""
    if not a.is_cuda:
        return _blas(a, b, trans_a, trans_b, bias, act, out, beta, pre)
    if a.dtype == torch.float32 and b.dtype == torch.float32 and K.use_hip(a, b):
        return _f32(a, b, trans_a, trans_b, bias, act, out, beta, pre)
    hip_ok = _hip_ok(a, b, trans_a, trans_b) and (
        out is None or (out.stride(1) == 1 and out.stride(0) % 4 == 0 and out.data_ptr() % 8 == 0))
    if not hip_ok or _MODE == "blas":
        return _blas(a, b, trans_a, trans_b, bias, act, out, beta, pre)
    if _MODE == "hip":
        return _hip(a, b, trans_a, trans_b, bias, act, out, beta, pre)
    # leading dims and pointer alignment are part of the signature: the
    # hipBLASLt plans behind ``lt:i`` are keyed by them and gemm256 checks them
    key = (tuple(a.shape), tuple(b.shape), trans_a, trans_b, bias is not None, act,
           None if out is None else out.dtype, bool(beta), pre is not None,
           a.stride(0), b.stride(0), None if out is None else out.stride(0),
           _align(a), _align(b), None if out is None else _align(out), bool(native_only))
    choice = _CHOICE.get(key)
    if choice is None:
        if torch.cuda.is_current_stream_capturing():
            # no library queries / timing inside a capture (hipBLASLt's
            # heuristic may allocate): the MFMA kernel, decided on the host
            choice = "hip"
        else:
            cands = _candidates(a, b, trans_a, trans_b, bias, act, pre, out, beta)
            if native_only:
                cands = {k: v for k, v in cands.items() if not _is_library(k)}
            scratch = None if out is None else out.clone()
            pscratch = None if pre is None else pre.clone()
            times = _time_all({name: (lambda fn=fn: fn(a, b, trans_a, trans_b, bias, act, scratch, beta, pscratch))
                               for name, fn in cands.items()})
            choice = _pick_fastest(times)
            _TIMES[key] = times
        _CHOICE[key] = choice
    if choice.startswith("hip256") and not K.gemm256_supported(a, b, trans_a, trans_b):
        choice = "hip"
    if choice[:2] in ("p:", "t:", "u:", "v:", "w:", "x:", "s:", "n:") and not K.gemmp_supported(a, b, trans_a, trans_b):
        choice = "hip"
    return _resolve(choice)(a, b, trans_a, trans_b, bias, act, out, beta, pre)


def sync_choices() -> int:
    """Make every rank use the same kernel for the same GEMM signature.

    Each rank times its candidates on its own, and near-ties can then fall
    differently on different ranks.  Replicas that must stay bitwise equal
    without a gradient sync (the bias gradients of partial-sum replicas,
    ops/dense.py) would then drift.  Every rank's decisions are all-gathered,
    and for each signature the lowest rank that tuned it decides.  This is a
    collective: all ranks call it, outside graph capture.  Returns the number
    of decisions this rank changed."""
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return 0
    from .dense import _DACT_CHOICE   # fused-vs-plain activation-gradient decisions
    tables = (_CHOICE, _DACT_CHOICE)
    objs: List[Any] = [None] * dist.get_world_size()
    dist.all_gather_object(objs, [dict(t) for t in tables])
    changed = 0
    for i, table in enumerate(tables):
        merged: Dict[Tuple, Any] = {}
        for d in objs:          # rank order: the lowest rank that tuned a signature wins
            for k, v in ((d or [{}] * len(tables))[i]).items():
                merged.setdefault(k, v)
        changed += sum(1 for k, v in merged.items() if table.get(k, v) != v)
        table.update(merged)
    return changed


def _align(t: torch.Tensor) -> int:
    p = t.data_ptr()
    return 16 if p % 16 == 0 else (8 if p % 8 == 0 else 2)


def _resolve(name: str):
    if name == "hip":
        return _hip
    if name == "blas":
        return _blas
    kind, _, arg = name.partition(":")
    if kind == "hip":
        return lambda *args: _hip(*args, splits=int(arg))
    if kind == "lt":
        return lambda *args: _lt(*args, algo=int(arg))
    if kind == "p":
        return lambda *args: _gp(*args, splits=int(arg))
    if kind == "t":
        return lambda *args: _gt(*args, splits=int(arg))
    if kind == "u":
        return lambda *args: _gt(*args, splits=int(arg), variant=4)
    if kind == "w":
        return lambda *args: _gt(*args, splits=int(arg), variant=6)
    if kind == "x":
        return lambda *args: _gt(*args, splits=int(arg), variant=10)
    if kind == "v":
        return lambda *args: _gt(*args, splits=int(arg), variant=5)
    if kind == "s":
        return lambda *args: _gs(*args, splits=int(arg))
    if kind == "n":
        return lambda *args: _gt(*args, splits=1, variant=9)
    if kind == "y":
        return lambda *args: _gt(*args, splits=1, variant=11)
    return lambda *args: _hip256(*args, splits=int(arg))


def wgrad_matmul(ctx, a: torch.Tensor, b: torch.Tensor, out: torch.Tensor, beta: float):
    """Weight gradient ``out = a^T b (+ beta * out)``.  When the executor
    attached its weight-gradient stream (``ctx.extra["wgrad_stream"]`` =
    (stream, keep-list, storage pointers)), the GEMM is queued there after the
    compute stream's work so far, and runs beside the rest of the backward
    pass; ``a`` / ``b`` stay referenced until the executor joins the stream."""
    wg = ctx.extra.get("wgrad_stream")
    if wg is None or not a.is_cuda:
        return matmul(a, b, trans_a=True, out=out, beta=beta)
    stream, keep, ptrs = wg
    stream.wait_stream(torch.cuda.current_stream(a.device))
    with torch.cuda.stream(stream):
        r = matmul(a, b, trans_a=True, out=out, beta=beta)
    for t in (a, b):
        keep.append(t)
        ptrs.add(t.untyped_storage().data_ptr())
    return r
