"""Host wrappers for the gfx950 HIP kernel library (``_ffkernels``).

Every wrapper validates device / dtype / contiguity / shape on the host before
launching (a bad launch on the GPU pool can reset the node, so nothing is
launched with shapes the kernel does not support), then passes raw pointers
and the current HIP stream.  Launches are asynchronous and capturable into
hipGraphs.

``STATS`` counts kernel launches per name so tests can assert that the native
path (not a PyTorch fallback) ran.
"""
from __future__ import annotations

import collections
import importlib
import math
import os
from typing import Dict, Optional

import torch

_ext = None
_ext_error: Optional[BaseException] = None
STATS: collections.Counter = collections.Counter()

DT_F32, DT_BF16, DT_F16 = 0, 1, 2
ACT_CODES = {"none": 0, "identity": 0, "relu": 1, "sigmoid": 2, "tanh": 3, "gelu": 4, "elu": 5, "exp": 6}


def _load():
    global _ext, _ext_error
    if _ext is not None or _ext_error is not None:
        return _ext
    try:
        # torch must be imported first so the extension binds to the HIP
        # runtime torch already loaded (same SONAME libamdhip64.so.7).
        _ext = importlib.import_module("flexflow_train_amd._ffkernels")
    except BaseException as e:  # pragma: no cover - depends on build state
        _ext_error = e
    return _ext


def available() -> bool:
    return _load() is not None


def ext():
    m = _load()
    if m is None:
        raise RuntimeError(
            "flexflow_train_amd._ffkernels is not built/loadable "
            f"({_ext_error!r}); run `python tools/build_native.py kernels`")
    return m


def use_hip(*tensors: torch.Tensor) -> bool:
    """True when the tensors live on a GPU, in which case the HIP kernels are
    mandatory (a missing extension raises instead of silently falling back)."""
    if not tensors or not all(t.is_cuda for t in tensors if t is not None):
        return False
    ext()
    return True


def _dt(t: torch.Tensor) -> int:
    if t.dtype == torch.float32:
        return DT_F32
    if t.dtype == torch.bfloat16:
        return DT_BF16
    raise TypeError(f"unsupported dtype {t.dtype} for HIP kernels")


def _p(t: Optional[torch.Tensor]) -> int:
    return 0 if t is None else t.data_ptr()


def _stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def _check(t: torch.Tensor, name: str, dtype=None, numel=None, aligned: bool = True):
    if not t.is_cuda:
        raise ValueError(f"{name}: expected a GPU tensor")
    if not t.is_contiguous():
        raise ValueError(f"{name}: expected a contiguous tensor")
    if dtype is not None and t.dtype != dtype:
        raise ValueError(f"{name}: expected {dtype}, got {t.dtype}")
    if numel is not None and t.numel() != numel:
        raise ValueError(f"{name}: expected {numel} elements, got {t.numel()}")
    if aligned and t.data_ptr() % 16:
        raise ValueError(f"{name}: data pointer must be 16-byte aligned")


# ---------------------------------------------------------------------------
def layernorm_fwd(x, gamma, beta, eps, residual=None, save_sum=True):
    """y = LN(x [+ residual]); returns (y, sum_or_x, mean, rstd)."""
    N = x.shape[-1]
    M = x.numel() // N
    _check(x, "x")
    if N % 8:
        raise ValueError("layernorm: last dim must be a multiple of 8")
    y = torch.empty_like(x)
    s = None
    if residual is not None:
        _check(residual, "residual", x.dtype, x.numel())
        s = torch.empty_like(x) if save_sum else None
    for name, w in (("gamma", gamma), ("beta", beta)):
        if w is not None:
            _check(w, name, x.dtype, N)
    mean = torch.empty(M, device=x.device, dtype=torch.float32)
    rstd = torch.empty(M, device=x.device, dtype=torch.float32)
    ext().layernorm_fwd(_dt(x), _p(x), _p(residual), _p(s), _p(gamma), _p(beta), _p(y), _p(mean), _p(rstd),
                        M, N, float(eps), _stream())
    STATS["layernorm_fwd"] += 1
    return y, (s if residual is not None else x), mean, rstd


def layernorm_bwd(dy, s, mean, rstd, gamma, dgamma=None, dbeta=None, dres=None, dsum=None):
    """dx = LN'(dy) [+ dres]; dgamma/dbeta/dsum (fp32) accumulate the column
    sums of dy*xhat, dy and the final dx (dsum: the producing Linear's bias
    gradient, fused here instead of a separate pass)."""
    N = dy.shape[-1]
    M = dy.numel() // N
    _check(dy, "dy")
    _check(s, "s", dy.dtype, dy.numel())
    if dres is not None:
        _check(dres, "dres", dy.dtype, dy.numel())
    dx = torch.empty_like(dy)
    for name, w in (("dgamma", dgamma), ("dbeta", dbeta), ("dsum", dsum)):
        if w is not None:
            _check(w, name, torch.float32, N)
    grid = ext().layernorm_bwd_grid(M, N)
    ws = None
    if grid and (dgamma is not None or dbeta is not None or dsum is not None):
        ws = torch.empty(3 * grid * N, device=dy.device, dtype=torch.float32)
    ext().layernorm_bwd(_dt(dy), _p(dy), _p(s), _p(mean), _p(rstd), _p(gamma), _p(dx), _p(dgamma), _p(dbeta),
                        _p(ws), M, N, _stream(), _p(dres), _p(dsum))
    STATS["layernorm_bwd"] += 1
    return dx


def bias_act_fwd(x, bias, act: str, alpha: float = 1.0, save_pre: bool = True):
    N = x.shape[-1]
    M = x.numel() // N
    _check(x, "x")
    if N % 8:
        raise ValueError("bias_act: last dim must be a multiple of 8")
    if bias is not None:
        _check(bias, "bias", x.dtype, N)
    y = torch.empty_like(x)
    pre = torch.empty_like(x) if (bias is not None and save_pre) else None
    ext().bias_act_fwd(_dt(x), _p(x), _p(bias), _p(pre), _p(y), M, N, ACT_CODES[act], float(alpha), _stream())
    STATS["bias_act_fwd"] += 1
    return y, (pre if pre is not None else x)


def act_bwd(dy, pre, act: str, alpha: float = 1.0):
    _check(dy, "dy")
    _check(pre, "pre", dy.dtype, dy.numel())
    if dy.numel() % 8:
        raise ValueError("act_bwd: numel must be a multiple of 8")
    dx = torch.empty_like(dy)
    ext().act_bwd(_dt(dy), _p(dy), _p(pre), _p(dx), dy.numel(), ACT_CODES[act], float(alpha), _stream())
    STATS["act_bwd"] += 1
    return dx


def colsum_act(dy, pre=None, act: str = "none", dbias=None, write_dx: bool = True, alpha: float = 1.0):
    """g = dy * act'(pre); dbias += colsum(g) (fp32); returns g (or None)."""
    N = dy.shape[-1]
    M = dy.numel() // N
    _check(dy, "dy")
    if N % 8:
        raise ValueError("colsum: last dim must be a multiple of 8")
    if pre is not None:
        _check(pre, "pre", dy.dtype, dy.numel())
    if dbias is not None:
        _check(dbias, "dbias", torch.float32, N)
    dx = torch.empty_like(dy) if write_dx else None
    ext().colsum_act(_dt(dy), _p(dy), _p(pre), _p(dx), _p(dbias), M, N, ACT_CODES[act], float(alpha), _stream())
    STATS["colsum_act"] += 1
    return dx


def dropout(x, p: float, seed: int):
    _check(x, "x")
    if x.numel() % 8:
        raise ValueError("dropout: numel must be a multiple of 8")
    y = torch.empty_like(x)
    ext().dropout_fwd(_dt(x), _p(x), _p(y), x.numel(), float(p), int(seed) & ((1 << 64) - 1), _stream())
    STATS["dropout"] += 1
    return y


def cast_(src, dst):
    _check(src, "src")
    _check(dst, "dst", numel=src.numel())
    if src.numel() % 8:
        raise ValueError("cast: numel must be a multiple of 8")
    ext().cast(_dt(src), _dt(dst), _p(src), _p(dst), src.numel(), _stream())
    STATS["cast"] += 1
    return dst


def softmax_ce(logits, labels, grad_scale: float, metrics=None, valid_cols: Optional[int] = None,
               ignore_index: int = -100, write_grad: bool = True, row_loss=None):
    """Fused softmax + sparse CE; overwrites logits with the gradient."""
    V = logits.shape[-1]
    M = logits.numel() // V
    _check(logits, "logits")
    if not labels.is_cuda or not labels.is_contiguous() or labels.numel() != M:
        raise ValueError("softmax_ce: labels must be a contiguous GPU tensor with one label per row")
    if labels.dtype not in (torch.int32, torch.int64):
        raise ValueError("softmax_ce: labels must be int32/int64")
    if metrics is not None:
        _check(metrics, "metrics", torch.float32)
        if metrics.numel() < 3:
            raise ValueError("softmax_ce: metrics buffer needs 3 floats")
    if row_loss is not None:
        _check(row_loss, "row_loss", torch.float32, M)
    vv = V if valid_cols is None else int(valid_cols)
    # per-row metric terms reduced by one block (no same-address atomics);
    # a stream-ordered temporary, so it is also valid inside a hipGraph capture
    row_stats = None if metrics is None else torch.empty(M * 3, device=logits.device, dtype=torch.float32)
    ext().softmax_ce(_dt(logits), 64 if labels.dtype == torch.int64 else 32, _p(logits), _p(labels), _p(row_loss),
                     _p(metrics), _p(row_stats), M, V, vv, float(grad_scale), int(ignore_index), int(write_grad),
                     _stream())
    STATS["softmax_ce"] += 1
    return logits


def softmax_fwd(x):
    N = x.shape[-1]
    _check(x, "x")
    y = torch.empty_like(x)
    ext().softmax_fwd(_dt(x), _p(x), _p(y), x.numel() // N, N, _stream())
    STATS["softmax_fwd"] += 1
    return y


def softmax_bwd(dy, y):
    N = dy.shape[-1]
    _check(dy, "dy")
    _check(y, "y", dy.dtype, dy.numel())
    dx = torch.empty_like(dy)
    ext().softmax_bwd(_dt(dy), _p(dy), _p(y), _p(dx), dy.numel() // N, N, _stream())
    STATS["softmax_bwd"] += 1
    return dx


def adam_step(w, g, m, v, w_bf16, lr, beta1, beta2, eps, weight_decay, step, grad_scale=1.0, decoupled=False,
              hp=None):
    """Fused Adam/AdamW over a flat buffer; g may be fp32 or bf16.  ``hp``: optional
    device float32 tensor {lr, step} read by the kernel (hipGraph replay)."""
    if hp is not None:
        _check(hp, "hp", torch.float32, 2)
    n = w.numel()
    for name, t in (("w", w), ("m", m), ("v", v)):
        _check(t, name, torch.float32, n)
    _check(g, "g", numel=n)
    if w_bf16 is not None:
        _check(w_bf16, "w_bf16", torch.bfloat16, n)
    if n % 4:
        raise ValueError("adam: flat buffer length must be a multiple of 4")
    ext().adam_step(_p(w), _p(g), _dt(g), _p(m), _p(v), _p(w_bf16), n, float(lr), float(beta1), float(beta2),
                    float(eps), float(weight_decay), int(step), float(grad_scale), int(decoupled), _p(hp), _stream())
    STATS["adam_step"] += 1


def sgd_step(w, g, mom, w_bf16, lr, momentum, weight_decay, nesterov, grad_scale=1.0):
    n = w.numel()
    _check(w, "w", torch.float32, n)
    _check(g, "g", numel=n)
    if mom is not None:
        _check(mom, "mom", torch.float32, n)
    if w_bf16 is not None:
        _check(w_bf16, "w_bf16", torch.bfloat16, n)
    if n % 4:
        raise ValueError("sgd: flat buffer length must be a multiple of 4")
    ext().sgd_step(_p(w), _p(g), _dt(g), _p(mom), _p(w_bf16), n, float(lr), float(momentum), float(weight_decay),
                   int(bool(nesterov)), float(grad_scale), _stream())
    STATS["sgd_step"] += 1


def sparse_sgd_rows(tables, step: float) -> bool:
    """Row-sparse SGD over embedding tables, two launches for all of them
    (csrc/kernels/optimizer.hip sparse_sgd_kernel).  ``tables``: list of
    (master [rows, dim] fp32, grad [rows, dim] fp32|bf16, compute [rows, dim]
    bf16 or None, idx 1-D int32|int64).  master[r] -= step * grad[r];
    compute[r] = bf16(master[r]); grad[r] = 0 for every looked-up row r
    (clamped into range).  Returns False (nothing launched) when a table does
    not meet the kernel's layout: the caller then takes the framework path."""
    if not tables or len(tables) > 16:
        return False
    desc, off = [], 0
    for m, g, c, idx in tables:
        rows, dim = m.shape
        ok = (m.dtype == torch.float32 and m.is_contiguous() and g.shape == m.shape and g.is_contiguous()
              and g.dtype in (torch.float32, torch.bfloat16) and dim % 4 == 0 and idx.dim() == 1
              and idx.dtype in (torch.int32, torch.int64) and idx.is_contiguous() and idx.is_cuda
              and m.data_ptr() % 16 == 0 and g.data_ptr() % (16 if g.dtype == torch.float32 else 8) == 0
              and (c is None or (c.dtype == torch.bfloat16 and c.shape == m.shape and c.is_contiguous()
                                 and c.data_ptr() % 8 == 0)))
        if not ok:
            return False
        desc.append((m.data_ptr(), g.data_ptr(), int(g.dtype == torch.bfloat16), 0 if c is None else c.data_ptr(),
                     idx.data_ptr(), int(idx.dtype == torch.int64), idx.numel(), rows, dim, off))
        off += idx.numel() * dim
    scratch = torch.empty(max(off, 4), dtype=torch.float32, device=tables[0][0].device)
    ext().sparse_sgd_rows(desc, _p(scratch), float(step), _stream())
    STATS["sparse_sgd"] += 1
    return True


def sum_squares(x, out):
    _check(x, "x", torch.float32)
    _check(out, "out", torch.float32)
    if x.numel() % 4:
        raise ValueError("sum_squares: length must be a multiple of 4")
    ext().sum_squares(_p(x), x.numel(), _p(out), _stream())
    STATS["sum_squares"] += 1


_AGGR = {"none": 0, "sum": 1, "avg": 2}


def embedding_fwd(idx, weight, aggr: str = "none"):
    """idx [..., L] -> out [..., L, D] (none) or [..., D] (sum/avg)."""
    _check(weight, "weight")
    if not idx.is_cuda or not idx.is_contiguous() or idx.dtype not in (torch.int32, torch.int64):
        raise ValueError("embedding: indices must be a contiguous int32/int64 GPU tensor")
    n, D = weight.shape
    if D % 8:
        raise ValueError("embedding: dim must be a multiple of 8")
    if aggr == "none":
        B, L = idx.numel(), 1
        out = torch.empty(*idx.shape, D, device=weight.device, dtype=weight.dtype)
    else:
        L = idx.shape[-1]
        B = idx.numel() // max(L, 1)
        out = torch.empty(*idx.shape[:-1], D, device=weight.device, dtype=weight.dtype)
    ext().embedding_fwd(_dt(weight), 64 if idx.dtype == torch.int64 else 32, _p(idx), _p(weight), _p(out), B, L, D,
                        _AGGR[aggr], n, _stream())
    STATS["embedding_fwd"] += 1
    return out


def embedding_bwd(idx, dout, dweight, aggr: str = "none"):
    _check(dweight, "dweight", torch.float32)
    _check(dout, "dout")
    n, D = dweight.shape
    if aggr == "none":
        B, L = idx.numel(), 1
    else:
        L = idx.shape[-1]
        B = idx.numel() // max(L, 1)
    if dout.numel() != B * D:
        raise ValueError("embedding_bwd: dout shape mismatch")
    # privatised accumulation copies for hot (small) tables: aim for <= ~8
    # contributions per (copy, row) and a workspace of at most 64 MiB
    rows = B * L
    copies = 1
    # tables of <= 8 rows without bags take the register-accumulating kernel
    # (embedding.hip embed_bwd_small_kernel): no replicas
    small = n <= 8 and aggr == "none" and os.environ.get("FFK_EMB_SMALL", "1") != "0"
    if rows > 8 * n and not small:
        copies = int(min(256, rows // (8 * n), max(1, (64 << 20) // max(1, n * D * 4))))
    ws = torch.zeros(copies * n * D, device=dweight.device, dtype=torch.float32) if copies > 1 else None
    ext().embedding_bwd(_dt(dout), 64 if idx.dtype == torch.int64 else 32, _p(idx), _p(dout), _p(dweight), B, L, D,
                        _AGGR[aggr], n, _p(ws), copies, _stream())
    STATS["embedding_bwd"] += 1


def _view4(t: torch.Tensor):
    """[B, S, H, D] view (d contiguous) -> (ptr, sb, ss, sh)."""
    if t.dim() != 4 or t.stride(3) != 1:
        raise ValueError("attention tensors must be 4-D [B, S, H, D] with contiguous D")
    if t.dtype != torch.bfloat16 or not t.is_cuda:
        raise ValueError("attention kernels take bf16 GPU tensors")
    if t.data_ptr() % 16 or any(s % 8 for s in t.stride()[:3]):
        raise ValueError("attention tensors must be 16-byte aligned with strides multiple of 8")
    return (t.data_ptr(), t.stride(0), t.stride(1), t.stride(2))


def attention_fwd(q, k, v, causal=False, scale=None, out=None):
    """Flash attention forward.  q,k,v: [B, S, H, D] bf16 views (any b/s/h
    strides, e.g. slices of a packed [B, S, 3, H, D] QKV buffer).
    Returns (o [B, Sq, H, D] contiguous, lse [B, H, Sq] fp32 log2-domain)."""
    B, Sq, H, D = q.shape
    Sk = k.shape[1]
    if D not in (64, 128):
        raise ValueError("attention: head dim must be 64 or 128")
    if k.shape != (B, Sk, H, D) or v.shape != (B, Sk, H, D):
        raise ValueError("attention: q/k/v shape mismatch")
    if out is None:
        out = torch.empty(B, Sq, H, D, device=q.device, dtype=q.dtype)
    lse = torch.empty(B, H, Sq, device=q.device, dtype=torch.float32)
    sc = float(scale) if scale is not None else 1.0 / math.sqrt(D)
    ext().attention_fwd(_view4(q), _view4(k), _view4(v), _view4(out), lse.data_ptr(), B, H, Sq, Sk, D, sc,
                        bool(causal), _stream())
    STATS["attention_fwd"] += 1
    return out, lse


def attention_bwd(q, k, v, o, lse, do, dq, dk, dv, causal=False, scale=None, dbias=None, dbias_atomic=False):
    """Flash-attention backward into dq / dk / dv.  ``dbias`` = optional
    (dbq, dbk, dbv) fp32 [H*D] projection-bias gradients, accumulated with the
    column sums of dq / dk / dv (over batch and sequence) computed in the
    kernels' epilogues: by default each wave stores its 32-row partial into a
    slab that one reduction then adds (no atomics); ``dbias_atomic`` uses
    per-column fp32 atomics instead (round 2's form, 2x slower kernels)."""
    B, Sq, H, D = q.shape
    Sk = k.shape[1]
    for name, t, shp in (("o", o, (B, Sq, H, D)), ("do", do, (B, Sq, H, D)), ("dq", dq, (B, Sq, H, D)),
                         ("dk", dk, (B, Sk, H, D)), ("dv", dv, (B, Sk, H, D))):
        if tuple(t.shape) != shp:
            raise ValueError(f"attention_bwd: {name} has shape {tuple(t.shape)}, expected {shp}")
    if lse.shape != (B, H, Sq) or lse.dtype != torch.float32 or not lse.is_contiguous():
        raise ValueError("attention_bwd: bad lse")
    delta = torch.empty(B, H, Sq, device=q.device, dtype=torch.float32)
    sc = float(scale) if scale is not None else 1.0 / math.sqrt(D)
    dbs, ld, slab = [0, 0, 0], 0, None
    HD = H * D
    if dbias is not None:
        for t in dbias:
            if t is not None:
                _check(t, "dbias", torch.float32, HD)
        if dbias_atomic:
            dbs = [t.data_ptr() if t is not None else 0 for t in dbias]
        else:
            nq, nk = (Sq + 31) // 32, (Sk + 31) // 32
            slab = torch.empty(B * max(nq, nk), 3 * HD, device=q.device, dtype=torch.float32)
            ld = 3 * HD
            dbs = [slab.data_ptr() + 4 * i * HD if t is not None else 0 for i, t in enumerate(dbias)]
    ext().attention_bwd(_view4(q), _view4(k), _view4(v), _view4(o), _view4(do), _view4(dq), _view4(dk), _view4(dv),
                        lse.data_ptr(), delta.data_ptr(), B, H, Sq, Sk, D, sc, bool(causal), _stream(), *dbs, ld)
    if slab is not None:
        # every (row block, column) of the slab was written once; rows past a
        # tensor's own row-block count (Sq != Sk) are not part of its sum
        rows = (B * nq, B * nk, B * nk)
        for i, t in enumerate(dbias):
            if t is not None:
                t.add_(slab[:rows[i], i * HD:(i + 1) * HD].sum(0))
    STATS["attention_bwd"] += 1


def gemm(a, b, trans_a=False, trans_b=False, bias=None, act="none", alpha=1.0, beta=0.0, out=None,
         out_dtype=None, pre=None, splits=1):
    """C = act(alpha * op(a) @ op(b) + bias) + beta * C with the MFMA GEMM.

    a: [M, K] (or [K, M] if trans_a), b: [K, N] (or [N, K] if trans_b), bf16.
    ``splits`` > 1: split-K into an fp32 workspace, then one epilogue pass
    (GEMMs whose 128x128 tiles cannot fill the chip, e.g. DLRM's MLPs).
    """
    if a.dtype != torch.bfloat16 or b.dtype != torch.bfloat16:
        raise ValueError("gemm: operands must be bf16")
    if a.dim() != 2 or b.dim() != 2 or a.stride(1) != 1 or b.stride(1) != 1:
        raise ValueError("gemm: operands must be 2-D with unit inner stride")
    M, K = (a.shape[1], a.shape[0]) if trans_a else (a.shape[0], a.shape[1])
    Kb, N = (b.shape[1], b.shape[0]) if trans_b else (b.shape[0], b.shape[1])
    if K != Kb:
        raise ValueError(f"gemm: inner dims differ ({K} vs {Kb})")
    dt = out_dtype or (out.dtype if out is not None else torch.bfloat16)
    if out is None:
        out = torch.empty(M, N, device=a.device, dtype=dt)
    if out.shape != (M, N) or out.stride(1) != 1:
        raise ValueError("gemm: bad output")
    if bias is not None:
        _check(bias, "bias", torch.bfloat16, N)
    if pre is not None:
        _check(pre, "pre", torch.bfloat16, M * N)
    splits = max(1, min(int(splits), (K + 63) // 64))
    if splits > 1 and (N % 4 or out.stride(0) % 4):
        splits = 1
    ws = _splitk_ws(a.device, splits * M * N) if splits > 1 else None
    ext().gemm(a.data_ptr(), b.data_ptr(), out.data_ptr(), _p(bias), _p(pre), M, N, K, a.stride(0), b.stride(0),
               out.stride(0), bool(trans_a), bool(trans_b), ACT_CODES[act], float(alpha), float(beta),
               int(out.dtype == torch.float32), _stream(), splits, _p(ws))
    STATS["gemm"] += 1
    if splits > 1:
        STATS["gemm_splitk"] += 1
    return out


_WS_CACHE: dict = {}


def _splitk_ws(dev, numel: int) -> torch.Tensor:
    """fp32 split-K partial slab, one per (device, stream, size): dW GEMMs on
    the weight-gradient side stream may run beside same-sized compute-stream
    GEMMs, which must not share a slab."""
    key = (dev, torch.cuda.current_stream(dev).cuda_stream, numel)
    ws = _WS_CACHE.get(key)
    if ws is None:
        ws = torch.empty(numel, device=dev, dtype=torch.float32)
        _WS_CACHE[key] = ws
    return ws


_GRAPH_CAPTURED = [False]


def note_graph_capture():
    """A hipGraph now holds workspace pointers: the cache is never trimmed
    again in this process."""
    _GRAPH_CAPTURED[0] = True


def trim_workspaces():
    """Drop the cached split-K slabs (the autotuner's candidates leave one per
    split degree they tried); kernels in use re-create theirs on their next
    call.  Only between steps, and never once a captured graph may read them."""
    if not _GRAPH_CAPTURED[0]:
        _WS_CACHE.clear()


def gemm256_supported(a, b, trans_a=False, trans_b=False) -> bool:
    if a.dtype != torch.bfloat16 or b.dtype != torch.bfloat16 or a.dim() != 2 or b.dim() != 2:
        return False
    if a.stride(1) != 1 or b.stride(1) != 1 or a.data_ptr() % 16 or b.data_ptr() % 16:
        return False
    M, K = (a.shape[1], a.shape[0]) if trans_a else (a.shape[0], a.shape[1])
    N = b.shape[0] if trans_b else b.shape[1]
    return bool(ext().gemm256_supported(M, N, K, a.stride(0), b.stride(0), bool(trans_a), bool(trans_b)))


def default_splits(M: int, N: int, K: int, target_blocks: int = 512) -> int:
    """Split-K degree that brings the grid near ``target_blocks`` (2 per CU)
    while keeping >= 8 K-tiles (512 deep) per split."""
    tiles = ((M + 255) // 256) * ((N + 255) // 256)
    s = max(1, min(target_blocks // max(1, tiles), K // 512, 16))
    return s


def gemm256(a, b, trans_a=False, trans_b=False, bias=None, act="none", alpha=1.0, beta=0.0, out=None,
            out_dtype=None, pre=None, splits=None):
    """256x256-tile MFMA GEMM with LDS-DMA staging and optional split-K
    (split-K: fp32 partial slabs + reduce; no bias/activation epilogue)."""
    if not gemm256_supported(a, b, trans_a, trans_b):
        raise ValueError("gemm256: unsupported operands (bf16, 16-B aligned, K % 64, dims % 8)")
    M, K = (a.shape[1], a.shape[0]) if trans_a else (a.shape[0], a.shape[1])
    Kb, N = (b.shape[1], b.shape[0]) if trans_b else (b.shape[0], b.shape[1])
    if K != Kb:
        raise ValueError(f"gemm256: inner dims differ ({K} vs {Kb})")
    dt = out_dtype or (out.dtype if out is not None else torch.bfloat16)
    if out is None:
        out = torch.empty(M, N, device=a.device, dtype=dt)
    if out.shape != (M, N) or out.stride(1) != 1:
        raise ValueError("gemm256: bad output")
    if bias is not None:
        _check(bias, "bias", torch.bfloat16, N)
    if pre is not None:
        _check(pre, "pre", torch.bfloat16, M * N)
    s = default_splits(M, N, K) if splits is None else int(splits)
    if bias is not None or pre is not None or act != "none":
        s = 1
    ws = None
    if s > 1:
        ws = _splitk_ws(a.device, s * M * N)
    ext().gemm256(a.data_ptr(), b.data_ptr(), out.data_ptr(), _p(bias), _p(pre), M, N, K, a.stride(0), b.stride(0),
                  out.stride(0), bool(trans_a), bool(trans_b), ACT_CODES[act], float(alpha), float(beta),
                  int(out.dtype == torch.float32), s, _p(ws), _stream())
    STATS["gemm256"] += 1
    return out


def gemmp_supported(a, b, trans_a=False, trans_b=False) -> bool:
    if a.dtype != torch.bfloat16 or b.dtype != torch.bfloat16 or a.dim() != 2 or b.dim() != 2:
        return False
    if a.stride(1) != 1 or b.stride(1) != 1 or a.data_ptr() % 16 or b.data_ptr() % 16:
        return False
    if not hasattr(ext(), "gemmp"):
        return False
    M, K = (a.shape[1], a.shape[0]) if trans_a else (a.shape[0], a.shape[1])
    N = b.shape[0] if trans_b else b.shape[1]
    return bool(ext().gemmp_supported(M, N, K, a.stride(0), b.stride(0), bool(trans_a), bool(trans_b)))


def gemmp(a, b, trans_a=False, trans_b=False, bias=None, act="none", alpha=1.0, beta=0.0, out=None,
          out_dtype=None, pre=None, aux=None, act_bwd=False, dbias=None, splits=1, _dbg=0, variant=0):
    """Phase-pipelined 256x256 MFMA GEMM (csrc/kernels/gemmp.hip):
    C = epi(alpha * op(a) op(b)); epi = [+bias] [pre := .] [act(.) or, with
    ``act_bwd``, . * act'(aux)] [dbias += colsum] [+ beta * C].  Split-K
    (``splits`` > 1): fp32 partial slabs + a reduce pass, plain epilogue only.
    ``variant`` 1 runs the same pipeline on 16x16x32 MFMAs (gemmq.hip)."""
    if not gemmp_supported(a, b, trans_a, trans_b):
        raise ValueError("gemmp: unsupported operands (bf16, 16-B aligned, K % 64, dims % 8)")
    M, K = (a.shape[1], a.shape[0]) if trans_a else (a.shape[0], a.shape[1])
    Kb, N = (b.shape[1], b.shape[0]) if trans_b else (b.shape[0], b.shape[1])
    if K != Kb:
        raise ValueError(f"gemmp: inner dims differ ({K} vs {Kb})")
    dt = out_dtype or (out.dtype if out is not None else torch.bfloat16)
    if out is None:
        out = torch.empty(M, N, device=a.device, dtype=dt)
    if out.shape != (M, N) or out.stride(1) != 1:
        raise ValueError("gemmp: bad output")
    for t, nm, n in ((bias, "bias", N), (pre, "pre", M * N), (aux, "aux", M * N)):
        if t is not None:
            _check(t, nm, torch.bfloat16, n)
    if dbias is not None:
        _check(dbias, "dbias", torch.float32, N)
    if act_bwd and (aux is None or act == "none"):
        raise ValueError("gemmp: act_bwd needs aux and an activation")
    s = max(1, int(splits))
    if bias is not None or pre is not None or act != "none" or dbias is not None:
        s = 1
    ws = None
    if s > 1:
        ws = _splitk_ws(a.device, s * M * N)
    ext().gemmp(a.data_ptr(), b.data_ptr(), out.data_ptr(), _p(bias), _p(pre), _p(aux), _p(dbias), M, N, K,
                a.stride(0), b.stride(0), out.stride(0), bool(trans_a), bool(trans_b), ACT_CODES[act], bool(act_bwd),
                float(alpha), float(beta), int(out.dtype == torch.float32), s, _p(ws), _stream(), int(_dbg),
                int(variant))
    STATS["gemmp"] += 1
    return out


def bmm_supported(a, b, trans_a=False, trans_b=False) -> bool:
    """Batched [..., M, K] x [..., K, N] (same batch dims, bf16, 16-B aligned
    rows, K % 64, M / N % 8) on the 64x64-tile kernel (gemms.hip)."""
    if not available() or a.dtype != torch.bfloat16 or b.dtype != torch.bfloat16 or not a.is_cuda:
        return False
    if a.dim() < 3 or a.dim() != b.dim() or a.shape[:-2] != b.shape[:-2] or not hasattr(ext(), "bmm"):
        return False
    if not (a.is_contiguous() and b.is_contiguous()) or a.data_ptr() % 16 or b.data_ptr() % 16:
        return False
    M, K = (a.shape[-1], a.shape[-2]) if trans_a else (a.shape[-2], a.shape[-1])
    N = b.shape[-2] if trans_b else b.shape[-1]
    return K % 64 == 0 and M % 8 == 0 and N % 8 == 0 and a.shape[-1] % 8 == 0 and b.shape[-1] % 8 == 0


def bmm(a, b, trans_a=False, trans_b=False, out=None, beta=0.0):
    """C[z] = op(a[z]) @ op(b[z]) (+ beta C[z]) over the flattened batch dims
    (the reference's batch_matmul_kernels.cu, here one launch: blockIdx.z =
    product)."""
    if not bmm_supported(a, b, trans_a, trans_b):
        raise ValueError("bmm: unsupported operands")
    lead = a.shape[:-2]
    Z = 1
    for d in lead:
        Z *= int(d)
    M, K = (a.shape[-1], a.shape[-2]) if trans_a else (a.shape[-2], a.shape[-1])
    N = b.shape[-2] if trans_b else b.shape[-1]
    if out is None:
        out = torch.empty(*lead, M, N, device=a.device, dtype=torch.bfloat16)
        beta = 0.0
    if not out.is_contiguous() or tuple(out.shape[-2:]) != (M, N):
        raise ValueError("bmm: bad output")
    ext().bmm(a.data_ptr(), b.data_ptr(), out.data_ptr(), Z, M, N, K, a.shape[-1], b.shape[-1], N,
              a.shape[-2] * a.shape[-1], b.shape[-2] * b.shape[-1], M * N, bool(trans_a), bool(trans_b), 1.0,
              float(beta), int(out.dtype == torch.float32), _stream())
    STATS["bmm"] += 1
    return out


# ---------------------------------------------------------------------------
# General tensor operators (csrc/kernels/tensorops.hip).  Inputs: contiguous
# GPU tensors in bf16 or fp32; _check's 16-byte alignment is not required.
def tensorop_ok(*ts) -> bool:
    return available() and all(t is not None and t.is_cuda and t.is_contiguous() and
                               t.dtype in (torch.bfloat16, torch.float32) for t in ts)


def _cstrides(shape):
    st, acc = [0] * len(shape), 1
    for i in range(len(shape) - 1, -1, -1):
        st[i] = acc
        acc *= shape[i]
    return st


def _bcast_strides(shape, out_shape):
    shape = [1] * (len(out_shape) - len(shape)) + list(shape)
    st = _cstrides(shape)
    return [0 if (s == 1 and o != 1) else t for s, o, t in zip(shape, out_shape, st)]


BINARY_CODES = {"EW_ADD": 0, "EW_SUB": 1, "EW_MUL": 2, "EW_DIV": 3, "EW_MAX": 4, "EW_MIN": 5}
CMP_CODES = {"EW_EQUAL": 6, "EW_GREATER": 7, "EW_LESS": 8}   # 0/1 in the operand dtype


def binary(a, b, op: str):
    """Broadcasting element-wise binary op (same dtype)."""
    out_shape = list(torch.broadcast_shapes(a.shape, b.shape))
    y = torch.empty(out_shape, device=a.device, dtype=a.dtype)
    ext().binary_nd(_dt(a), a.data_ptr(), b.data_ptr(), y.data_ptr(), out_shape or [1],
                    _bcast_strides(a.shape, out_shape) or [0], _bcast_strides(b.shape, out_shape) or [0],
                    BINARY_CODES[op] if op in BINARY_CODES else CMP_CODES[op], _stream())
    STATS["binary"] += 1
    return y


def binary_grad(dy, a, b, op: str, which: int, a_shape=None, b_shape=None):
    """Gradient of ``op`` w.r.t. a (0) or b (1), reduced to that operand's
    shape.  For add / sub the operand values are not read: a / b may be None
    (then ``a_shape`` / ``b_shape`` give the shapes)."""
    out_shape = list(dy.shape)
    a_shape = list(a.shape) if a is not None else list(a_shape)
    b_shape = list(b.shape) if b is not None else list(b_shape)
    tgt0 = a_shape if which == 0 else b_shape
    if op in ("EW_ADD", "EW_SUB") and tgt0 == out_shape:   # no broadcast: dy (or -dy) itself
        return dy if (op == "EW_ADD" or which == 0) else unary(dy, "SCALAR_MULTIPLY", -1.0)
    pa = a.data_ptr() if a is not None else dy.data_ptr()
    pb = b.data_ptr() if b is not None else dy.data_ptr()
    g = torch.empty(out_shape, device=dy.device, dtype=torch.float32)
    ext().binary_grad_nd(_dt(dy), dy.data_ptr(), pa, pb, g.data_ptr(), out_shape,
                         _bcast_strides(a_shape, out_shape), _bcast_strides(b_shape, out_shape),
                         BINARY_CODES[op], int(which), _stream())
    STATS["binary_grad"] += 1
    tgt = a_shape if which == 0 else b_shape
    if list(tgt) == out_shape:
        return g.to(dy.dtype)
    padded = [1] * (len(out_shape) - len(tgt)) + list(tgt)
    r = torch.empty(padded, device=dy.device, dtype=dy.dtype)
    ext().sum_to(_dt(r), g.data_ptr(), r.data_ptr(), out_shape, padded, 0.0, _stream())
    return r.reshape(tgt)


def permute(x, perm):
    out_shape = [x.shape[p] for p in perm]
    st = _cstrides(list(x.shape))
    y = torch.empty(out_shape, device=x.device, dtype=x.dtype)
    ext().permute_nd(_dt(x), x.data_ptr(), y.data_ptr(), out_shape, [st[p] for p in perm], _stream())
    STATS["permute"] += 1
    return y


def _oli(shape, axis):
    axis = axis % len(shape)
    outer = 1
    for s in shape[:axis]:
        outer *= s
    inner = 1
    for s in shape[axis + 1:]:
        inner *= s
    return outer, shape[axis], inner, axis


def concat(xs, axis):
    shape = list(xs[0].shape)
    outer, _, inner, axis = _oli(shape, axis)
    total = sum(int(x.shape[axis]) for x in xs)
    shape[axis] = total
    y = torch.empty(shape, device=xs[0].device, dtype=xs[0].dtype)
    off, pieces = 0, []
    for x in xs:
        ln = int(x.shape[axis])
        pieces.append((x.data_ptr(), ln, off))
        off += ln
    for i in range(0, len(pieces), 16):   # one launch per 16 pieces
        ext().slice_copy_multi(_dt(y), y.data_ptr(), pieces[i:i + 16], outer, inner, total, 0, _stream())
    STATS["concat"] += 1
    return y


def split(x, sizes, axis):
    outer, total, inner, axis = _oli(list(x.shape), axis)
    outs, off, pieces = [], 0, []
    for ln in sizes:
        shape = list(x.shape)
        shape[axis] = ln
        y = torch.empty(shape, device=x.device, dtype=x.dtype)
        pieces.append((y.data_ptr(), int(ln), off))
        outs.append(y)
        off += ln
    for i in range(0, len(pieces), 16):
        ext().slice_copy_multi(_dt(x), x.data_ptr(), pieces[i:i + 16], outer, inner, total, 1, _stream())
    STATS["split"] += 1
    return outs


def reverse(x, axis):
    outer, ln, inner, _ = _oli(list(x.shape), axis)
    y = torch.empty_like(x)
    ext().reverse_axis(_dt(x), x.data_ptr(), y.data_ptr(), outer, ln, inner, _stream())
    return y


def gather(x, idx, dim):
    outer, lx, inner, dim = _oli(list(x.shape), dim)
    li = idx.shape[dim]
    y = torch.empty(idx.shape, device=x.device, dtype=x.dtype)
    ext().gather_axis(_dt(x), 64 if idx.dtype == torch.int64 else 32, x.data_ptr(), idx.contiguous().data_ptr(),
                      y.data_ptr(), outer, lx, li, inner, _stream())
    return y


def scatter_add(dy, idx, dim, x_shape):
    outer, lx, inner, dim = _oli(list(x_shape), dim)
    dx = torch.zeros(x_shape, device=dy.device, dtype=torch.float32)
    ext().scatter_add_axis(_dt(dy), 64 if idx.dtype == torch.int64 else 32, dy.data_ptr(),
                           idx.contiguous().data_ptr(), dx.data_ptr(), outer, lx, idx.shape[dim], inner, _stream())
    return dx


REDUCE_CODES = {"sum": 0, "mean": 1, "max": 2, "min": 3, "prod": 4}


def reduce_contig(x, first: int, last: int, op: str):
    """Reduce the contiguous dim range [first, last] of x; returns the
    tensor with those dims removed."""
    shape = list(x.shape)
    outer = 1
    for s in shape[:first]:
        outer *= s
    red = 1
    for s in shape[first:last + 1]:
        red *= s
    inner = 1
    for s in shape[last + 1:]:
        inner *= s
    out = torch.empty(shape[:first] + shape[last + 1:], device=x.device, dtype=x.dtype)
    ext().reduce_axis(_dt(x), x.data_ptr(), out.data_ptr(), outer, red, inner, REDUCE_CODES[op], _stream())
    return out


def topk(x, k: int):
    n = x.shape[-1]
    rows = x.numel() // n
    vals = torch.empty(list(x.shape[:-1]) + [k], device=x.device, dtype=x.dtype)
    idx = torch.empty(list(x.shape[:-1]) + [k], device=x.device, dtype=torch.int64)
    ext().topk_rows(_dt(x), x.data_ptr(), vals.data_ptr(), idx.data_ptr(), rows, n, int(k), _stream())
    return vals, idx


UNARY_CODES = {"SCALAR_ADD": 0, "SCALAR_SUB": 1, "SCALAR_MULTIPLY": 2, "SCALAR_TRUE_DIV": 3, "POW": 4, "LOG": 5,
               "SQRT": 6, "RSQRT": 7, "SIN": 8, "COS": 9, "LEAKYRELU": 10, "CEIL": 11, "ROUND": 12,
               "IDENTITY": 13, "NOOP": 13}


def unary(x, op: str, scalar: float = 0.0, dy=None):
    """Forward (dy None) or backward (returns dy * op'(x)) of a unary / scalar op."""
    y = torch.empty_like(x if dy is None else dy)
    ext().unary_op(_dt(x), x.data_ptr(), _p(dy), y.data_ptr(), x.numel(), UNARY_CODES[op], float(scalar),
                   int(dy is not None), _stream())
    STATS["unary"] += 1
    return y


def mse(pred, label, grad=None, metrics=None, scale: float = 1.0):
    """grad = scale * (pred - label); metrics[0] += sum sq err, metrics[1] += sum abs err."""
    ext().mse_loss(_dt(pred), pred.data_ptr(), label.data_ptr(), _p(grad), _p(metrics), pred.numel(), float(scale),
                   _stream())
    STATS["mse"] += 1
    return grad


def mse_full(pred, label, grad, metrics, scale: float, cols: int, rows: int):
    """grad = scale * (pred - label) and the loss-metrics block updated in the
    same pass (loss += sq err / cols, count += rows, sq / abs error sums);
    ``label`` fp32 or pred's dtype."""
    if label.dtype not in (pred.dtype, torch.float32) or label.numel() != pred.numel():
        raise ValueError("mse: label must match pred (same numel, pred dtype or fp32)")
    _check(metrics, "metrics", torch.float32, None, aligned=False)
    if metrics.numel() < 5:
        raise ValueError("mse: the metrics block needs 5 slots")
    ext().mse_loss_full(_dt(pred), _dt(label), pred.data_ptr(), label.data_ptr(), _p(grad), metrics.data_ptr(),
                        pred.numel(), float(scale), 1, int(cols), int(rows), _stream())
    STATS["mse"] += 1
    return grad


def zero_(t):
    """t.zero_() on the device by the library's own kernel (16-B stores)."""
    if t.numel() == 0:
        return t
    if not t.is_contiguous() or t.data_ptr() % 16:
        return t.zero_()
    ext().zero_fill(t.data_ptr(), t.numel() * t.element_size(), _stream())
    STATS["zero_fill"] += 1
    return t


def narrow_ok(x, w) -> bool:
    """The narrow-Linear kernels' shapes: bf16, N <= 8, K % 8, K * N <= 16384."""
    if not (x.is_cuda and x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and available()):
        return False
    K, N = w.shape
    return (x.dim() == 2 and x.shape[1] == K and 1 <= N <= 8 and K % 8 == 0 and K * N <= 16384 and x.is_contiguous()
            and w.is_contiguous() and x.data_ptr() % 16 == 0)


def narrow_linear_fwd(x, w, bias=None, act: str = "none", pre=None):
    """y = act(x @ w + bias) for a narrow w [K, N <= 8]; ``pre`` (optional,
    [M, N] bf16) receives the pre-activation."""
    if not narrow_ok(x, w):
        raise ValueError("narrow_linear_fwd: unsupported shapes / dtypes")
    M, N = x.shape[0], w.shape[1]
    y = torch.empty(M, N, device=x.device, dtype=x.dtype)
    if bias is not None:
        bias = bias.float().contiguous()
    if pre is not None:
        _check(pre, "pre", x.dtype, M * N, aligned=False)
    ext().narrow_linear_fwd(x.data_ptr(), w.data_ptr(), _p(bias), y.data_ptr(), _p(pre), M, w.shape[0], N,
                            ACT_CODES[act], _stream())
    STATS["narrow_linear"] += 1
    return y


def narrow_linear_bwd(x, w, dy, pre=None, act: str = "none", dw=None, wbeta: float = 0.0, db=None, dx=None,
                      dx_beta: float = 0.0, need_dx: bool = True):
    """Backward of ``narrow_linear_fwd``: g = dy * act'(pre); dw = wbeta dw +
    x^T g (fp32 or bf16), db += colsum(g) (fp32), dx = g w^T (+ dx_beta dx).
    Returns dx (None when not needed)."""
    M, K, N = x.shape[0], w.shape[0], w.shape[1]
    if not narrow_ok(x, w) or dy.shape != (M, N) or dy.dtype != torch.bfloat16 or not dy.is_contiguous():
        raise ValueError("narrow_linear_bwd: unsupported shapes / dtypes")
    if act != "none":
        if pre is None:
            raise ValueError("narrow_linear_bwd: an activation needs the saved pre-activation")
        _check(pre, "pre", torch.bfloat16, M * N, aligned=False)
    if db is not None:
        _check(db, "db", torch.float32, N, aligned=False)
    code = ACT_CODES[act]
    st = _stream()
    if dw is not None or db is not None:
        if dw is not None and (tuple(dw.shape) != (K, N) or not dw.is_contiguous()
                               or dw.dtype not in (torch.float32, torch.bfloat16)):
            raise ValueError("narrow_linear_bwd: dW must be a contiguous [K, N] fp32 / bf16 tensor")
        blocks = int(ext().narrow_wgrad_blocks(M))
        part = torch.empty(blocks * (K + 1) * N, device=x.device, dtype=torch.float32)
        ext().narrow_linear_wgrad(x.data_ptr(), dy.data_ptr(), _p(pre), part.data_ptr(), blocks, _p(dw),
                                  _dt(dw) if dw is not None else 0, float(wbeta), _p(db), M, K, N, code, st)
    if not need_dx:
        return None
    if dx is None:
        dx = torch.empty(M, K, device=x.device, dtype=x.dtype)
        dx_beta = 0.0
    else:
        _check(dx, "dx", torch.bfloat16, M * K)
    ext().narrow_linear_dgrad(dy.data_ptr(), _p(pre), w.data_ptr(), dx.data_ptr(), M, K, N, code, float(dx_beta), st)
    STATS["narrow_linear"] += 1
    return dx


INIT_KINDS = {"uniform": 0, "normal": 1, "truncated_normal": 2, "constant": 3}


def init_piece(out, full_shape, box_lo, kind: str, seed: int, a=0.0, b=1.0, c=-2.0, d=2.0):
    """Fill ``out`` (a box of the logical tensor ``full_shape`` starting at
    ``box_lo``) from a counter-based RNG keyed by (seed, global index)."""
    ext().init_tensor(_dt(out), out.data_ptr(), list(out.shape) or [1], list(full_shape) or [1],
                      list(box_lo) or [0], INIT_KINDS[kind], int(seed) & ((1 << 64) - 1), float(a), float(b),
                      float(c), float(d), _stream())
    STATS["init"] += 1
    return out


# ---------------------------------------------------------------------------
# Convolution / BatchNorm / pooling over NHWC (torch channels_last) bf16
# activations.  Activation tensors keep their logical NCHW shape; the kernels
# read the channels_last storage.  Conv weights are physically [K][R][S][C].
def _check_nhwc(t: torch.Tensor, name: str):
    if not t.is_cuda:
        raise ValueError(f"{name}: expected a GPU tensor")
    if t.dtype != torch.bfloat16:
        raise ValueError(f"{name}: expected bfloat16, got {t.dtype}")
    if t.dim() != 4 or not t.is_contiguous(memory_format=torch.channels_last):
        raise ValueError(f"{name}: expected a 4-d channels_last tensor")
    if t.data_ptr() % 16:
        raise ValueError(f"{name}: data pointer must be 16-byte aligned")


def nhwc(t: torch.Tensor) -> torch.Tensor:
    """channels_last bf16 view/copy of a 4-d activation."""
    return t.contiguous(memory_format=torch.channels_last)


def pad_channels_nhwc(x: torch.Tensor, Cp: int) -> torch.Tensor:
    """Any-stride bf16 [N, C, H, W] -> channels_last [N, Cp, H, W] with the
    channels past C zero, in one pass (conv.hip pad_channels_kernel)."""
    if x.dtype != torch.bfloat16 or not x.is_cuda or x.dim() != 4:
        raise ValueError("pad_channels_nhwc: 4-d bf16 GPU tensor (any strides)")
    N, C, H, W = x.shape
    y = torch.empty((N, Cp, H, W), device=x.device, dtype=x.dtype, memory_format=torch.channels_last)
    sn, sc, sh, sw = x.stride()
    ext().pad_channels_nhwc(_p(x), _p(y), N, C, H, W, sn, sc, sh, sw, Cp, _stream())
    STATS["pad_channels"] += 1
    return y


def conv_out_hw(H, W, R, S, sh, sw, ph, pw, dh=1, dw=1):
    return (H + 2 * ph - dh * (R - 1) - 1) // sh + 1, (W + 2 * pw - dw * (S - 1) - 1) // sw + 1


def _conv_geom(x_shape, K, R, S, stride, pad, dil):
    N, C, H, W = x_shape
    if C % 8 or K % 8:
        raise ValueError("conv2d: input and output channels must be multiples of 8")
    return [int(N), int(H), int(W), int(C), int(K), int(R), int(S), int(stride[0]), int(stride[1]),
            int(pad[0]), int(pad[1]), int(dil[0]), int(dil[1])]


def conv2d_fwd(x, w, bias=None, stride=(1, 1), pad=(0, 0), dil=(1, 1), act: str = "none", stats=None):
    """x [N,C,H,W] channels_last bf16; w [K,R,S,C] contiguous bf16 -> y [N,K,P,Q]
    channels_last.  ``stats`` (fp32 [2,K]) receives the per-channel sum / sumsq of y."""
    _check_nhwc(x, "x")
    K_, R, S, C = w.shape
    _check(w, "w", torch.bfloat16)
    if C != x.shape[1]:
        raise ValueError(f"conv2d: weight has {C} input channels, input has {x.shape[1]}")
    g = _conv_geom(x.shape, K_, R, S, stride, pad, dil)
    P, Q = conv_out_hw(x.shape[2], x.shape[3], R, S, *stride, *pad, *dil)
    if bias is not None:
        _check(bias, "bias", torch.bfloat16, K_)
    if stats is not None:
        _check(stats, "stats", torch.float32, 2 * K_)
    y = torch.empty((x.shape[0], K_, P, Q), device=x.device, dtype=x.dtype, memory_format=torch.channels_last)
    ws = None
    if stats is not None:
        ws = torch.empty(ext().conv2d_stats_ws_floats(g), device=x.device, dtype=torch.float32)
    ext().conv2d_fwd(g, _p(x), _p(w), _p(bias), _p(y), _p(stats), _p(ws), ACT_CODES[act], _stream())
    STATS["conv2d_fwd"] += 1
    return y


def conv2d_dgrad(dy, w, x_shape, stride=(1, 1), pad=(0, 0), dil=(1, 1), out=None, beta: float = 0.0,
                 bn=None):
    """dx of a convolution.  ``bn = (x, mean, rstd, scale_shift or None)`` of
    the BatchNorm(+ReLU) that produced the conv input: the epilogue also
    reduces that BN's backward sums over the ReLU-masked dx (fp32 [2, C]:
    sum g, sum g * xhat), returned as ``dx._ff_bn_sums = (sums, x)`` for
    ``bn_bwd(pre_sums=...)`` (stride-1 convs, no accumulation)."""
    _check_nhwc(dy, "dy")
    K_, R, S, C = w.shape
    _check(w, "w", torch.bfloat16)
    g = _conv_geom(x_shape, K_, R, S, stride, pad, dil)
    P, Q = conv_out_hw(x_shape[2], x_shape[3], R, S, *stride, *pad, *dil)
    if tuple(dy.shape) != (x_shape[0], K_, P, Q):
        raise ValueError(f"conv2d_dgrad: dy shape {tuple(dy.shape)} != {(x_shape[0], K_, P, Q)}")
    if out is None:
        out = torch.empty(tuple(x_shape), device=dy.device, dtype=dy.dtype, memory_format=torch.channels_last)
        beta = 0.0
    else:
        _check_nhwc(out, "dx")
        if tuple(out.shape) != tuple(x_shape):
            raise ValueError("conv2d_dgrad: out has the wrong shape")
    if bn is not None:
        bx, mean, rstd, ss = bn
        C = x_shape[1]
        if beta != 0.0 or tuple(stride) != (1, 1) or tuple(dil) != (1, 1):
            raise ValueError("conv2d_dgrad: BN sums need a stride-1 dgrad without accumulation")
        _check_nhwc(bx, "bn x")
        if tuple(bx.shape) != tuple(x_shape):
            raise ValueError("conv2d_dgrad: BN input shape mismatch")
        for name, t, n in (("mean", mean, C), ("rstd", rstd, C), ("scale_shift", ss, 2 * C)):
            if t is not None:
                _check(t, name, torch.float32, n)
        sums = torch.empty(2 * C, device=dy.device, dtype=torch.float32)
        ws = torch.empty(ext().conv2d_dgrad_bn_ws_floats(g), device=dy.device, dtype=torch.float32)
        ext().conv2d_dgrad_bn(g, _p(dy), _p(w), _p(out), _p(bx), _p(mean), _p(rstd), _p(ss), _p(sums), _p(ws),
                              _stream())
        out._ff_bn_sums = (sums, bx)
        STATS["conv2d_dgrad_bn"] += 1
        return out
    ext().conv2d_dgrad(g, _p(dy), _p(w), _p(out), float(beta), _stream())
    STATS["conv2d_dgrad"] += 1
    return out


def conv2d_wgrad(x, dy, dw, R, S, stride=(1, 1), pad=(0, 0), dil=(1, 1), splits: int = 0):
    """dw (fp32, K*R*S*C elements, layout [K][R][S][C]) += wgrad."""
    _check_nhwc(x, "x")
    _check_nhwc(dy, "dy")
    K_ = dy.shape[1]
    g = _conv_geom(x.shape, K_, R, S, stride, pad, dil)
    P, Q = conv_out_hw(x.shape[2], x.shape[3], R, S, *stride, *pad, *dil)
    if tuple(dy.shape) != (x.shape[0], K_, P, Q):
        raise ValueError("conv2d_wgrad: dy shape mismatch")
    if not dw.is_cuda or dw.dtype != torch.float32 or not dw.is_contiguous() or dw.numel() != K_ * R * S * x.shape[1]:
        raise ValueError("conv2d_wgrad: dw must be a contiguous fp32 [K,R,S,C] buffer")
    nws = ext().conv2d_wgrad_ws_floats(g, int(splits))
    ws = torch.empty(nws, device=x.device, dtype=torch.float32) if nws else None
    ext().conv2d_wgrad(g, _p(x), _p(dy), _p(dw), _p(ws), int(splits), _stream())
    STATS["conv2d_wgrad"] += 1


def _grouped_geom(x_shape, K, R, S, stride, pad, dil, groups):
    N, C, H, W = x_shape
    if groups <= 0 or C % groups or K % groups:
        raise ValueError(f"conv2d_grouped: C={C} and K={K} must be multiples of groups={groups}")
    return [int(N), int(H), int(W), int(C), int(K), int(R), int(S), int(stride[0]), int(stride[1]),
            int(pad[0]), int(pad[1]), int(dil[0]), int(dil[1])]


def conv2d_grouped_expand(w, x_shape, stride=(1, 1), pad=(0, 0), dil=(1, 1), groups: int = 1):
    """Compact bf16 weight [K,R,S,C/groups] -> the block-diagonal super-group
    weight the grouped kernels read (conv.hip group_plan)."""
    K_, R, S, Cg = w.shape
    _check(w, "w", torch.bfloat16)
    if Cg * groups != x_shape[1]:
        raise ValueError(f"conv2d_grouped: weight has {Cg} x {groups} input channels, input has {x_shape[1]}")
    g = _grouped_geom(x_shape, K_, R, S, stride, pad, dil, groups)
    wexp = torch.empty(ext().conv2d_grouped_wexp_elems(g, int(groups)), device=w.device, dtype=torch.bfloat16)
    ext().conv2d_grouped_expand(g, int(groups), _p(w), _p(wexp), _stream())
    return wexp


def conv2d_grouped_fwd(x, w, bias=None, stride=(1, 1), pad=(0, 0), dil=(1, 1), groups: int = 1, act: str = "none",
                       stats=None, wexp=None):
    """Grouped bf16 convolution on the MFMA implicit-GEMM kernels: x [N,C,H,W]
    channels_last, w [K,R,S,C/groups] -> (y channels_last, the expanded
    weight, reused by the dgrad)."""
    _check_nhwc(x, "x")
    K_, R, S, Cg = w.shape
    g = _grouped_geom(x.shape, K_, R, S, stride, pad, dil, groups)
    if wexp is None:
        wexp = conv2d_grouped_expand(w, x.shape, stride, pad, dil, groups)
    P, Q = conv_out_hw(x.shape[2], x.shape[3], R, S, *stride, *pad, *dil)
    if bias is not None:
        _check(bias, "bias", torch.bfloat16, K_)
    if stats is not None:
        _check(stats, "stats", torch.float32, 2 * K_)
    y = torch.empty((x.shape[0], K_, P, Q), device=x.device, dtype=x.dtype, memory_format=torch.channels_last)
    ws = None
    if stats is not None:
        ws = torch.empty(ext().conv2d_stats_ws_floats(g), device=x.device, dtype=torch.float32)
    ext().conv2d_grouped_fwd(g, int(groups), _p(x), _p(wexp), _p(bias), _p(y), _p(stats), _p(ws), ACT_CODES[act],
                             _stream())
    STATS["conv2d_grouped_fwd"] += 1
    return y, wexp


def conv2d_grouped_dgrad(dy, wexp, w_shape, x_shape, stride=(1, 1), pad=(0, 0), dil=(1, 1), groups: int = 1,
                         out=None, beta: float = 0.0):
    """dx of a grouped convolution from the expanded weight."""
    _check_nhwc(dy, "dy")
    K_, R, S, Cg = w_shape
    g = _grouped_geom(x_shape, K_, R, S, stride, pad, dil, groups)
    P, Q = conv_out_hw(x_shape[2], x_shape[3], R, S, *stride, *pad, *dil)
    if tuple(dy.shape) != (x_shape[0], K_, P, Q) or Cg * groups != x_shape[1]:
        raise ValueError(f"conv2d_grouped_dgrad: dy {tuple(dy.shape)} / weight {tuple(w_shape)} do not match "
                         f"{tuple(x_shape)}")
    if wexp.numel() != ext().conv2d_grouped_wexp_elems(g, int(groups)) or wexp.dtype != torch.bfloat16:
        raise ValueError("conv2d_grouped_dgrad: wexp is not this convolution's expanded weight")
    if out is None:
        out = torch.empty(tuple(x_shape), device=dy.device, dtype=dy.dtype, memory_format=torch.channels_last)
        beta = 0.0
    else:
        _check_nhwc(out, "dx")
        if tuple(out.shape) != tuple(x_shape):
            raise ValueError("conv2d_grouped_dgrad: out has the wrong shape")
    ext().conv2d_grouped_dgrad(g, int(groups), _p(dy), _p(wexp), _p(out), float(beta), _stream())
    STATS["conv2d_grouped_dgrad"] += 1
    return out


def conv2d_grouped_wgrad(x, dy, dw, R, S, stride=(1, 1), pad=(0, 0), dil=(1, 1), groups: int = 1):
    """dw (fp32, [K][R][S][C/groups] contiguous) += grouped wgrad."""
    _check_nhwc(x, "x")
    _check_nhwc(dy, "dy")
    K_ = dy.shape[1]
    g = _grouped_geom(x.shape, K_, R, S, stride, pad, dil, groups)
    P, Q = conv_out_hw(x.shape[2], x.shape[3], R, S, *stride, *pad, *dil)
    if tuple(dy.shape) != (x.shape[0], K_, P, Q):
        raise ValueError("conv2d_grouped_wgrad: dy shape mismatch")
    if (not dw.is_cuda or dw.dtype != torch.float32 or not dw.is_contiguous()
            or dw.numel() != K_ * R * S * (x.shape[1] // groups)):
        raise ValueError("conv2d_grouped_wgrad: dw must be a contiguous fp32 [K,R,S,C/groups] buffer")
    ws = torch.empty(ext().conv2d_grouped_wgrad_ws_floats(g, int(groups)), device=x.device, dtype=torch.float32)
    ext().conv2d_grouped_wgrad(g, int(groups), _p(x), _p(dy), _p(dw), _p(ws), _stream())
    STATS["conv2d_grouped_wgrad"] += 1


def _rm2d(t: torch.Tensor) -> torch.Tensor:
    """A 2-D operand the kernels can address as rows of unit-stride elements
    (size-1 dims may carry any stride)."""
    if t.shape[1] == 1 or t.stride(1) == 1:
        return t
    return t.contiguous()


def _ld2d(t: torch.Tensor) -> int:
    """Leading dimension of a row-major 2-D tensor (its row stride; a
    single row or a size-1 row dim reports the row length)."""
    if t.shape[0] == 1:
        return max(1, t.shape[1])
    return t.stride(0)


def gemm_f32(a, b, trans_a=False, trans_b=False, bias=None, act="none", alpha=1.0, beta=0.0, out=None, pre=None,
             out_dtype=None):
    """C = act(alpha op(a) op(b) + bias) (+ beta C) on the exact-fp32 MFMA
    (igemm32.hip).  a / b: 2-D fp32 (or bf16) with unit inner stride;
    bias / pre / out in the output dtype (default: the inputs')."""
    if a.dtype != b.dtype or a.dtype not in (torch.float32, torch.bfloat16):
        raise ValueError("gemm_f32: operands must share dtype fp32 / bf16")
    if a.dim() != 2 or b.dim() != 2:
        raise ValueError("gemm_f32: operands must be 2-D")
    a, b = _rm2d(a), _rm2d(b)
    if not (a.is_cuda and b.is_cuda):
        raise ValueError("gemm_f32: GPU tensors expected")
    M, Kd = (a.shape[1], a.shape[0]) if trans_a else (a.shape[0], a.shape[1])
    Kb, N = (b.shape[1], b.shape[0]) if trans_b else (b.shape[0], b.shape[1])
    if Kd != Kb:
        raise ValueError(f"gemm_f32: inner dims differ ({Kd} vs {Kb})")
    dt = out_dtype or (out.dtype if out is not None else a.dtype)
    if out is None:
        out = torch.empty(M, N, device=a.device, dtype=dt)
        beta = 0.0
    if tuple(out.shape) != (M, N) or (out.stride(1) != 1 and N > 1) or out.dtype not in (torch.float32,
                                                                                        torch.bfloat16):
        raise ValueError("gemm_f32: bad output")
    # bias is read in the inputs' dtype, pre written in the output's
    for name, t, want in (("bias", bias, a.dtype), ("pre", pre, out.dtype)):
        if t is not None and (t.dtype != want or not t.is_contiguous() or not t.is_cuda):
            raise ValueError(f"gemm_f32: {name} must be a contiguous GPU {want} tensor")
    if bias is not None and bias.numel() != N:
        raise ValueError("gemm_f32: bias must have N elements")
    if pre is not None and (pre.numel() != M * N or _ld2d(out) != N):
        raise ValueError("gemm_f32: pre needs a dense output")
    ext().gemm_f32(_p(a), _p(b), _p(out), _p(bias), _p(pre), M, N, Kd, _ld2d(a), _ld2d(b), _ld2d(out),
                   bool(trans_a), bool(trans_b), ACT_CODES[act], float(alpha), float(beta),
                   int(a.dtype == torch.float32), int(out.dtype == torch.float32), _stream(), 1, 0, 0, 0)
    STATS["gemm_f32"] += 1
    return out


def bmm_f32(a, b, trans_a=False, trans_b=False, alpha=1.0):
    """Batched fp32 product over the leading dims (one launch, blockIdx.z =
    batch): a [..., M, K] (or [..., K, M]), b [..., K, N] (or [..., N, K])."""
    if a.dtype != torch.float32 or b.dtype != torch.float32 or a.dim() < 3 or a.shape[:-2] != b.shape[:-2]:
        raise ValueError("bmm_f32: fp32 operands with equal batch dims")
    lead = a.shape[:-2]
    a3 = a.reshape(-1, a.shape[-2], a.shape[-1]).contiguous()
    b3 = b.reshape(-1, b.shape[-2], b.shape[-1]).contiguous()
    M, Kd = (a3.shape[2], a3.shape[1]) if trans_a else (a3.shape[1], a3.shape[2])
    Kb, N = (b3.shape[2], b3.shape[1]) if trans_b else (b3.shape[1], b3.shape[2])
    if Kd != Kb:
        raise ValueError("bmm_f32: inner dims differ")
    nb = a3.shape[0]
    out = torch.empty(nb, M, N, device=a.device, dtype=torch.float32)
    if nb > 65535:
        raise ValueError("bmm_f32: batch > 65535")
    ext().gemm_f32(_p(a3), _p(b3), _p(out), 0, 0, M, N, Kd, a3.stride(1), b3.stride(1), N, bool(trans_a),
                   bool(trans_b), 0, float(alpha), 0.0, 1, 1, _stream(), nb, a3.stride(0), b3.stride(0), M * N)
    STATS["gemm_f32"] += 1
    return out.reshape(*lead, M, N)


def _check_nhwc_any(t: torch.Tensor, name: str, dtype):
    if not t.is_cuda or t.dtype != dtype:
        raise ValueError(f"{name}: expected a GPU {dtype} tensor")
    if t.dim() != 4 or not t.is_contiguous(memory_format=torch.channels_last):
        raise ValueError(f"{name}: expected a 4-d channels_last tensor")


def _conv32_geom(x_shape, K, R, S, stride, pad, dil, groups):
    N, C, H, W = x_shape
    if groups <= 0 or C % groups or K % groups:
        raise ValueError(f"conv32: C={C} and K={K} must be multiples of groups={groups}")
    return [int(N), int(H), int(W), int(C), int(K), int(R), int(S), int(stride[0]), int(stride[1]),
            int(pad[0]), int(pad[1]), int(dil[0]), int(dil[1])]


def conv32_fwd(x, w, bias=None, stride=(1, 1), pad=(0, 0), dil=(1, 1), groups: int = 1, act: str = "none"):
    """Grouped / fp32 convolution (igemm32.hip): x [N,C,H,W] channels_last
    fp32 or bf16, w [K,R,S,C/groups] contiguous in x's dtype -> y channels_last."""
    _check_nhwc_any(x, "x", x.dtype)
    K_, R, S, Cg = w.shape
    _check(w, "w", x.dtype)
    if Cg * groups != x.shape[1]:
        raise ValueError(f"conv32: weight has {Cg} x {groups} input channels, input has {x.shape[1]}")
    g = _conv32_geom(x.shape, K_, R, S, stride, pad, dil, groups)
    P, Q = conv_out_hw(x.shape[2], x.shape[3], R, S, *stride, *pad, *dil)
    if bias is not None and (bias.dtype != x.dtype or bias.numel() != K_ or not bias.is_contiguous()):
        raise ValueError("conv32: bias must be a contiguous [K] tensor in x's dtype")
    y = torch.empty((x.shape[0], K_, P, Q), device=x.device, dtype=x.dtype, memory_format=torch.channels_last)
    ext().conv32_fwd(g, int(groups), _p(x), _p(w), _p(bias), _p(y), ACT_CODES[act], int(x.dtype == torch.float32),
                     _stream())
    STATS["conv32_fwd"] += 1
    return y


def conv32_dgrad(dy, w, x_shape, stride=(1, 1), pad=(0, 0), dil=(1, 1), groups: int = 1, out=None,
                 beta: float = 0.0):
    _check_nhwc_any(dy, "dy", dy.dtype)
    K_, R, S, Cg = w.shape
    _check(w, "w", dy.dtype)
    g = _conv32_geom(x_shape, K_, R, S, stride, pad, dil, groups)
    P, Q = conv_out_hw(x_shape[2], x_shape[3], R, S, *stride, *pad, *dil)
    if tuple(dy.shape) != (x_shape[0], K_, P, Q) or Cg * groups != x_shape[1]:
        raise ValueError(f"conv32_dgrad: dy {tuple(dy.shape)} / weight {tuple(w.shape)} do not match {tuple(x_shape)}")
    if out is None:
        out = torch.empty(tuple(x_shape), device=dy.device, dtype=dy.dtype, memory_format=torch.channels_last)
        beta = 0.0
    else:
        _check_nhwc_any(out, "dx", dy.dtype)
        if tuple(out.shape) != tuple(x_shape):
            raise ValueError("conv32_dgrad: out has the wrong shape")
    ext().conv32_dgrad(g, int(groups), _p(dy), _p(w), _p(out), float(beta), int(dy.dtype == torch.float32), _stream())
    STATS["conv32_dgrad"] += 1
    return out


def conv32_wgrad(x, dy, dw, R, S, stride=(1, 1), pad=(0, 0), dil=(1, 1), groups: int = 1):
    """dw (fp32, contiguous, layout [K][R][S][C/groups]) += weight gradient."""
    _check_nhwc_any(x, "x", x.dtype)
    _check_nhwc_any(dy, "dy", x.dtype)
    K_ = dy.shape[1]
    g = _conv32_geom(x.shape, K_, R, S, stride, pad, dil, groups)
    P, Q = conv_out_hw(x.shape[2], x.shape[3], R, S, *stride, *pad, *dil)
    if tuple(dy.shape) != (x.shape[0], K_, P, Q):
        raise ValueError("conv32_wgrad: dy shape mismatch")
    if (not dw.is_cuda or dw.dtype != torch.float32 or not dw.is_contiguous()
            or dw.numel() != K_ * R * S * (x.shape[1] // groups)):
        raise ValueError("conv32_wgrad: dw must be a contiguous fp32 [K,R,S,C/groups] buffer")
    ext().conv32_wgrad(g, int(groups), _p(x), _p(dy), _p(dw), int(x.dtype == torch.float32), _stream())
    STATS["conv32_wgrad"] += 1


_BN_WS: Dict[tuple, torch.Tensor] = {}


def _bn_workspace(dev, C: int):
    """(workspace of 35 C floats, clean): a persistent per-(device, stream, C)
    buffer whose 16 atomic buckets start zero and are left zero by the kernel
    that consumes them (bn_fold_buckets / bn_bwd_coef), so no memset runs per
    call.  Inside a graph capture a first use gets a per-call buffer instead
    (zeroed by the launcher)."""
    key = (dev, C)   # one stream runs the BN passes: stream order keeps uses apart
    ws = _BN_WS.get(key)
    if ws is not None:
        return ws, 1
    if torch.cuda.is_current_stream_capturing():
        return torch.empty(35 * C, device=dev, dtype=torch.float32), 0
    ws = _BN_WS[key] = torch.zeros(35 * C, device=dev, dtype=torch.float32)
    return ws, 1


def bn_stats(x, stats, overwrite: bool = False):
    """stats (fp32 [2, C]) += per-channel (sum, sum of squares) of x;
    ``overwrite``: stats = ... (no zeroing pass needed)."""
    _check_nhwc(x, "x")
    C = x.shape[1]
    _check(stats, "stats", torch.float32, 2 * C)
    ws, clean = _bn_workspace(x.device, C)
    ext().bn_stats(_p(x), _p(stats), x.numel() // C, C, _stream(), _p(ws), clean | (2 if overwrite else 0))
    STATS["bn_stats"] += 1


def bn_finalize(stats, gamma, beta, count, eps, momentum=0.0, running_mean=None, running_var=None):
    """-> (scale, shift, mean, rstd) fp32 [C]."""
    C = stats.numel() // 2
    f = torch.empty(4, C, device=stats.device, dtype=torch.float32)
    pdt = DT_BF16
    for name, t in (("gamma", gamma), ("beta", beta)):
        if t is not None:
            if t.numel() != C or not t.is_contiguous():
                raise ValueError(f"bn_finalize: {name} must have {C} contiguous elements")
            pdt = _dt(t)
    if gamma is not None and beta is not None and gamma.dtype != beta.dtype:
        raise ValueError("bn_finalize: gamma/beta dtype mismatch")
    for t in (running_mean, running_var):
        if t is not None:
            _check(t, "running stat", torch.float32, C)
    ext().bn_finalize(_p(stats), _p(gamma), _p(beta), pdt, _p(running_mean), _p(running_var), _p(f[0]), _p(f[1]),
                      _p(f[2]), _p(f[3]), C, float(count), float(momentum), float(eps), _stream())
    STATS["bn_finalize"] += 1
    return f[0], f[1], f[2], f[3]


def bn_apply(x, scale, shift, relu: bool, residual=None):
    _check_nhwc(x, "x")
    C = x.shape[1]
    if residual is not None:
        _check_nhwc(residual, "residual")
        if residual.shape != x.shape:
            raise ValueError("bn_apply: residual shape mismatch")
    y = torch.empty_like(x, memory_format=torch.channels_last)
    ext().bn_apply(_p(x), _p(residual), _p(scale), _p(shift), _p(y), x.numel() // C, C, int(relu), _stream())
    STATS["bn_apply"] += 1
    return y


def bn_bwd(dy, x, y, mean, rstd, gamma, relu: bool, dgamma=None, dbeta=None, want_masked: bool = False,
           scale_shift=None, pre_sums=None):
    """-> (dx, masked dy or None).  With ``relu`` the mask comes from ``y``,
    or — when ``y`` is None — is recomputed from ``x`` with the forward's
    ``scale_shift`` (fp32 [2, C]: scale, shift), so y is never re-read."""
    _check_nhwc(dy, "dy")
    _check_nhwc(x, "x")
    C = x.shape[1]
    relu_code = 0
    if relu and y is not None:
        _check_nhwc(y, "y")
        relu_code = 1
    elif relu:
        _check(scale_shift, "scale_shift", torch.float32, 2 * C)
        relu_code = 2
    for name, t in (("dgamma", dgamma), ("dbeta", dbeta)):
        if t is not None and (t.dtype != torch.float32 or t.numel() != C or not t.is_contiguous()):
            raise ValueError(f"bn_bwd: {name} must be fp32 [{C}]")
    pdt = _dt(gamma) if gamma is not None else DT_BF16
    dx = torch.empty_like(x, memory_format=torch.channels_last)
    dres = torch.empty_like(x, memory_format=torch.channels_last) if want_masked else None
    if pre_sums is not None:
        _check(pre_sums, "pre_sums", torch.float32, 2 * C)
        if want_masked:
            raise ValueError("bn_bwd: precomputed sums cannot serve the residual form")
    ws, clean = _bn_workspace(x.device, C)
    ext().bn_bwd(_p(dy), _p(x), _p(y if relu_code == 1 else None), _p(mean), _p(rstd), _p(gamma), pdt, _p(dx),
                 _p(dres), _p(dgamma), _p(dbeta), _p(ws), x.numel() // C, C, relu_code, _stream(),
                 _p(scale_shift if relu_code == 2 else None), clean, _p(pre_sums))
    STATS["bn_bwd"] += 1
    return dx, dres


def _pool_geom(x_shape, k, s, p, avg, count_pad):
    N, C, H, W = x_shape
    if C % 8:
        raise ValueError("pool2d: channels must be a multiple of 8")
    if k[0] * k[1] > 256:
        raise ValueError("pool2d: window larger than 256 taps")
    return [int(N), int(H), int(W), int(C), int(k[0]), int(k[1]), int(s[0]), int(s[1]), int(p[0]), int(p[1]),
            int(avg), int(count_pad)]


def pool2d_fwd(x, k, s, p, avg: bool, count_pad: bool = False, need_argmax: bool = True):
    _check_nhwc(x, "x")
    g = _pool_geom(x.shape, k, s, p, avg, count_pad)
    P = (x.shape[2] + 2 * p[0] - k[0]) // s[0] + 1
    Q = (x.shape[3] + 2 * p[1] - k[1]) // s[1] + 1
    y = torch.empty((x.shape[0], x.shape[1], P, Q), device=x.device, dtype=x.dtype,
                    memory_format=torch.channels_last)
    arg = None
    if not avg and need_argmax:
        arg = torch.empty(y.numel(), device=x.device, dtype=torch.uint8)
    ext().pool2d_fwd(g, _p(x), _p(y), _p(arg), _stream())
    STATS["pool2d_fwd"] += 1
    return y, arg


def pool2d_bwd(dy, arg, x_shape, k, s, p, avg: bool, count_pad: bool = False):
    _check_nhwc(dy, "dy")
    g = _pool_geom(x_shape, k, s, p, avg, count_pad)
    if not avg and (arg is None or arg.numel() != dy.numel()):
        raise ValueError("pool2d_bwd: max pooling needs the forward's argmax")
    dx = torch.empty(tuple(x_shape), device=dy.device, dtype=dy.dtype, memory_format=torch.channels_last)
    ext().pool2d_bwd(g, _p(dy), _p(arg), _p(dx), 0.0, _stream())
    STATS["pool2d_bwd"] += 1
    return dx


# ---------------------------------------------------------------------------
# hipBLASLt GEMMs with fused epilogues (csrc/kernels/blaslt.hip)
EPI_NONE, EPI_BIAS, EPI_GELU_BIAS, EPI_BGRADB = 0, 1, 3, 4
_BLT_WS = {}
_BLT_WS_BYTES = 64 << 20


def _blaslt_ws(dev):
    # one workspace per (device, stream): GEMMs on the weight-gradient stream
    # run concurrently with those on the compute stream
    key = (dev, torch.cuda.current_stream(dev).cuda_stream)
    w = _BLT_WS.get(key)
    if w is None:
        w = torch.empty(_BLT_WS_BYTES, dtype=torch.uint8, device=dev)
        _BLT_WS[key] = w
    return w


def _gemm_dims(a, b, trans_a, trans_b):
    M, K = (a.shape[1], a.shape[0]) if trans_a else (a.shape[0], a.shape[1])
    Kb, N = (b.shape[1], b.shape[0]) if trans_b else (b.shape[0], b.shape[1])
    if K != Kb:
        raise ValueError(f"gemm: inner dims differ ({K} vs {Kb})")
    return M, N, K


def _rowmajor(t, name):
    if not t.is_cuda or t.dim() != 2 or t.stride(1) != 1 or t.data_ptr() % 16 or t.stride(0) % 8:
        raise ValueError(f"{name}: expected a 2-D row-major GPU matrix (16-byte aligned rows)")
    return t.stride(0)


def blaslt_num_algos(a, b, trans_a, trans_b, out, beta: float = 0.0, bias_epilogue: bool = False) -> int:
    """Heuristic candidates hipBLASLt offers for C(out) = op(a) op(b) [+ bias]
    (row-strided operands allowed); 0 when unsupported."""
    M, N, K = _gemm_dims(a, b, trans_a, trans_b)
    odt = torch.bfloat16 if out is None else out.dtype
    if a.dtype != torch.bfloat16 or b.dtype != torch.bfloat16 or odt not in (torch.bfloat16, torch.float32):
        return 0
    try:
        lda, ldb = _rowmajor(a, "a"), _rowmajor(b, "b")
        ldc = N if out is None else _rowmajor(out, "out")
    except ValueError:
        return 0
    return ext().blaslt_num_algos(M, N, K, lda, ldb, ldc, bool(trans_a), bool(trans_b),
                                  EPI_BIAS if bias_epilogue else EPI_NONE, int(odt == torch.float32),
                                  bool(beta), N, _BLT_WS_BYTES)


def blaslt_matmul(a, b, trans_a, trans_b, out, beta: float = 0.0, bias=None, algo: int = 0):
    """out = op(a) op(b) [+ bias] (+ beta * out) with hipBLASLt's ``algo``-th
    heuristic candidate; operands may be row-strided views."""
    M, N, K = _gemm_dims(a, b, trans_a, trans_b)
    lda, ldb, ldc = _rowmajor(a, "a"), _rowmajor(b, "b"), _rowmajor(out, "out")
    if tuple(out.shape) != (M, N):
        raise ValueError("blaslt_matmul: out has the wrong shape")
    if bias is not None:
        _check(bias, "bias", torch.bfloat16, N)
    ext().blaslt_gemm(_p(a), _p(b), _p(out), M, N, K, lda, ldb, ldc, bool(trans_a), bool(trans_b),
                      EPI_BIAS if bias is not None else EPI_NONE, _p(bias), 0, N, 1.0, float(beta),
                      int(out.dtype == torch.float32), _p(_blaslt_ws(a.device)), _BLT_WS_BYTES, _stream(), int(algo))
    STATS["blaslt_gemm"] += 1
    return out


def blaslt_solutions(a, b, trans_a, trans_b, out, beta: float = 0.0):
    """Library solution indices (every hipBLASLt kernel, not just the
    heuristic's top candidates) that support C(out) = op(a) op(b) [+ out]."""
    M, N, K = _gemm_dims(a, b, trans_a, trans_b)
    return list(ext().blaslt_solutions(M, N, K, _rowmajor(a, "a"), _rowmajor(b, "b"), _rowmajor(out, "out"),
                                       bool(trans_a), bool(trans_b), int(out.dtype == torch.float32), bool(beta),
                                       _BLT_WS_BYTES))


def blaslt_matmul_solution(a, b, trans_a, trans_b, out, beta: float = 0.0, index: int = 0):
    """C = op(a) op(b) (+ beta * out) with hipBLASLt solution ``index``."""
    M, N, K = _gemm_dims(a, b, trans_a, trans_b)
    if tuple(out.shape) != (M, N):
        raise ValueError("blaslt_matmul_solution: out has the wrong shape")
    ext().blaslt_gemm_solution(_p(a), _p(b), _p(out), M, N, K, _rowmajor(a, "a"), _rowmajor(b, "b"),
                               _rowmajor(out, "out"), bool(trans_a), bool(trans_b), 1.0, float(beta),
                               int(out.dtype == torch.float32), _p(_blaslt_ws(a.device)), _BLT_WS_BYTES, _stream(),
                               int(index))
    STATS["blaslt_gemm"] += 1
    return out


def blaslt_ok(a, b, trans_a=False, trans_b=False, epilogue=EPI_NONE, out_f32=False, beta=0.0) -> bool:
    """True when hipBLASLt has an algorithm for this GEMM + epilogue (cached)."""
    if not (a.is_cuda and b.is_cuda and a.dtype == torch.bfloat16 and b.dtype == torch.bfloat16):
        return False
    if not (a.is_contiguous() and b.is_contiguous()):
        return False
    M, N, K = _gemm_dims(a, b, trans_a, trans_b)
    return ext().blaslt_supported(M, N, K, a.shape[1], b.shape[1], N, bool(trans_a), bool(trans_b), int(epilogue),
                                  int(out_f32), bool(beta), N, _BLT_WS_BYTES)


def blaslt_gemm(a, b, trans_a=False, trans_b=False, epilogue=EPI_NONE, bias=None, aux=None, out=None,
                beta: float = 0.0, alpha: float = 1.0, out_f32: bool = False):
    """C = op(a) @ op(b) with a hipBLASLt epilogue (see blaslt.hip).  ``bias``:
    bf16 [N] input for BIAS / GELU_BIAS, fp32 OUTPUT (overwritten) for
    BGRADB = colsum of op(a) over K."""
    for name, t in (("a", a), ("b", b)):
        _check(t, name, torch.bfloat16)
    M, N, K = _gemm_dims(a, b, trans_a, trans_b)
    if out is None:
        out = torch.empty(M, N, device=a.device, dtype=torch.float32 if out_f32 else torch.bfloat16)
        beta = 0.0
    else:
        out_f32 = out.dtype == torch.float32
        if tuple(out.shape) != (M, N) and out.numel() != M * N:
            raise ValueError("blaslt_gemm: out has the wrong shape")
        _check(out, "out")
    if epilogue in (EPI_BIAS, EPI_GELU_BIAS):
        _check(bias, "bias", torch.bfloat16, N)
    elif epilogue == EPI_BGRADB:
        _check(bias, "bias grad", torch.float32, M)
    ws = _blaslt_ws(a.device)
    ext().blaslt_gemm(_p(a), _p(b), _p(out), M, N, K, a.shape[1], b.shape[1], N, bool(trans_a), bool(trans_b),
                      int(epilogue), _p(bias), _p(aux), N, float(alpha), float(beta), int(out_f32), _p(ws),
                      _BLT_WS_BYTES, _stream(), 0)
    STATS["blaslt_gemm"] += 1
    return out
