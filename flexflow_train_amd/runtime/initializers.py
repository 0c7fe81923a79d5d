"""Weight initializers (reference: lib/pcg/include/pcg/initializers/*.struct.toml —
glorot uniform/normal, zero, uniform, normal, truncated normal, constant —
and lib/runtime/src/initializer_kernels.cu).  Generated on the host from a
seeded generator so every replica of a weight is bit-identical without a
broadcast."""
from __future__ import annotations

import math
from typing import Sequence

import torch


def _fans(shape: Sequence[int]):
    shape = list(shape)
    if len(shape) == 0:
        return 1, 1
    if len(shape) == 1:
        return shape[0], shape[0]
    if len(shape) == 2:       # Linear kernel [in, out]
        return shape[0], shape[1]
    rf = math.prod(shape[2:])  # Conv kernel [out, in, kh, kw]
    return shape[1] * rf, shape[0] * rf


def make_initializer_tensor(init: dict, shape: Sequence[int], gen: torch.Generator) -> torch.Tensor:
    t = (init or {}).get("type", "zero")
    shape = tuple(int(s) for s in shape)
    if t == "zero":
        return torch.zeros(shape)
    if t == "constant":
        return torch.full(shape, float(init.get("value", 0.0)))
    if t == "uniform":
        lo, hi = float(init.get("min", init.get("min_val", -0.05))), float(init.get("max", init.get("max_val", 0.05)))
        return torch.rand(shape, generator=gen) * (hi - lo) + lo
    if t == "normal":
        return torch.randn(shape, generator=gen) * float(init.get("stddev", 1.0)) + float(init.get("mean", 0.0))
    if t == "truncated_normal":
        mean, std = float(init.get("mean", 0.0)), float(init.get("stddev", 1.0))
        lo = float(init.get("min_cutoff", mean - 2 * std))
        hi = float(init.get("max_cutoff", mean + 2 * std))
        x = torch.randn(shape, generator=gen) * std + mean
        for _ in range(8):
            bad = (x < lo) | (x > hi)
            if not bad.any():
                break
            x[bad] = torch.randn(int(bad.sum()), generator=gen) * std + mean
        return x.clamp(lo, hi)
    fan_in, fan_out = _fans(shape)
    if t == "glorot_uniform":
        b = math.sqrt(6.0 / (fan_in + fan_out))
        return (torch.rand(shape, generator=gen) * 2 - 1) * b
    if t == "glorot_normal":
        return torch.randn(shape, generator=gen) * math.sqrt(2.0 / (fan_in + fan_out))
    raise ValueError(f"unknown initializer {t}")


# ---------------------------------------------------------------------------
# Counter-based sharded initialisation.  Each element's value is a pure
# function of (seed, its GLOBAL linear index in the logical tensor), so a rank
# generates only the box it owns -- O(piece) work and memory instead of
# materialising the full weight on every rank -- and the result is
# independent of the parallelisation.  GPU: ffk::init_tensor
# (csrc/kernels/tensorops.hip); CPU: the same splitmix64 stream in numpy.
# ---------------------------------------------------------------------------
KIND_UNIFORM, KIND_NORMAL, KIND_TRUNC, KIND_CONST = 0, 1, 2, 3


def counter_spec(init: dict, shape: Sequence[int]):
    """initializer JSON -> (kind, a, b, c, d) for the counter generator."""
    t = (init or {}).get("type", "zero")
    if t == "zero":
        return KIND_CONST, 0.0, 0.0, 0.0, 0.0
    if t == "constant":
        return KIND_CONST, float(init.get("value", 0.0)), 0.0, 0.0, 0.0
    if t == "uniform":
        lo, hi = float(init.get("min", init.get("min_val", -0.05))), float(init.get("max", init.get("max_val", 0.05)))
        return KIND_UNIFORM, lo, hi, 0.0, 0.0
    if t == "normal":
        return KIND_NORMAL, float(init.get("mean", 0.0)), float(init.get("stddev", 1.0)), 0.0, 0.0
    if t == "truncated_normal":
        mean, std = float(init.get("mean", 0.0)), float(init.get("stddev", 1.0))
        return (KIND_TRUNC, mean, std, float(init.get("min_cutoff", mean - 2 * std)),
                float(init.get("max_cutoff", mean + 2 * std)))
    fan_in, fan_out = _fans(shape)
    if t == "glorot_uniform":
        b = math.sqrt(6.0 / (fan_in + fan_out))
        return KIND_UNIFORM, -b, b, 0.0, 0.0
    if t == "glorot_normal":
        return KIND_NORMAL, 0.0, math.sqrt(2.0 / (fan_in + fan_out)), 0.0, 0.0
    raise ValueError(f"unknown initializer {t}")


_M64 = (1 << 64) - 1


def _hash_u32(seed: int, idx):
    import numpy as np
    with np.errstate(over="ignore"):
        z = np.uint64(seed & _M64) + np.uint64(0x9E3779B97F4A7C15) * (idx + np.uint64(1))
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z ^= z >> np.uint64(31)
    return (z & np.uint64(0xFFFFFFFF)).astype(np.uint32)


def _uniform01(seed: int, idx):
    import numpy as np
    return (_hash_u32(seed, idx) >> np.uint32(8)).astype(np.float32) * np.float32(1.0 / 16777216.0)


def counter_values_cpu(global_idx, spec, seed: int):
    """Host mirror of init_kernel for an array of global indices (uint64)."""
    import numpy as np
    kind, a, b, c, d = spec
    shape = global_idx.shape
    g = global_idx.astype(np.uint64).reshape(-1)
    if kind == KIND_CONST:
        return np.full(shape, a, np.float32)
    if kind == KIND_UNIFORM:
        return (np.float32(a) + np.float32(b - a) * _uniform01(seed, np.uint64(2) * g)).astype(np.float32).reshape(shape)
    out = np.empty(g.shape, np.float32)
    todo = np.ones(g.shape, bool)
    for attempt in range(16):
        s = (seed ^ (0x9E37 * (attempt + 1))) & _M64
        gi = g[todo]
        u1 = np.maximum(_uniform01(s, np.uint64(2) * gi), np.float32(1e-7))
        u2 = _uniform01(s, np.uint64(2) * gi + np.uint64(1))
        z = np.float32(a) + np.float32(b) * np.sqrt(-2.0 * np.log(u1)) * np.cos(np.float32(6.283185307) * u2)
        z = z.astype(np.float32)
        if kind != KIND_TRUNC:
            out[todo] = z
            break
        ok = (z >= c) & (z <= d)
        idx = np.flatnonzero(todo)
        out[idx] = np.clip(z, c, d)
        todo[idx[ok]] = False
        if not todo.any():
            break
    return out.reshape(shape)


def counter_init_piece(spec, full_shape: Sequence[int], box, seed: int, device, dtype=torch.float32) -> torch.Tensor:
    """The box ``[(lo, hi), ...]`` of the logical tensor ``full_shape``."""
    from .. import kernels as K
    full_shape = [int(s) for s in full_shape]
    piece = [int(hi) - int(lo) for lo, hi in box]
    lo = [int(l) for l, _ in box]
    dev = torch.device(device)
    if dev.type == "cuda" and K.available():
        out = torch.empty(piece, dtype=dtype, device=dev)
        if out.numel():
            K.init_piece(out, full_shape, lo, ("uniform", "normal", "truncated_normal", "constant")[spec[0]],
                         seed, *spec[1:])
        return out
    import numpy as np
    if not piece:
        g = np.zeros((), np.uint64)
    else:
        g = np.zeros(piece, np.uint64)
        mul = 1
        for dd in range(len(piece) - 1, -1, -1):
            ar = (np.arange(piece[dd], dtype=np.uint64) + np.uint64(lo[dd])) * np.uint64(mul)
            g += ar.reshape([-1 if i == dd else 1 for i in range(len(piece))])
            mul *= full_shape[dd]
    return torch.from_numpy(counter_values_cpu(g, spec, seed)).to(device=dev, dtype=dtype)
