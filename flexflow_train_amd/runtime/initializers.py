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
