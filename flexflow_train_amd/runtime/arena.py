"""The step's device memory arena (csrc/runtime/arena.cpp, lib/libffarena.so).

One region per device, reserved before the first step at the size the
liveness memory plan gives (csrc/ffcore/src/memory_plan.cc), becomes the
segment source of a ``torch.cuda.MemPool`` through
``CUDAPluggableAllocator``: while the executor runs a step inside
``Arena.use()`` -- and when it captures the step into hipGraphs, whose pool is
this MemPool -- every activation, gradient and workspace comes out of the
region (torch's block cache splits the segments).  A request that does not
fit is served by hipMalloc and counted as overflow, so the step never fails
on the arena's account.  ``stats()`` reads the native tracker (capacity, live,
high water, overflow), the reference's tracked allocator
(lib/local-execution/src/tracked_allocator.cc:8-23).
"""
from __future__ import annotations

import contextlib
import ctypes
import os
from typing import Dict, Optional

import torch

_LIB = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "lib", "libffarena.so")
_POOLS: Dict[int, tuple] = {}


def available() -> bool:
    return os.path.exists(_LIB) and torch.cuda.is_available()


class Arena:
    def __init__(self, device: torch.device, nbytes: int):
        if not os.path.exists(_LIB):
            raise RuntimeError(f"arena library missing: {_LIB} (python tools/build_native.py kernels)")
        self.device = torch.device(device)
        self.index = self.device.index if self.device.index is not None else torch.cuda.current_device()
        # torch's device allocator is set up before a MemPool is made on top
        # of a pluggable one
        torch.cuda.init()
        torch.empty(1, device=self.device)
        self._lib = ctypes.CDLL(_LIB)
        self._lib.ff_arena_reserve.argtypes = [ctypes.c_int, ctypes.c_size_t]
        self._lib.ff_arena_reserve.restype = ctypes.c_int
        self._lib.ff_arena_stats.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_double)]
        self._lib.ff_arena_reset_high.argtypes = [ctypes.c_int]
        self._lib.ff_arena_reset_counts.argtypes = [ctypes.c_int]
        rc = self._lib.ff_arena_reserve(self.index, int(nbytes))
        if rc != 0:
            raise RuntimeError(f"arena: reserving {nbytes / 1e9:.2f} GB on device {self.index} failed ({rc})")
        self.requested = int(nbytes)
        # one allocator + MemPool per device for the life of the process (the
        # native region is never released either): a MemPool that dies
        # releases its blocks through its allocator, and the pluggable
        # allocator object may already be gone by then
        if self.index not in _POOLS:
            alloc = torch.cuda.memory.CUDAPluggableAllocator(_LIB, "ff_arena_alloc", "ff_arena_free")
            _POOLS[self.index] = (alloc, torch.cuda.MemPool(alloc.allocator()))
        self.allocator, self.pool = _POOLS[self.index]
        self._lib.ff_arena_reset_counts(self.index)

    def use(self):
        """Route this thread's allocations on the arena's device to it."""
        return torch.cuda.use_mem_pool(self.pool, self.device)

    @property
    def pool_id(self):
        return self.pool.id

    def stats(self) -> Dict[str, float]:
        buf = (ctypes.c_double * 8)()
        self._lib.ff_arena_stats(self.index, buf)
        cap, live, high, top, n, n_of, of_live, of_high = list(buf)
        return {"capacity_gb": round(cap / 1e9, 3), "live_gb": round(live / 1e9, 3),
                "high_water_gb": round(high / 1e9, 3), "top_gb": round(top / 1e9, 3),
                "segments": int(n), "overflow_segments": int(n_of),
                "overflow_high_gb": round(of_high / 1e9, 3)}

    def reset_high(self):
        self._lib.ff_arena_reset_high(self.index)


def bytes_per_param(optimizer_cfg) -> float:
    """Resident bytes per parameter outside the arena: fp32 master + bf16
    compute copy + gradient + optimizer state (Adam: two moments, SGD with
    momentum: one)."""
    from .optimizer import AdamConfig
    if isinstance(optimizer_cfg, AdamConfig):
        return 16.0
    return 14.0 if getattr(optimizer_cfg, "momentum", 0.0) else 10.0


def plan_bytes(pcg, views, world: int, rank: int, bytes_per_param: float, bf16: bool) -> int:
    """Arena size for one rank's step: the liveness plan's peak
    (csrc/ffcore/src/memory_plan.cc, executor fusions) minus the resident
    weights / optimizer state, +15 % and 2 GiB for workspaces and the block
    cache's slack."""
    from ..search import native
    plans = native.plan_memory(pcg, world, views, weight_bytes_per_param=bytes_per_param,
                               act_elem_bytes=2.0 if bf16 else 0.0, executor_fusions=True)
    p = plans[min(rank, len(plans) - 1)]
    return int(max(0.0, p["arena_bytes"] - p["weight_bytes"]) * 1.15 + (2 << 30))


def maybe(arena: Optional[Arena]):
    return arena.use() if arena is not None else contextlib.nullcontext()
