"""Rank-local prefetching data loader over the native BatchPrefetcher.

Parity: python/flexflow_dataloader.cc/.cu and SingleDataLoader
(flexflow_cffi.py:2449): the dataset stays in host memory and every
iteration moves each device's slice of the next batch to it.  Here:

* the C++ prefetcher (csrc/ffcore/src/dataloader.cc) gathers ONLY this
  rank's rows of each batch (its layout box on the sample dim) on background
  threads, ``depth`` batches ahead, into pinned staging slots;
* the staged slot is copied to HBM with a non-blocking H2D copy on a side
  HIP stream; the compute stream waits on that copy's event, so the copy
  overlaps the previous step's kernels;
* a slot is handed back to the prefetcher once its copy event completed.

Inputs that are not sharded on the sample dimension (replicated pieces) are
gathered whole; inputs sharded on other dims fall back to host slicing.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from .. import _ffcore as C

_NP_TO_TORCH = {np.dtype(np.float32): torch.float32, np.dtype(np.float64): torch.float64,
                np.dtype(np.int32): torch.int32, np.dtype(np.int64): torch.int64,
                np.dtype(np.float16): torch.float16, np.dtype(np.bool_): torch.bool,
                np.dtype(np.uint8): torch.uint8}


def _row_range(lay, rank: int, batch: int) -> Optional[Tuple[int, int]]:
    """(lo, hi) of the sample dim this rank holds, or None if the piece is cut
    along any other dim (host slicing then)."""
    c = lay.coord(rank)
    if c is None:
        return None
    box = lay.box(c.shard)
    for d, (lo, hi) in enumerate(box[1:], start=1):
        if lo != 0 or hi != lay.sizes[d]:
            return None
    lo, hi = box[0]
    if lay.sizes[0] != batch:
        return None
    return int(lo), int(hi)


class NativeDataLoader:
    """Iterates (feeds, labels) of rank-local device tensors.

    ``arrays``: name -> full host array [num_samples, ...]; ``label_name`` names
    the label array.  ``executor`` supplies the layouts (which rows this rank
    keeps) and the device."""

    def __init__(self, executor, arrays: Dict[str, np.ndarray], label_name: str, batch: int,
                 shuffle: bool = False, seed: int = 0, depth: int = 4, workers: int = 2):
        self.ex = executor
        self.batch = int(batch)
        self.names = [n for n in arrays if n != label_name]
        self.label_name = label_name
        self.dev = executor.cfg.device
        arrs: List[np.ndarray] = []
        rows: List[Tuple[int, int]] = []
        for n in self.names + [label_name]:
            a = np.ascontiguousarray(arrays[n])
            if n == label_name:
                lay = executor._loss_layout()
            else:
                lay = executor.inputs[n][1]
            rr = _row_range(lay, executor.rank, self.batch)
            if rr is None:
                raise ValueError(f"input {n}: layout is not a sample-dim split; use SingleDataLoader")
            arrs.append(a)
            rows.append(rr)
        self.arrays = arrs
        self.rows = rows
        self.pf = C.BatchPrefetcher(arrs, rows, self.batch, shuffle, seed, depth, workers)
        pin = self.dev.type == "cuda"
        self.staging: List[List[torch.Tensor]] = []
        for s in range(self.pf.depth):
            slot = []
            for i, a in enumerate(arrs):
                lo, hi = rows[i]
                t = torch.empty((hi - lo,) + a.shape[1:], dtype=_NP_TO_TORCH[a.dtype], pin_memory=pin)
                self.pf.set_slot(s, i, t.data_ptr())
                slot.append(t)
            self.staging.append(slot)
        self.copy_stream = torch.cuda.Stream(device=self.dev) if pin else None
        self._held: Optional[Tuple[int, Optional[torch.cuda.Event]]] = None
        self.started = False

    @property
    def iters_per_epoch(self) -> int:
        return self.pf.iters_per_epoch

    def start(self, first_batch: int = 0):
        self.pf.start(first_batch)
        self.started = True

    def _release_held(self):
        if self._held is not None:
            slot, ev = self._held
            if ev is not None:
                ev.synchronize()
            self.pf.release(slot)
            self._held = None

    def next(self):
        """-> (feeds {name: device tensor}, labels device tensor, batch index)."""
        if not self.started:
            self.start()
        self._release_held()
        slot, b = self.pf.next()
        host = self.staging[slot]
        if self.copy_stream is not None:
            with torch.cuda.stream(self.copy_stream):
                dev = [t.to(self.dev, non_blocking=True) for t in host]
                ev = torch.cuda.Event()
                ev.record(self.copy_stream)
            torch.cuda.current_stream().wait_event(ev)
            for t in dev:  # allocated on the copy stream, consumed on the compute stream
                t.record_stream(torch.cuda.current_stream())
            self._held = (slot, ev)
        else:
            dev = [t.clone() for t in host]
            self._held = (slot, None)
        feeds = {n: dev[i] for i, n in enumerate(self.names)}
        labels = dev[-1]
        return feeds, labels, b

    def __iter__(self):
        return self

    def __next__(self):
        return self.next()

    def close(self):
        if self.started:
            self._release_held()
            self.pf.stop()
            self.started = False

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001 — interpreter shutdown
            pass
