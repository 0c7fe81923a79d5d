"""Piecewise hipGraph capture of a distributed training step.

A single-rank training step is one hipGraph (``Executor.make_graphed_train_step``).
Across ranks the step contains RCCL collectives — the bucketed gradient
all-reduces that overlap the backward pass, the sharded optimizer's
reduce-scatter / all-gather, the parameter server's reduce / broadcast.
Instead of capturing the collectives themselves, the step is captured as a
chain of graph SEGMENTS cut at every collective:

    [graph 0: forward + loss + backward up to bucket 0 ready]
    all_reduce(bucket 0, async)            <- issued eagerly at replay
    [graph 1: backward up to bucket 1 ready]   (runs while bucket 0 reduces)
    ...
    wait(bucket 0..n)
    [graph n+1: optimizer update]

Replaying walks the chain: each segment is one ``hipGraphLaunch``; each
collective is re-issued through torch.distributed on the same (persistent)
gradient buffers, so RCCL runs exactly as in an eager step, on its own
stream, overlapped with the next segment, while the hundreds of per-op
kernel launches collapse into a handful of graph launches.  All segments
share one memory pool and are replayed in capture order, which is what
makes tensors flowing from one segment into the next valid.

Collectives that allocate their outputs (redistribution all-to-alls, MoE
dispatch, ring attention) cannot be cut this way; reaching one during a
segmented capture raises ``NotCapturable`` and the caller runs eagerly.

This is the MI355X replacement of the reference's Legion tracing
(``begin_trace``/``end_trace`` around every iteration,
python/flexflow/core/flexflow_cffi.py:562-566) for multi-GPU runs.

When every collective of the chain came with a descriptor (kind, operands,
process group, root), the chain is also handed to the native replayer
(``csrc/runtime/replay.cpp``, ``_ffreplay``): one call walks the graph
launches and issues the RCCL collectives through the C++ ``c10d``
ProcessGroup, with the interpreter out of the step (``FF_NATIVE_REPLAY=0``
keeps the Python walk).
"""
from __future__ import annotations

import os
import warnings
from typing import Callable, List, Optional, Tuple

import torch


# collective kinds of the native replayer (csrc/runtime/replay.cpp enum Kind)
NATIVE_KINDS = {"all_reduce": 1, "reduce_scatter": 2, "all_gather": 3, "reduce": 4, "broadcast": 5,
                "all_to_all": 7}


def _native_module():
    if os.environ.get("FF_NATIVE_REPLAY", "1") == "0":
        return None
    try:
        from .. import _ffreplay
    except ImportError:
        return None
    return _ffreplay


class NotCapturable(RuntimeError):
    """A collective with freshly allocated outputs was reached inside a
    segmented capture."""


def check_capturable(what: str):
    """Call before a collective that is not routed through the recorder."""
    if torch.cuda.is_available() and torch.cuda.is_current_stream_capturing():
        raise NotCapturable(f"{what} cannot be issued inside a segmented hipGraph capture")


class _PendingWork:
    """Stands in for a torch.distributed Work during capture: ``wait()``
    becomes a segment boundary whose replay waits on the real work."""

    def __init__(self, rec: "SegmentRecorder", slot: int):
        self.rec = rec
        self.slot = slot

    def wait(self):
        self.rec.wait(self.slot)
        return True

    def is_completed(self):
        return False


class SegmentRecorder:
    def __init__(self, pool=None):
        self.pool = pool if pool is not None else torch.cuda.graph_pool_handle()
        self.items: List[Tuple] = []
        self.cur: Optional[torch.cuda.CUDAGraph] = None
        self.n_async = 0
        self._native = None   # _ffreplay.Replayer once built

    # ---- capture side
    def begin(self):
        g = torch.cuda.CUDAGraph()
        # thread-local capture: RCCL's watchdog thread polls its works' events
        # while a segment is being captured; under the default global mode
        # that query is illegal and aborts the process ("operation not
        # permitted when stream is capturing"); this thread's own unsafe calls
        # still fail the capture
        g.capture_begin(pool=self.pool, capture_error_mode="thread_local")
        self.cur = g

    def end(self):
        if self.cur is None:
            return
        g, self.cur = self.cur, None
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")   # an empty segment (two collectives in a row) is fine
            g.capture_end()
        self.items.append(("graph", g))

    def abort(self):
        """End a capture interrupted by an exception (the stream must leave
        capture mode before anything else runs on it)."""
        if self.cur is not None:
            try:
                self.end()
            except Exception:  # noqa: BLE001 — the capture is discarded anyway
                self.cur = None
        self.items = []

    def collective(self, fn: Callable, async_op: bool, desc: Optional[Tuple] = None):
        """Cut the current segment; ``fn()`` issues the collective at replay.
        ``desc`` = (kind, input, output, process group, group-local root)
        lets the native replayer issue it without ``fn``."""
        self.end()
        slot = None
        if async_op:
            slot = self.n_async
            self.n_async += 1
        self.items.append(("coll", fn, slot, desc))
        self.begin()
        return _PendingWork(self, slot) if async_op else None

    def wait(self, slot: int):
        self.end()
        self.items.append(("wait", slot))
        self.begin()

    # ---- replay side
    def n_graphs(self) -> int:
        return sum(1 for it in self.items if it[0] == "graph")

    def n_collectives(self) -> int:
        return sum(1 for it in self.items if it[0] == "coll")

    def build_native(self) -> bool:
        """Hand the chain to the native replayer; False (Python walk) when the
        extension is absent or a collective has no descriptor."""
        R = _native_module()
        if R is None:
            return False
        rp = R.Replayer()
        for it in self.items:
            if it[0] == "graph":
                rp.add_graph(it[1])
            elif it[0] == "coll":
                desc = it[3]
                if desc is not None and desc[0] == "send_recv":
                    # replay.cpp kSendRecv (ncclGroupStart/End through c10d
                    # coalescing) is opt-in until it has run on more than one
                    # GPU; by default the step keeps torch's batch_isend_irecv
                    if os.environ.get("FF_NATIVE_SENDRECV", "0") != "1":
                        return False
                    _, sends, recvs, pg = desc[:4]
                    try:
                        rp.add_send_recv(pg, [int(p) for p, _ in sends], [t for _, t in sends],
                                         [int(p) for p, _ in recvs], [t for _, t in recvs],
                                         -1 if it[2] is None else int(it[2]))
                    except (TypeError, AttributeError):
                        return False
                    continue
                if desc is None or desc[0] not in NATIVE_KINDS:
                    return False
                kind, a, b, pg, root = desc[:5]
                out_splits, in_splits = (desc[5], desc[6]) if len(desc) > 6 else ([], [])
                try:
                    rp.add_collective(NATIVE_KINDS[kind], pg, a, a if b is None else b, int(root),
                                      -1 if it[2] is None else int(it[2]), [int(v) for v in out_splits],
                                      [int(v) for v in in_splits])
                except TypeError:   # not a c10d ProcessGroup (e.g. a non-member sentinel)
                    return False
            else:
                rp.add_wait(int(it[1]))
        self._native = rp
        return True

    @property
    def native(self) -> bool:
        return self._native is not None

    def replay(self):
        if self._native is not None:
            self._native.replay()
            return
        works = {}
        for it in self.items:
            kind = it[0]
            if kind == "graph":
                it[1].replay()
            elif kind == "coll":
                w = it[1]()
                if it[2] is not None:
                    works[it[2]] = w
            else:
                w = works.pop(it[1], None)
                if w is not None:
                    w.wait()
        for w in works.values():   # never waited inside the step: keep stream order anyway
            if w is not None:
                w.wait()
