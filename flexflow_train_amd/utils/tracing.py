"""Per-operator tracing and chrome://tracing export.

Parity: the reference's profiling wrapper (lib/kernels/include/kernels/
profiling.h:10-49: events around warm-up + measured iterations, logged as
"[Linear] forward_time = ...ms" by local-execution/profiling.h:11-20) and the
simulator's task-graph export (--taskgraph).  Here the executor brackets
every forward / backward operator and every redistribution with a ``span``:

* on GPU, two HIP events per span recorded on the current stream — nothing
  synchronises while the step runs; events are resolved when a report or
  trace is requested;
* on CPU, wall-clock stamps.

``report()`` aggregates milliseconds per ``name:phase``; ``export_chrome_trace``
writes a Trace-Event-Format JSON (one process per rank, one thread per
category) that chrome://tracing / Perfetto load directly.  Kernel-level
timelines come from ``rocprofv3 --kernel-trace`` (see tools/prof_summary.py).
"""
from __future__ import annotations

import json
import time
from typing import Dict, List, Optional

import torch


class Tracer:
    def __init__(self, device: torch.device, rank: int = 0, enabled: bool = False):
        self.device = device
        self.rank = rank
        self.enabled = enabled
        self.gpu = device.type == "cuda"
        self.spans: List[list] = []     # [name, cat, step, start, end]
        self._t0 = None

    def clear(self):
        self.spans = []
        self._t0 = None

    def begin(self, name: str, cat: str = "compute", step: int = 0):
        if not self.enabled:
            return None
        if self.gpu:
            if torch.cuda.is_current_stream_capturing():
                return None   # spans inside a hipGraph capture would replay without being read
            s = torch.cuda.Event(enable_timing=True)
            s.record()
        else:
            s = time.perf_counter()
        rec = [name, cat, step, s, None]
        self.spans.append(rec)
        return rec

    def end(self, rec):
        if rec is None:
            return
        if self.gpu:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            rec[4] = e
        else:
            rec[4] = time.perf_counter()

    def _resolved(self):
        """[(name, cat, step, start_ms, dur_ms)] relative to the first span."""
        if not self.spans:
            return []
        if self.gpu:
            torch.cuda.synchronize(self.device)
            first = self.spans[0][3]
            out = []
            for name, cat, step, s, e in self.spans:
                if e is None:
                    continue
                out.append((name, cat, step, first.elapsed_time(s), s.elapsed_time(e)))
            return out
        first = self.spans[0][3]
        return [(n, c, st, (s - first) * 1e3, (e - s) * 1e3) for n, c, st, s, e in self.spans if e is not None]

    def report(self) -> Dict[str, float]:
        agg: Dict[str, float] = {}
        for name, _cat, _step, _s, d in self._resolved():
            agg[name] = agg.get(name, 0.0) + d
        return dict(sorted(agg.items(), key=lambda kv: -kv[1]))

    def export_chrome_trace(self, path: str, extra: Optional[dict] = None):
        events = []
        tids = {}
        for name, cat, step, s, d in self._resolved():
            tid = tids.setdefault(cat, len(tids))
            events.append({"name": name, "cat": cat, "ph": "X", "pid": self.rank, "tid": tid,
                           "ts": s * 1e3, "dur": max(d, 0.0) * 1e3, "args": {"step": step}})
        for cat, tid in tids.items():
            events.append({"name": "thread_name", "ph": "M", "pid": self.rank, "tid": tid, "args": {"name": cat}})
        events.append({"name": "process_name", "ph": "M", "pid": self.rank, "args": {"name": f"rank {self.rank}"}})
        doc = {"traceEvents": events, "displayTimeUnit": "ms", "otherData": extra or {}}
        with open(path, "w") as f:
            json.dump(doc, f)
        return path
