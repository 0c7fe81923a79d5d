"""Measured operator costs for the search (the reference's
LocalCostEstimator, lib/local-execution/src/local_cost_estimator.cc:29-105,
and the legacy Simulator::measure_operator_cost cache, simulator.cc:531-571).

For every distinct (operator, per-device piece shapes) of a set of PCGs a
one-operator graph is executed on the local GPU through the real Executor
(same kernels, fused epilogues and bf16 weight-gradient paths as training)
and forward / backward times are recorded under
``CostModel.signature(op, input pieces + output pieces)`` — the key the C++
cost model looks up.  Parallel / input / weight ops are not profiled (their
cost is the xGMI collective model).
"""
from __future__ import annotations

import json
import time
from typing import Dict, Iterable, List, Optional, Tuple

import torch

from .. import _ffcore as C
from ..parallel.comm import DistContext
from ..runtime.executor import ExecConfig, Executor

_SKIP = {"INPUT", "WEIGHT", "REPARTITION", "COMBINE", "REPLICATE", "REDUCTION", "ALLTOALL", "FUSED_PARALLEL", "NOOP"}


def _pieces(pcg, node) -> Tuple[List, List]:
    ins = [pcg.shape(v).piece_shape() for v in pcg.layer_data_inputs(node)]
    outs = [pcg.shape(C.ValueRef(node, k)).piece_shape() for k in range(pcg.num_outputs(node))]
    return ins, outs


def collect_signatures(pcgs: Iterable) -> Dict[str, Tuple]:
    """signature -> (op attrs, input piece shapes) over every compute node."""
    out: Dict[str, Tuple] = {}
    for pcg in pcgs:
        for n in pcg.topo_order():
            op = pcg.layer_op(n)
            if op.op_type in _SKIP or pcg.is_weight_path(n):
                continue
            ins, outs = _pieces(pcg, n)
            sig = C.CostModel.signature(op, ins + outs)
            if sig not in out:
                out[sig] = (op, ins)
    return out


def _one_op_pcg(op, in_shapes):
    p = C.ParallelComputationGraph()
    vals = []
    for i, s in enumerate(in_shapes):
        vals.append(p.add_input(C.ParallelTensorShape(list(s.dims), [1] * len(s.dims), 1, 1, s.dtype), True,
                                f"in{i}"))
    outs = p.add_layer_auto_weights(op, vals, "op")
    return p, outs[0]


def _random_input(shape, dtype, op, device):
    dims = tuple(int(d) for d in shape.dims)
    name = C.datatype_to_string(dtype)
    if name.startswith("int"):
        hi = 2
        items = dict(op.items())
        if "num_entries" in items:
            hi = int(items["num_entries"])
        return torch.randint(0, hi, dims, device=device, dtype=torch.int32 if name == "int32" else torch.int64)
    return torch.randn(dims, device=device)


def _measure_memory(ex, feeds, g, device) -> Tuple[float, float]:
    """(resident MB, peak MB) of one eager forward + backward, above the
    allocation the op's inputs and weights already hold: resident = what the
    forward leaves alive for the backward (outputs + saved tensors), peak =
    the caching allocator's high-water mark over forward + backward (the
    reference's TrackedAllocator, local-execution/src/tracked_allocator.cc)."""
    ex._saved, ex._env = {}, {}
    torch.cuda.synchronize(device)
    base = torch.cuda.memory_allocated(device)
    torch.cuda.reset_peak_memory_stats(device)
    ex.forward(feeds, training=True, keep_outputs=True)
    torch.cuda.synchronize(device)
    resident = torch.cuda.memory_allocated(device) - base
    if g is not None:
        ex.backward(g)
    torch.cuda.synchronize(device)
    peak = torch.cuda.max_memory_allocated(device) - base
    ex._saved, ex._env = {}, {}
    return max(0.0, resident / 1e6), max(0.0, peak / 1e6)


def profile_op(op, in_shapes, device: torch.device, dtype=torch.bfloat16, warmup: int = 3,
               iters: int = 10, memory: Optional[dict] = None) -> Tuple[float, float]:
    """(forward ms, backward ms) of one operator on its piece shapes; with a
    ``memory`` dict on a GPU, also its measured resident / peak MB."""
    pcg, out = _one_op_pcg(op, in_shapes)
    ex = Executor(pcg, DistContext(0, 1, device), ExecConfig(compute_dtype=dtype, device=device),
                  output=(out.node, out.idx))
    ex.init_parameters()
    feeds = {f"in{i}": _random_input(s, s.dtype, op, device) for i, s in enumerate(in_shapes)}
    y = ex.forward(feeds, training=True, keep_outputs=True)
    g = torch.randn_like(y.float()).to(y.dtype) if y.is_floating_point() else None

    def fwd():
        ex.forward(feeds, training=True, keep_outputs=True)

    def both():
        ex.forward(feeds, training=True, keep_outputs=True)
        ex.backward(g)

    sync = torch.cuda.synchronize if device.type == "cuda" else (lambda: None)

    def timeit(fn):
        for _ in range(warmup):
            fn()
        sync()
        if device.type == "cuda":
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(iters):
                fn()
            e.record()
            e.synchronize()
            return s.elapsed_time(e) / iters
        t0 = time.perf_counter()
        for _ in range(iters):
            fn()
        return (time.perf_counter() - t0) * 1e3 / iters

    def graph_time(fn):
        """GPU time of ``fn`` replayed from a hipGraph: excludes the host
        launch overhead that the training loop hides by running ahead."""
        fn()
        sync()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            fn()
        torch.cuda.current_stream().wait_stream(s)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, capture_error_mode="thread_local"):
            fn()
        return timeit(graph.replay)

    if device.type == "cuda" and memory is not None:
        memory["resident_mb"], memory["peak_mb"] = _measure_memory(ex, feeds, g, device)
    if device.type == "cuda":
        try:
            t_f = graph_time(fwd)
            t_fb = graph_time(both) if g is not None else t_f
            return t_f, max(0.0, t_fb - t_f)
        except Exception:  # noqa: BLE001 — op not capturable: eager timing
            torch.cuda.synchronize()
    t_f = timeit(fwd)
    t_fb = timeit(both) if g is not None else t_f
    return t_f, max(0.0, t_fb - t_f)


def build_profile_table(pcgs: Iterable, device: torch.device, out_path: Optional[str] = None,
                        existing: Optional[dict] = None, log=print) -> dict:
    table = dict(existing or {})
    sigs = collect_signatures(pcgs)
    for i, (sig, (op, ins)) in enumerate(sigs.items()):
        if sig in table:
            continue
        mem: dict = {}
        try:
            f, b = profile_op(op, ins, device, memory=mem)
        except Exception as e:  # noqa: BLE001 — unsupported op on this device: analytic fallback
            log(f"[profile] skip {op.op_type}: {type(e).__name__}: {str(e)[:120]}")
            continue
        table[sig] = {"fwd_ms": round(f, 5), "bwd_ms": round(b, 5), **{k: round(v, 3) for k, v in mem.items()}}
        log(f"[profile] {i + 1}/{len(sigs)} {op.op_type:<22} fwd {f:8.4f} ms  bwd {b:8.4f} ms"
            + (f"  resident {mem['resident_mb']:.1f} MB  peak {mem['peak_mb']:.1f} MB" if mem else ""))
        if out_path:
            with open(out_path, "w") as fh:
                json.dump(table, fh, indent=0, sort_keys=True)
    return table
