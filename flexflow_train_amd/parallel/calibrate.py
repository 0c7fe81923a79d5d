"""Self-calibration of the collective cost model from measured RCCL times.

The reference prices NCCL gradient syncs and ring all-reduces over modelled
links (lib/runtime/src/simulator.cc:1087-1215 per-op sync ``2 piece/bw``,
:1684-1795 ring expansion of all-reduce) with link parameters taken from a
machine-model file.  Here the multi-GPU run measures the collectives it is
about to use, at the message sizes its step actually issues (gradient
buckets, redistribution all-to-alls / all-gathers), on the live process
group, and fits the cost model's latency (alpha) and effective bus bandwidth
(beta) per collective kind to those times:

    all_reduce      t = a_ar + 2 (p - 1) / p * bytes / bw_ar
    all_gather      t = a    +     (p - 1) / p * bytes / bw_ag      (bytes of the gathered result)
    reduce_scatter  t = a    +     (p - 1) / p * bytes / bw_rs      (bytes of the full input)
    all_to_all      t = a    +     (p - 1) / p * bytes / bw_a2a     (bytes per rank)

(the forms of ``CollectiveCost`` in csrc/ffcore/src/machine.cc).  The fitted
values go into ``MachineSpecification.collective_latency`` /
``collective_bw[p]`` / ``all_to_all_bw[p]``, so the simulator's prediction of
the step can be compared with the measured step time (bench.py emits
``comm_measured`` / ``comm_simulated`` and the predicted-vs-measured step).

Every rank takes part in every measurement (collectives); times are the max
over ranks of the mean of ``iters`` back-to-back calls.  ``timer`` can be
injected (tests use a fake clock).
"""
from __future__ import annotations

import time
from typing import Callable, Dict, List, Optional, Sequence

import torch

KINDS = ("all_reduce", "all_gather", "reduce_scatter", "all_to_all")


def _factor(kind: str, p: int) -> float:
    """Bytes-on-the-busiest-link multiplier of each collective (ring forms)."""
    if kind == "all_reduce":
        return 2.0 * (p - 1) / p
    return (p - 1.0) / p


def step_message_sizes(ex, cap: int = 256 << 20) -> Dict[str, List[int]]:
    """The message sizes (bytes) a distributed training step issues: the
    gradient buckets' all-reduces (or reduce-scatter + all-gather under the
    sharded optimizer) and the redistribution collectives recorded by the
    executor's DistContext (``ex.dist.msg_sizes`` when the step ran once)."""
    sizes: Dict[str, set] = {k: set() for k in KINDS}
    for f in getattr(ex, "flats", []):
        g = f.get("grad")
        if g is None:
            continue
        esz = g.element_size()
        for b in f.get("buckets", []):
            n = int(b.get("hi", 0)) - int(b.get("lo", 0))
            if n <= 0:
                continue
            if f.get("zero"):
                sizes["reduce_scatter"].add(min(cap, n * esz))
                sizes["all_gather"].add(min(cap, n * 4))
            else:
                sizes["all_reduce"].add(min(cap, n * esz))
    for kind, n in getattr(getattr(ex, "dist", None), "msg_sizes", {}).items():
        if kind in sizes:
            sizes[kind].update(min(cap, int(v)) for v in n)
    return {k: sorted(v) for k, v in sizes.items() if v}


def _sample_sizes(used: Sequence[int]) -> List[int]:
    """Two or three sizes spanning what the step uses (a small one fixes the
    latency term, the largest the bandwidth term)."""
    out = {1 << 20}
    if used:
        out.add(max(used))
        out.add(sorted(used)[len(used) // 2])
    out.add(16 << 20)
    return sorted(s for s in out if s > 0)


def _event_timer(device: torch.device) -> Callable[[Callable[[], None], int], float]:
    def timer(fn, iters):
        if device.type == "cuda":
            torch.cuda.synchronize(device)
            s = torch.cuda.Event(enable_timing=True)
            e = torch.cuda.Event(enable_timing=True)
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
    return timer


def measure(dist_ctx, sizes: Dict[str, Sequence[int]], device: torch.device, iters: int = 5, warmup: int = 2,
            timer: Optional[Callable] = None) -> List[dict]:
    """Time each collective kind at each size on the whole world group.
    Returns [{"kind", "bytes", "p", "ms"}] (ms = max over ranks).  With an
    injected ``timer(kind, nbytes, p) -> ms`` nothing is issued (tests)."""
    import torch.distributed as dist
    p = dist_ctx.world
    clock = _event_timer(device)
    out = []
    for kind in KINDS:
        for nbytes in sizes.get(kind, ()):
            n = max(p, int(nbytes) // 4 // p * p)        # fp32 elements, divisible by p
            if timer is not None:
                out.append({"kind": kind, "bytes": n * 4, "p": p, "ms": float(timer(kind, n * 4, p))})
                continue
            if kind == "all_reduce":
                t = torch.ones(n, device=device)
                fn = (lambda t=t: dist.all_reduce(t))
            elif kind == "all_gather":
                src = torch.ones(n // p, device=device)
                dst = torch.empty(n, device=device)
                fn = (lambda s=src, d=dst: dist.all_gather_into_tensor(d, s))
            elif kind == "reduce_scatter":
                src = torch.ones(n, device=device)
                dst = torch.empty(n // p, device=device)
                fn = (lambda s=src, d=dst: dist.reduce_scatter_tensor(d, s))
            else:
                src = torch.ones(n, device=device)
                dst = torch.empty(n, device=device)
                fn = (lambda s=src, d=dst: dist.all_to_all_single(d, s))
            for _ in range(warmup):
                fn()
            ms = dist_ctx.max_scalar(float(clock(fn, iters)))
            out.append({"kind": kind, "bytes": n * 4, "p": p, "ms": ms})
            del fn
    return out


def fit(samples: List[dict]) -> Dict[str, dict]:
    """Least-squares fit of t = a + factor * bytes / bw per kind (>= 2 sizes;
    one size: bandwidth from that point with the smallest-size latency of
    the other kinds, or zero)."""
    by: Dict[str, List[dict]] = {}
    for s in samples:
        by.setdefault(s["kind"], []).append(s)
    res: Dict[str, dict] = {}
    for kind, ss in by.items():
        p = ss[0]["p"]
        xs = [_factor(kind, p) * s["bytes"] for s in ss]     # busiest-link bytes
        ys = [s["ms"] * 1e-3 for s in ss]
        if len(ss) >= 2 and max(xs) > min(xs):
            mx, my = sum(xs) / len(xs), sum(ys) / len(ys)
            sxx = sum((x - mx) ** 2 for x in xs)
            slope = sum((x - mx) * (y - my) for x, y in zip(xs, ys)) / sxx
            a = my - slope * mx
        else:
            slope, a = ys[0] / max(xs[0], 1.0), 0.0
        slope = max(slope, 1e-15)
        res[kind] = {"p": p, "latency_s": max(0.0, a), "bw_bytes_per_s": 1.0 / slope}
    return res


def calibrated_spec(spec, fits: Dict[str, dict]):
    """A copy of ``spec`` with the fitted latency / bandwidths for group size
    p.  collective_latency = the all-reduce fit's latency mapped back through
    CollectiveCost's alpha terms (2 (p - 1) / 4 + 1 per all-reduce, 1 per
    other collective), averaged over the kinds measured."""
    from .. import _ffcore as C
    out = C.MachineSpecification.from_json(spec.to_json())
    alphas = []
    bw = dict(out.collective_bw)
    a2a = dict(out.all_to_all_bw)
    for kind, f in fits.items():
        p = int(f["p"])
        if kind == "all_reduce":
            alphas.append(f["latency_s"] / (2.0 * (p - 1) / 4.0 + 1.0))
            bw[p] = f["bw_bytes_per_s"]
        elif kind == "all_to_all":
            alphas.append(f["latency_s"])
            a2a[p] = f["bw_bytes_per_s"]
        else:
            alphas.append(f["latency_s"])
            bw.setdefault(p, f["bw_bytes_per_s"])
    if alphas:
        out.collective_latency = float(sum(alphas) / len(alphas))
    out.collective_bw = bw
    out.all_to_all_bw = a2a
    return out


def comparison(samples: List[dict], nominal, calibrated) -> List[dict]:
    """measured vs the cost model before / after calibration, per sample."""
    from .. import _ffcore as C
    rows = []
    for s in samples:
        rows.append({"kind": s["kind"], "bytes": s["bytes"], "p": s["p"], "measured_ms": round(s["ms"], 4),
                     "simulated_ms": round(C.collective_cost(s["kind"], float(s["bytes"]), s["p"], nominal) * 1e3, 4),
                     "calibrated_ms": round(C.collective_cost(s["kind"], float(s["bytes"]), s["p"], calibrated) * 1e3,
                                            4)})
    return rows


def calibrate_for_step(ex, iters: int = 5, timer: Optional[Callable] = None) -> dict:
    """Measure the collectives of ``ex``'s step on its process group, fit the
    model, and return {"samples", "fits", "sizes_used", "spec_nominal",
    "spec_calibrated", "comparison"} (spec_* as MachineSpecification)."""
    from ..search.native import machine_spec
    sizes_used = step_message_sizes(ex)
    if timer is None:
        # every rank must issue the same collectives at the same sizes: the
        # union over ranks (redistribution messages differ from rank to rank)
        import torch.distributed as dist
        if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
            everyone = [None] * dist.get_world_size()
            dist.all_gather_object(everyone, sizes_used)
            merged: Dict[str, set] = {}
            for d in everyone:
                for k, v in (d or {}).items():
                    merged.setdefault(k, set()).update(v)
            sizes_used = {k: sorted(v) for k, v in merged.items()}
    sizes = {k: _sample_sizes(sizes_used.get(k, [])) for k in KINDS}
    samples = measure(ex.dist, sizes, ex.cfg.device, iters=iters, timer=timer)
    fits = fit(samples)
    nominal = machine_spec(None, ex.world)
    cal = calibrated_spec(nominal, fits)
    return {"samples": samples, "fits": fits, "sizes_used": sizes_used, "spec_nominal": nominal,
            "spec_calibrated": cal, "comparison": comparison(samples, nominal, cal)}


def predicted_step_ms(pcg, views, world: int, spec, ffconfig=None) -> float:
    """The event simulator's iteration time for ``pcg`` under ``spec`` (with
    the committed measured op-cost tables, as the search uses)."""
    from ..search import native
    cm = native.cost_model(ffconfig, world, spec=spec)
    kw = {k: v for k, v in native.sim_config(ffconfig, world).items() if k != "world"}
    res = native.simulate(pcg, cm, world, views or {}, **kw)
    return float(res.get("iteration_time", 0.0)) * 1e3


def summary(cal: dict, pcg=None, views=None, world: int = 1, measured_ms: Optional[float] = None,
            ffconfig=None) -> dict:
    """The JSON-able record bench.py emits: fitted parameters, per-sample
    measured vs modelled times, and the predicted vs measured step."""
    out = {"fits": {k: {"latency_us": round(v["latency_s"] * 1e6, 2), "bw_GBps": round(v["bw_bytes_per_s"] / 1e9, 2)}
                    for k, v in cal["fits"].items()},
           "sizes_used": {k: v[:8] for k, v in cal["sizes_used"].items()},
           "comm": cal["comparison"]}
    if pcg is not None:
        try:
            out["predicted_ms_nominal"] = round(predicted_step_ms(pcg, views, world, cal["spec_nominal"], ffconfig), 3)
            out["predicted_ms_calibrated"] = round(predicted_step_ms(pcg, views, world, cal["spec_calibrated"],
                                                                     ffconfig), 3)
        except Exception as e:  # noqa: BLE001 -- the record must not cost the run
            out["predict_error"] = f"{type(e).__name__}: {e}"[:200]
    if measured_ms is not None:
        out["measured_ms"] = round(measured_ms, 3)
    return out
