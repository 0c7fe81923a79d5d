"""Python helpers over the native machine/cost/simulator/search bindings.

* ``machine_spec(ffconfig)``: MI355X defaults, overridden by
  ``--machine-model-file`` (JSON with MachineSpecification fields — the
  analogue of the reference's EnhancedMachineModel config file,
  machine_config_example:1-60).
* ``cost_model(ffconfig)``: analytic MI355X model plus an optional measured
  profile table (``FF_PROFILE_TABLE`` / ``ffconfig.profile_table_file``,
  written by tools/profile_ops.py) — the reference's measure_operator_cost
  cache (simulator.cc:531-571).
* ``simulate(pcg, ...)`` / ``machine_mapping(...)`` / ``sp_decomposition``
  return parsed Python structures.
"""
from __future__ import annotations

import json
import os
from typing import Dict, Optional, Sequence, Tuple

from .. import _ffcore as C


def machine_spec(ffconfig=None, world: Optional[int] = None):
    """MachineSpecification for the search.  ``--machine-model-file``: JSON
    with MachineSpecification fields, or a reference-style ``key = value``
    machine config (machine_config_example).  ``--machine-model-version 1``
    (or any key=value file) runs the topology-aware network model
    (csrc/ffcore/src/network.cc) and calibrates the per-group-size
    collective bandwidths from its routed ring / all-to-all link loads."""
    spec = C.MachineSpecification.mi355x()
    path = getattr(ffconfig, "machine_model_file", "") if ffconfig is not None else ""
    version = int(getattr(ffconfig, "machine_model_version", 0) or 0) if ffconfig is not None else 0
    topo = None
    if path:
        with open(path) as f:
            text = f.read()
        if text.lstrip().startswith("{"):
            spec = C.MachineSpecification.from_json(text)
        else:
            topo, spec = C.NetworkTopology.from_config_text(text)
    if ffconfig is not None:
        nn = getattr(ffconfig, "search_num_nodes", -1)
        if nn and nn > 0:
            spec.num_nodes = nn
        nw = getattr(ffconfig, "search_num_workers", -1)
        if nw and nw > 0:
            spec.num_gpus_per_node = nw
    if world is not None and world > spec.num_devices():
        spec.num_nodes = (world + spec.num_gpus_per_node - 1) // spec.num_gpus_per_node
    if topo is None and version >= 1:
        topo = C.NetworkTopology.mi355x_cluster(spec.num_nodes, spec.num_gpus_per_node, spec.xgmi_link_bandwidth,
                                                1e-6, spec.inter_node_bandwidth, 5e-6)
    if topo is not None:
        spec = C.NetworkModel(topo).calibrate(spec)
    return spec


PROFILE_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                           "profiles")


def cost_model(ffconfig=None, world: Optional[int] = None, use_profiles: bool = True, spec=None):
    """Analytic MI355X model + measured op costs.  Tables: ``FF_PROFILE_TABLE``
    (os.pathsep-separated), ``ffconfig.profile_table_file``, and every
    committed ``profiles/op_costs_*.json`` (keys are exact op/piece
    signatures, so tables for different models/worlds merge safely; where
    two tables hold the same key the later one in the order below wins)."""
    cm = C.CostModel(spec if spec is not None else machine_spec(ffconfig, world))
    if not use_profiles or os.environ.get("FF_NO_PROFILE_TABLES"):
        return cm
    # later tables override earlier entries: committed standalone tables, then
    # committed in-situ ones (measured inside the fused training step), then
    # the tables the user named
    paths = []
    if os.path.isdir(PROFILE_DIR):
        paths += sorted((os.path.join(PROFILE_DIR, f) for f in os.listdir(PROFILE_DIR)
                         if f.startswith("op_costs_") and f.endswith(".json")), key=lambda p: ("insitu" in p, p))
    paths += [p for p in os.environ.get("FF_PROFILE_TABLE", "").split(os.pathsep) if p]
    if ffconfig is not None and getattr(ffconfig, "profile_table_file", ""):
        paths.append(ffconfig.profile_table_file)
    for path in paths:
        if os.path.exists(path):
            with open(path) as f:
                cm.load_profiles(f.read())
    return cm


def sim_config(ffconfig=None, world: int = 1) -> dict:
    cfg = {"world": world}
    if ffconfig is not None:
        cfg["overlap_grad_sync"] = bool(getattr(ffconfig, "search_overlap_backward_update", True))
    return cfg


def plan_memory(pcg, world: int = 1, views: Optional[Dict[int, Sequence[int]]] = None, training: bool = True,
                weight_bytes_per_param: float = 16.0, with_blocks: bool = False,
                live_copies: Optional[Dict[int, float]] = None, act_elem_bytes: float = 0.0,
                executor_fusions: bool = False):
    """Liveness-based memory plan of one step per device
    (csrc/ffcore/src/memory_plan.cc): [{device, weight_bytes,
    peak_live_bytes, arena_bytes, naive_bytes, [blocks]}].  ``live_copies``:
    PCG node -> micro-batches of its activations held live at once (a
    pipeline stage under 1F1B keeps min(m, S - s)).  ``act_elem_bytes``:
    bytes per activation element as stored (2 for bf16 compute; 0 = the PCG
    dtype); ``executor_fusions``: model the executor's fused / saved tensors
    (memory_plan.h)."""
    return json.loads(C.plan_memory(pcg, {int(k): [int(d) for d in v] for k, v in (views or {}).items()}, int(world),
                                    bool(training), float(weight_bytes_per_param), bool(with_blocks),
                                    {int(k): float(v) for k, v in (live_copies or {}).items()},
                                    float(act_elem_bytes), bool(executor_fusions)))


def simulate(pcg, cm, world: int, views: Optional[Dict[int, Sequence[int]]] = None, dot: bool = False,
             network=None, **sim_kw):
    """Simulated iteration; ``views``: PCG node -> placement (device list in
    task order); ``network``: a NetworkModel for routed transfers /
    collectives; ``dot``: also the task list and its dot graph."""
    cfg = {"world": world, **sim_kw}
    res, dot_s = C.simulate(pcg, cm, json.dumps(cfg), {int(k): [int(d) for d in v] for k, v in (views or {}).items()},
                            dot, network)
    out = json.loads(res)
    if dot:
        out["dot"] = dot_s
    return out


def machine_mapping(pcg, cm, world: int, contiguous_only: bool = False):
    """The machine-mapping DP (csrc/ffcore/src/mapping.cc): runtime, and per
    PCG node its placement (device tuple) and MachineView."""
    runtime, feasible, views, rep = C.machine_mapping(pcg, cm, world, contiguous_only)
    rep = json.loads(rep)
    return {"runtime": runtime, "feasible": feasible, "views": {int(k): tuple(v) for k, v in views.items()},
            "machine_views": {int(k): v for k, v in rep.get("machine_views", {}).items()},
            "cache_entries": rep.get("cache_entries", 0)}


def sp_decomposition(graph, strict: bool = False):
    if isinstance(graph, C.ComputationGraph):
        s = C.cg_sp_decomposition(graph, strict)
    else:
        s = C.sp_decomposition(graph, strict)
    return None if s is None else json.loads(s)


def strategy_speedup_report(cg, world: int, ffconfig=None, strategy_pcg=None, views=None) -> dict:
    """Simulated iteration time of data parallel vs a given PCG."""
    cm = cost_model(ffconfig, world)
    dp = C.data_parallel_pcg(cg, world)
    t_dp = simulate(dp, cm, world)["iteration_time"]
    out = {"dp_iteration_time": t_dp}
    if strategy_pcg is not None:
        t = simulate(strategy_pcg, cm, world, views)["iteration_time"]
        out["iteration_time"] = t
        out["predicted_speedup_over_dp"] = t_dp / t if t > 0 else None
    return out
