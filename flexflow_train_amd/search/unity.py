"""Strategy search entry point used by FFModel.compile().

Runs the native search (csrc/ffcore/src/search.cc) on rank 0 and
broadcasts the chosen PCG + placement to every rank, so all ranks execute
the same strategy even when the search is time-bounded.

Algorithms (``FFConfig.search_algorithm``):
  * ``unity``  — MCMC over per-layer parallel configs, then Unity best-first
    refinement over PCG substitutions (reference: unity_algorithm.cc:27-91,
    legacy strategy_search_task);
  * ``mcmc``   — MCMC only;
  * ``data_parallel`` handled by strategy.build_pcg.

The report carries the simulated data-parallel and searched iteration times
and their ratio (``predicted_speedup_over_dp``), the reference's headline
"speedup over DP after search".
"""
from __future__ import annotations

import json
import os
from typing import Dict, Tuple

from .. import _ffcore as C
from . import native


DEFAULT_RULES = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "data", "taso_rules.json")


def substitution_path(ffconfig) -> str:
    """The Unity rule-set file FFConfig asks for ("" -> the bundled TASO
    corpus, "none" -> no rule set)."""
    p = getattr(ffconfig, "substitution_json_path", "") or ""
    if p.lower() == "none":
        return ""
    if not p:
        return DEFAULT_RULES if os.path.exists(DEFAULT_RULES) else ""
    if not os.path.exists(p):
        raise FileNotFoundError(f"--substitution-json {p}: no such file")
    return p


def _search_local(cg, ffconfig, world: int):
    cm = native.cost_model(ffconfig)
    budget = ffconfig.search_budget if ffconfig.search_budget and ffconfig.search_budget > 0 else 400
    cfg = {
        "world": world,
        "budget": budget,
        "alpha": float(ffconfig.search_alpha),
        "time_limit": float(getattr(ffconfig, "search_time_limit", 45.0)),
        "enable_parameter_parallel": True,
        "enable_attribute_parallel": bool(ffconfig.enable_attribute_parallel),
        "seed": int(ffconfig.seed) & 0x7FFFFFFF,
        "sim": native.sim_config(ffconfig, world),
        # Unity expands as many states as the reference's single --budget
        # (unity_algorithm.cc:37-90), over the built-in rules + the rule set
        "unity_budget": budget,
        "substitution_path": substitution_path(ffconfig),
        # pipeline-parallel stage splits priced against the other strategies
        # at equal work: micro_batches batches per optimizer step
        "micro_batches": max(1, int(getattr(ffconfig, "micro_batches", 1) or 1)),
        "pipeline": True,
    }
    algo = ffconfig.search_algorithm
    if algo == "mcmc":
        pcg, rep, views = C.mcmc_search(cg, cm, json.dumps(cfg))
    else:
        pcg, rep, views = C.graph_optimize(cg, cm, json.dumps(cfg))
    rep = json.loads(rep)
    rep["source"] = "search:" + rep.get("algorithm", algo)
    return pcg, {int(k): tuple(v) for k, v in views.items()}, rep


def search(cg, ffconfig, world: int):
    import torch.distributed as dist

    distributed = dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1
    if not distributed or dist.get_rank() == 0:
        pcg, views, rep = _search_local(cg, ffconfig, world)
        payload = [pcg.to_json(), {str(k): list(v) for k, v in views.items()}, rep]
    else:
        payload = [None, None, None]
    if distributed:
        dist.broadcast_object_list(payload, src=0)
    pcg = C.ParallelComputationGraph.from_json(payload[0])
    views: Dict[int, Tuple[int, ...]] = {int(k): tuple(v) for k, v in payload[1].items()}
    rep = payload[2]
    # a predicted gain inside the cost model's error (the calibrated
    # simulator is within ~3 % of measured steps) does not pay for running a
    # strategy other than data parallelism: keep DP below search_min_speedup
    pred = rep.get("predicted_speedup_over_dp") if isinstance(rep, dict) else None
    min_gain = float(getattr(ffconfig, "search_min_speedup", 1.0) or 1.0)
    if world > 1 and pred is not None and float(pred) < min_gain:
        pcg = C.data_parallel_pcg(cg, world)
        views = {}
        rep = dict(rep)
        rep["kept_data_parallel"] = f"predicted speedup {float(pred):.4f} < search_min_speedup {min_gain:g}"
    return pcg, views, rep
