"""Strategy construction / import / export for FFModel.compile().

Parity: the reference's compile path chooses between a searched strategy
(Unity graph_optimize / legacy MCMC strategy_search_task), the
--only-data-parallel baseline, and --import-strategy; --export-strategy
writes the chosen strategy (bin/arg_parser/arg_parser.cc:42-52,
lib/runtime/src/model.cc compile, examples/cpp/DLRM/strategies/*.pb).

Strategy file (JSON, "ffmi355x.strategy.v1"):
  {"world": N, "pcg": <ParallelComputationGraph v1 JSON>,
   "placements": {"<node>": [device, ...]},      (task order; round <= 3 files:
   "views": {"<node>": [start, block]}, still read)
   "ops": [{"name", "op_type", "device_type": "GPU", "degrees": [...],
            "sum_degree", "discard_copy_degree", "device_ids": [...]}]}
The "ops" list mirrors the reference's per-op FFProtoBuf::Strategy records
(keyed by op name) and is informational; the PCG + placements are
authoritative.
A ``.pb`` path reads / writes the reference's protobuf strategy format itself
(legacy_strategy.py), e.g. examples/cpp/DLRM/strategies/*.pb.
"""
from __future__ import annotations

import json
import os
from typing import Dict, Tuple

from .. import _ffcore as C
from ..parallel.layout import block as _block
from ..utils.logging import get_logger
from . import legacy_strategy as legacy


def _cg_to_pcg_map_by_name(cg, pcg) -> Dict[int, int]:
    by_name = {}
    for n in pcg.topo_order():
        nm = pcg.layer_name(n)
        if nm and pcg.layer_op(n).op_type not in ("REPARTITION", "COMBINE", "REPLICATE", "REDUCTION"):
            by_name.setdefault(nm, n)
    out = {}
    for n in cg.topo_order():
        nm = cg.layer_name(n)
        if nm in by_name:
            out[n] = by_name[nm]
    return out


def build_pcg(cg, ffconfig, world: int):
    report = {"world": world}
    if ffconfig.import_strategy_file and legacy.is_legacy_file(ffconfig.import_strategy_file):
        # the reference's FFProtoBuf::Strategy (.pb) files, keyed by op name
        with open(ffconfig.import_strategy_file, "rb") as f:
            pcg, views, rep = legacy.to_pcg(cg, legacy.decode(f.read()), world)
        report.update(rep)
    elif ffconfig.import_strategy_file:
        pcg, views = import_strategy(ffconfig.import_strategy_file, world)
        report["source"] = "import"
    elif world == 1:
        pcg, mapping = C.pcg_from_computation_graph(cg)
        views = {}
        report["source"] = "single_device"
    elif ffconfig.only_data_parallel or ffconfig.search_algorithm == "data_parallel":
        pcg = C.data_parallel_pcg(cg, world)
        views = {}
        report["source"] = "data_parallel"
    else:
        from . import unity

        pcg, views, rep = unity.search(cg, ffconfig, world)
        report.update(rep)
    report["cg_to_pcg"] = _cg_to_pcg_map_by_name(cg, pcg)
    get_logger("search").info("strategy for %d ranks: %s", world,
                              {k: v for k, v in report.items() if k not in ("cg_to_pcg", "trace", "strategy")})
    return pcg, views, report


def export_strategy(path: str, pcg, views: Dict[int, Tuple[int, ...]], report=None):
    if path.endswith(".pb"):
        # the reference's protobuf format (per-op degrees + device ids)
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        with open(path, "wb") as f:
            f.write(legacy.encode(legacy.from_pcg(pcg, views)))
        return
    ops = []
    for n in pcg.topo_order():
        op = pcg.layer_op(n)
        if op.op_type in ("INPUT", "WEIGHT") or pcg.is_weight_path(n):
            continue
        ps = pcg.shape(C.ValueRef(n, 0))
        total = ps.total_parallel_degree()
        ops.append({"name": pcg.layer_name(n), "op_type": op.op_type, "device_type": "GPU",
                    "degrees": list(ps.shard_degrees()), "sum_degree": ps.sum_degree,
                    "discard_copy_degree": ps.discard_copy_degree,
                    "device_ids": legacy.task_devices(views.get(n), total)})
    doc = {"format": "ffmi355x.strategy.v1", "world": (report or {}).get("world"),
           "pcg": json.loads(pcg.to_json()), "placements": {str(k): list(v) for k, v in views.items()},
           "ops": ops}
    if report:
        doc["search"] = {k: v for k, v in report.items() if k != "cg_to_pcg"}
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    with open(path, "w") as f:
        json.dump(doc, f, indent=1)


def import_strategy(path: str, world: int):
    with open(path) as f:
        doc = json.load(f)
    if doc.get("format") != "ffmi355x.strategy.v1":
        raise ValueError(f"{path}: not a strategy file")
    if doc.get("world") not in (None, world):
        raise ValueError(f"{path}: strategy is for {doc['world']} ranks, running on {world}")
    pcg = C.ParallelComputationGraph.from_json(json.dumps(doc["pcg"]))
    if "placements" in doc:
        views = {int(k): tuple(int(d) for d in v) for k, v in doc["placements"].items()}
    else:  # round <= 3 files: contiguous blocks [start, block]
        views = {int(k): _block(int(v[0]), int(v[1])) for k, v in doc.get("views", {}).items()}
    return pcg, views
