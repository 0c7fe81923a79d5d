#!/usr/bin/env python3
"""Strategy-search predictions for the BASELINE.json configs: the simulated
iteration time of the searched strategy vs pure data parallelism on N
MI355X GPUs (the reference's "speedup over DP after search" protocol,
scripts/osdi22ae/*.sh), plus which layers left data parallelism.  Runs on the
CPU (cost model + simulator only); one JSON line per (config, world)."""
import argparse
import collections
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from flexflow_train_amd import _ffcore as C  # noqa: E402
from flexflow_train_amd import models as Z  # noqa: E402
from flexflow_train_amd.core import FFConfig, FFModel  # noqa: E402
from flexflow_train_amd.models.bert import bert_large, build_bert  # noqa: E402
from flexflow_train_amd.search import unity  # noqa: E402

CONFIGS = {
    # name: (builder(model, global_batch), per-GPU batch): bench.py's per-GPU
    # batches, so a prediction lines up with the driver's weak-scaling runs
    "bert-large": (lambda m, B: build_bert(m, bert_large(batch_size=B, sequence_length=512)), 64),
    "bert-large-ae": (lambda m, B: build_bert(m, bert_large(batch_size=B, sequence_length=512)), 2),  # AE: batch 8 on 4 GPUs
    "gpt3-medium": (lambda m, B: Z.build("gpt", m, batch_size=B, hidden_size=1024, num_layers=24, num_heads=16,
                                         sequence_length=2048), 16),
    "dlrm": (lambda m, B: Z.build("dlrm", m, batch_size=B, embedding_size=[1000000] * 8, mlp_bot=[64, 512, 512, 64],
                                  mlp_top=[576, 1024, 1024, 1024, 1]), 1024),
    "mlp_unify": (lambda m, B: Z.build("mlp_unify", m, batch_size=B), 8),
    "resnet50": (lambda m, B: Z.build("resnet50", m, batch_size=B, image_size=224, num_classes=1000), 256),
}


def layer_kinds(pcg):
    """Count of operator layers by (batch, model) parallel degrees."""
    cnt = collections.Counter()
    for n in pcg.topo_order():
        op = pcg.layer_op(n)
        if op.op_type in ("INPUT", "WEIGHT") or pcg.is_weight_path(n) or C.is_parallel_op(op.type):
            continue
        ps = pcg.shape(C.ValueRef(n, 0))
        cnt[f"shard{list(ps.shard_degrees())}/sum{ps.sum_degree}/copy{ps.discard_copy_degree}"] += 1
    return dict(cnt.most_common(6))


# simulator calibration: the four BASELINE bench configs at bench.py's per-GPU
# batch on one GPU (data parallel, the measured strategy), with the optimizer
# the bench runs: (builder, per-GPU batch, optimizer update bytes / param,
# row-sparse embedding update)
CALIB = {
    "bert-large": (lambda m, B: build_bert(m, bert_large(batch_size=B, sequence_length=512)), 64, 30.0, False),
    "gpt3-medium": (lambda m, B: Z.build("gpt", m, batch_size=B, hidden_size=1024, num_layers=24, num_heads=16,
                                         sequence_length=2048), 16, 30.0, False),
    "resnet50": (lambda m, B: Z.build("resnet50", m, batch_size=B, image_size=224, num_classes=1000), 256, 22.0,
                 False),
    "dlrm": (lambda m, B: Z.build("dlrm", m, batch_size=B, embedding_size=[1000000] * 8, sparse_feature_size=64,
                                  mlp_bot=[64, 512, 512, 64], mlp_top=[576, 1024, 1024, 1024, 1]), 1024, 14.0, True),
}


def calibrate(calib_dir, names, out_path=None):
    """Simulated vs measured 1-GPU step time per config.  Cost tables: every
    ``op_costs_*.json`` in ``calib_dir`` (measured on the box that ran the
    bench) on top of the committed ones; measured: ``bench_<config>.json``
    (bench.py --strategy dp) in the same directory."""
    from flexflow_train_amd.search import native
    # standalone per-op tables first, in-situ tables (op_costs_*_insitu*.json)
    # last so their entries win
    tables = sorted((os.path.join(calib_dir, f) for f in os.listdir(calib_dir)
                     if f.startswith("op_costs_") and f.endswith(".json")), key=lambda p: ("insitu" in p, p))
    rows = []
    for name in names:
        build, bpg, upd, sparse = CALIB[name]
        m = FFModel(FFConfig())
        build(m, bpg)
        pcg = C.data_parallel_pcg(m.cg, 1)
        cm = native.cost_model(world=1, use_profiles=False)
        for t in tables:
            with open(t) as fh:
                cm.load_profiles(fh.read())
        sim = native.simulate(pcg, cm, 1, update_bytes_per_param=upd, sparse_embedding_update=sparse)
        # the analytic MI355X model alone (no measured entries)
        ana = native.simulate(pcg, native.cost_model(world=1, use_profiles=False), 1, update_bytes_per_param=upd,
                              sparse_embedding_update=sparse)
        measured = None
        bpath = os.path.join(calib_dir, f"bench_{name}.json")
        if os.path.exists(bpath):
            for line in open(bpath):
                line = line.strip()
                if line.startswith("{"):
                    measured = json.loads(line).get("ms_per_step")
        row = {"config": name, "per_gpu_batch": bpg, "world": 1, "simulated_ms": round(1000 * sim["iteration_time"], 3),
               "sim_forward_ms": round(1000 * sim["forward_time"], 3),
               "sim_backward_end_ms": round(1000 * sim["backward_end"], 3),
               "sim_update_ms": round(1000 * sim["update_time"], 3), "measured_ms": measured,
               "error_pct": (round(100.0 * (1000 * sim["iteration_time"] - measured) / measured, 2)
                             if measured else None),
               "analytic_ms": round(1000 * ana["iteration_time"], 3),
               "analytic_error_pct": (round(100.0 * (1000 * ana["iteration_time"] - measured) / measured, 2)
                                      if measured else None),
               "tables": [os.path.basename(t) for t in tables]}
        rows.append(row)
        print(json.dumps(row), flush=True)
    if out_path:
        with open(out_path, "w") as f:
            for r in rows:
                f.write(json.dumps(r) + "\n")
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default=",".join(CONFIGS))
    ap.add_argument("--worlds", default="4,8")
    ap.add_argument("--budget", type=int, default=400)
    ap.add_argument("--micro-batches", type=int, default=1,
                    help="micro-batches per step: pipeline-parallel candidates priced at this count")
    ap.add_argument("--calibrate", default="", help="directory with op_costs_*.json + bench_<config>.json: "
                    "simulated vs measured 1-GPU step time of the bench configs")
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    if args.calibrate:
        names = [c for c in args.configs.split(",") if c in CALIB] if args.configs != ",".join(CONFIGS) \
            else list(CALIB)
        calibrate(args.calibrate, names, args.out or None)
        return
    for name in args.configs.split(","):
        build, bpg = CONFIGS[name]
        for world in [int(w) for w in args.worlds.split(",")]:
            cfg = FFConfig()
            cfg.batch_size = bpg * world
            cfg.search_budget = args.budget
            cfg.micro_batches = args.micro_batches
            m = FFModel(cfg)
            build(m, bpg * world)
            t0 = time.time()
            pcg, views, rep = unity.search(m.cg, cfg, world)
            print(json.dumps({"config": name, "world": world, "global_batch": bpg * world,
                              "dp_ms": round(1000 * rep["data_parallel_cost"], 3),
                              "searched_ms": round(1000 * rep["cost"], 3),
                              "predicted_speedup_over_dp": round(rep["predicted_speedup_over_dp"], 3),
                              "algorithm": rep.get("algorithm"), "search_s": round(time.time() - t0, 1),
                              "micro_batches": args.micro_batches, "pipeline_stages": rep.get("pipeline_stages"),
                              "mapped_states": rep.get("mapped_states"),
                              "views": len(views), "layer_degrees": layer_kinds(pcg)}), flush=True)


if __name__ == "__main__":
    main()
