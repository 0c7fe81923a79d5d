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
    # name: (builder(model, global_batch), per-GPU batch)
    "bert-large": (lambda m, B: build_bert(m, bert_large(batch_size=B, sequence_length=512)), 32),
    "bert-large-ae": (lambda m, B: build_bert(m, bert_large(batch_size=B, sequence_length=512)), 2),  # AE: batch 8 on 4 GPUs
    "gpt3-medium": (lambda m, B: Z.build("gpt", m, batch_size=B), 8),
    "dlrm": (lambda m, B: Z.build("dlrm", m, batch_size=B, embedding_size=[1000000] * 8, mlp_bot=[64, 512, 512, 64],
                                  mlp_top=[576, 1024, 1024, 1024, 1]), 1024),
    "mlp_unify": (lambda m, B: Z.build("mlp_unify", m, batch_size=B), 8),
    "resnet50": (lambda m, B: Z.build("resnet50", m, batch_size=B, image_size=224, num_classes=1000), 32),
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default=",".join(CONFIGS))
    ap.add_argument("--worlds", default="4,8")
    ap.add_argument("--budget", type=int, default=400)
    args = ap.parse_args()
    for name in args.configs.split(","):
        build, bpg = CONFIGS[name]
        for world in [int(w) for w in args.worlds.split(",")]:
            cfg = FFConfig()
            cfg.batch_size = bpg * world
            cfg.search_budget = args.budget
            m = FFModel(cfg)
            build(m, bpg * world)
            t0 = time.time()
            pcg, views, rep = unity.search(m.cg, cfg, world)
            print(json.dumps({"config": name, "world": world, "global_batch": bpg * world,
                              "dp_ms": round(1000 * rep["data_parallel_cost"], 3),
                              "searched_ms": round(1000 * rep["cost"], 3),
                              "predicted_speedup_over_dp": round(rep["predicted_speedup_over_dp"], 3),
                              "algorithm": rep.get("algorithm"), "search_s": round(time.time() - t0, 1),
                              "views": len(views), "layer_degrees": layer_kinds(pcg)}), flush=True)


if __name__ == "__main__":
    main()
