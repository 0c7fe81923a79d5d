#!/usr/bin/env python3
"""Profile every operator piece the strategy search can choose for a model
and write the measured cost table the C++ cost model loads
(FF_PROFILE_TABLE / FFConfig.profile_table_file).

    python tools/profile_ops.py --model bert-large --world 8 --batch-per-gpu 64 \
        --out profiles/op_costs_bert_large_mi355x.json
    python tools/profile_ops.py --model gpt3-medium | resnet50 | dlrm ...   (bench.py's configs)

Strategies profiled: data parallel, and for every model-parallel degree m
dividing the world the uniform column / row / head-parallel variants (each
layer takes the config if it is valid for it, else data parallel), so the
table covers the pieces MCMC / Unity explore most.
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from flexflow_train_amd import _ffcore as C  # noqa: E402
from flexflow_train_amd.core import FFConfig, FFModel  # noqa: E402
from flexflow_train_amd.search.profiler import build_profile_table  # noqa: E402


def uniform_strategies(cg, world):
    dp = json.loads(C.data_parallel_strategy(cg, world))
    out = [dp]
    names = {cg.layer_name(n): n for n in cg.topo_order()}
    for m in [d for d in range(2, world + 1) if world % d == 0]:
        for kinds in (("column", "heads"), ("row", "heads")):
            s = dict(dp)
            for nm, n in names.items():
                if nm not in s:
                    continue
                cands = [json.loads(c) for c in C.candidate_configs(cg, n, world)]
                pick = [c for c in cands if c["model"] == m and c["kind"] in kinds]
                if pick:
                    s[nm] = pick[0]
            out.append(s)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="bert-large",
                    choices=["bert-large", "bert-base", "gpt3-medium", "resnet50", "dlrm"])
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--batch-per-gpu", type=int, default=0, help="default: bench.py's per-GPU batch")
    ap.add_argument("--seq", type=int, default=512)
    ap.add_argument("--out", required=True)
    args = ap.parse_args()
    m = FFModel(FFConfig())
    if args.model in ("bert-large", "bert-base"):
        from flexflow_train_amd.models.bert import bert_base, bert_large, build_bert
        mk = bert_large if args.model == "bert-large" else bert_base
        build_bert(m, mk(batch_size=(args.batch_per_gpu or 64) * args.world, sequence_length=args.seq))
    else:
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        import bench
        from flexflow_train_amd import models as Z
        zname, bpg, over, _, _ = bench._ZOO[args.model]
        Z.build(zname, m, batch_size=(args.batch_per_gpu or bpg) * args.world, **over)
    pcgs = []
    for s in uniform_strategies(m.cg, args.world):
        try:
            pcgs.append(C.lower_strategy(m.cg, json.dumps(s), args.world)[0])
        except Exception as e:  # noqa: BLE001
            print("skip strategy:", e)
    existing = {}
    if os.path.exists(args.out):
        with open(args.out) as f:
            existing = json.load(f)
    dev = torch.device("cuda:0" if torch.cuda.is_available() else "cpu")
    table = build_profile_table(pcgs, dev, args.out, existing)
    with open(args.out, "w") as f:
        json.dump(table, f, indent=0, sort_keys=True)
    print(f"{len(table)} entries -> {args.out}")


if __name__ == "__main__":
    main()
