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


def in_situ(model_name: str, out_path: str, rounds: int = 3, batch_per_gpu: int = 0):
    """Per-operator costs measured INSIDE the bench's own data-parallel
    training step on one GPU: the executor's fused kernels (add + LayerNorm,
    softmax + cross-entropy, conv -> BN statistics, BN + add + ReLU, GEMM
    epilogues) are timed as they run, an operator fused into another costs 0,
    and the fused loss is charged to the trailing softmax.  Each profiled step
    is queued behind a device busy-wait so the host runs ahead and the event
    spans measure device time only.  Keys are the cost model's op signatures
    (the same ones ``build_profile_table`` writes)."""
    import collections
    import types

    import bench
    from flexflow_train_amd.ops.gemm import _gpu_busy

    args = types.SimpleNamespace(gpus=1, steps=2, warmup=3, batch_per_gpu=batch_per_gpu, seq=512, model=model_name,
                                 layers=None, strategy="dp", no_dp_compare=True, budget=0, gemm="auto", profile=True,
                                 graph=0)
    runner = bench._run_bert if model_name.startswith("bert") else bench._run_zoo
    res = runner(args, 1, 0, only_dp=True)
    ex, model = res["ex"], res["model"]
    feeds, labels = res["feeds"], res["labels"]
    per = collections.defaultdict(float)
    for _ in range(rounds):
        ex.tracer.clear()
        torch.cuda.synchronize()
        _gpu_busy(400.0)
        ex.train_step(feeds, labels)
        for name, _cat, _st, _s, dur in ex.tracer._resolved():
            per[name] += dur / rounds
    pcg = model.pcg
    fused_softmax = getattr(ex, "softmax_fused_step", None)
    sums = collections.defaultdict(lambda: [0.0, 0.0, 0])
    for n in pcg.topo_order():
        op = pcg.layer_op(n)
        if op.op_type in ("INPUT", "WEIGHT", "NOOP") or pcg.is_weight_path(n) or C.is_parallel_op(op.type):
            continue
        nm = pcg.layer_name(n)
        ins = [pcg.shape(v).piece_shape() for v in pcg.layer_data_inputs(n)]
        outs = [pcg.shape(C.ValueRef(n, k)).piece_shape() for k in range(pcg.num_outputs(n))]
        sig = C.CostModel.signature(op, ins + outs)
        f, b = per.get(f"{nm}:fwd", 0.0), per.get(f"{nm}:bwd", 0.0)
        if fused_softmax is not None and nm == fused_softmax.name:
            f += per.get("__loss__:fwd", 0.0)
        e = sums[sig]
        e[0] += f
        e[1] += b
        e[2] += 1
    table = {sig: {"fwd_ms": round(f / k, 5), "bwd_ms": round(b / k, 5), "source": "in_situ"}
             for sig, (f, b, k) in sums.items()}
    with open(out_path, "w") as fh:
        json.dump(table, fh, indent=0, sort_keys=True)
    total = sum(v for k, v in per.items() if not k.startswith("__"))
    print(json.dumps({"model": model_name, "entries": len(table), "op_ms": round(total, 3),
                      "loss_ms": round(per.get("__loss__:fwd", 0.0), 3),
                      "update_ms": round(per.get("__update__:fwd", 0.0), 3),
                      "bench_ms_per_step": round(res["ms"], 3)}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="bert-large",
                    choices=["bert-large", "bert-base", "gpt3-medium", "resnet50", "dlrm"])
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--batch-per-gpu", type=int, default=0, help="default: bench.py's per-GPU batch")
    ap.add_argument("--seq", type=int, default=512)
    ap.add_argument("--out", required=True)
    ap.add_argument("--in-situ", action="store_true",
                    help="time every operator inside the bench's own 1-GPU training step (fusions included)")
    args = ap.parse_args()
    if args.in_situ:
        return in_situ(args.model, args.out, batch_per_gpu=args.batch_per_gpu)
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
