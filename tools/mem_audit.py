#!/usr/bin/env python3
"""Which tensors a training step really keeps (GPU): after one training
forward, every distinct storage referenced by the executor's saved-for-
backward tuples and its value environment, attributed to the step (PCG
node) that produced it, summed by operator type; next to the liveness
plan's activation blocks for the same PCG (csrc/ffcore/src/memory_plan.cc)
and the allocator's live bytes.  Drives the plan's executor-fusion rules.

    python tools/mem_audit.py resnet50 [batch]    |  bert-large [batch]
"""
import collections
import json
import sys

import numpy as np
import torch


def _tensors(o, out):
    if torch.is_tensor(o):
        out.append(o)
    elif isinstance(o, (list, tuple)):
        for x in o:
            _tensors(x, out)
    elif isinstance(o, dict):
        for x in o.values():
            _tensors(x, out)


def main():
    from flexflow_train_amd import _ffcore as C
    from flexflow_train_amd import models as Z
    from flexflow_train_amd.core import (AdamOptimizer, FFConfig, FFModel, LossType, MetricsType, SGDOptimizer)
    from flexflow_train_amd.search import native

    name = sys.argv[1]
    sys.argv = [a for a in sys.argv if a != "--trace"] + (["--trace"] if "--trace" in sys.argv else [])
    cfg = FFConfig()
    m = FFModel(cfg)
    if name.startswith("gpt"):
        b = int(sys.argv[2]) if len(sys.argv) > 2 and sys.argv[2].isdigit() else 16
        cfg.batch_size = b
        inputs, out, mc = Z.build("gpt", m, batch_size=b, hidden_size=1024, num_layers=24, num_heads=16,
                                  sequence_length=2048)
        m.compile(optimizer=AdamOptimizer(m, alpha=1e-4), loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY,
                  metrics=[MetricsType.METRICS_ACCURACY])
        ex = m.executor
        fn, ln = Z.synthetic("gpt", mc, inputs, np.random.default_rng(0))
        feeds = {k: ex._local_piece(k, torch.as_tensor(v)) for k, v in fn.items()}
        labels = ex.local_labels(torch.as_tensor(ln))
        wbytes = 16.0
    elif name.startswith("bert"):
        from flexflow_train_amd.models.bert import bert_large, build_bert
        b = int(sys.argv[2]) if len(sys.argv) > 2 and sys.argv[2].isdigit() else 64
        cfg.batch_size = b
        bc = bert_large(batch_size=b, sequence_length=512)
        build_bert(m, bc)
        m.compile(optimizer=AdamOptimizer(m, alpha=1e-4), loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY,
                  metrics=[MetricsType.METRICS_ACCURACY])
        ex = m.executor
        dev = ex.cfg.device
        feeds = {}
        for n in ex.inputs:
            shp = ex.local_input_shape(n)
            hi = bc.vocab_size if n == "input_ids" else (shp[-1] if n == "position_ids" else bc.type_vocab_size)
            feeds[n] = torch.randint(0, hi, shp, device=dev, dtype=torch.int32)
        labels = torch.randint(0, bc.vocab_size, ex._loss_layout().piece_shape[:-1], device=dev)
        wbytes = 16.0
    else:
        b = int(sys.argv[2]) if len(sys.argv) > 2 and sys.argv[2].isdigit() else 256
        cfg.batch_size = b
        inputs, out, mc = Z.build(name, m, batch_size=b, image_size=224, num_classes=1000)
        m.compile(optimizer=SGDOptimizer(m, lr=0.01, momentum=0.9),
                  loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY, metrics=[MetricsType.METRICS_ACCURACY])
        ex = m.executor
        fn, ln = Z.synthetic(name, mc, inputs, np.random.default_rng(0))
        feeds = {k: ex._local_piece(k, torch.as_tensor(v)) for k, v in fn.items()}
        labels = ex.local_labels(torch.as_tensor(ln))
        wbytes = 12.0
    if "--trace" in sys.argv:
        torch.cuda.memory._record_memory_history(max_entries=200000)
    ex.train_step(feeds, labels)          # autotune / workspaces settle
    torch.cuda.synchronize()
    base = torch.cuda.memory_allocated()
    if "--trace" in sys.argv:
        # the largest blocks alive between steps, with the Python frames that allocated them
        snap = torch.cuda.memory._snapshot()
        blocks = []
        for seg in snap["segments"]:
            for blk in seg["blocks"]:
                if blk["state"] == "active_allocated":
                    fr = [f"{f['filename'].split('/')[-1]}:{f['line']}:{f['name']}" for f in blk.get("frames", [])
                          if f["filename"].endswith(".py") and "torch/" not in f["filename"]]
                    blocks.append((blk["size"], fr[:4]))
        blocks.sort(key=lambda b: -b[0])
        by_site = collections.Counter()
        for sz, fr in blocks:
            by_site[" <- ".join(fr[:3])] += sz
        for site, sz in by_site.most_common(15):
            print(json.dumps({"base_site": site, "gb": round(sz / 1e9, 3)}))
    n0 = 0
    if "--trace" in sys.argv:
        n0 = sum(len(tr) for tr in torch.cuda.memory._snapshot().get("device_traces", []))
    torch.cuda.reset_peak_memory_stats()
    ex.train_step(feeds, labels)
    torch.cuda.synchronize()
    step_peak = torch.cuda.max_memory_allocated()
    if "--trace" in sys.argv:
        snap = torch.cuda.memory._snapshot()
        # what is live at the step's peak: replay the step's alloc / free
        # events from the live set at its start, grouped by allocation site
        evs = [e for tr in snap.get("device_traces", []) for e in tr][n0:]
        live = {}
        cur = 0
        best, best_live = -1, {}
        for e in evs:
            a = e.get("action")
            if a == "alloc":
                live[e["addr"]] = e
                cur += e["size"]
                if cur > best:
                    best, best_live = cur, dict(live)
            elif a == "free_requested" and e["addr"] in live:
                cur -= live.pop(e["addr"])["size"]
        by_site = collections.Counter()
        for e in best_live.values():
            fr = [f"{f['filename'].split('/')[-1]}:{f['line']}:{f['name']}" for f in e.get("frames", [])
                  if f["filename"].endswith(".py") and "torch/" not in f["filename"]]
            by_site[" <- ".join(fr[:3])] += e["size"]
        print(json.dumps({"step_peak_new_gb": round(best / 1e9, 3), "sites": len(by_site)}))
        for site, sz in by_site.most_common(20):
            print(json.dumps({"peak_site": site, "gb": round(sz / 1e9, 3)}))
        # the step's largest single allocations, with the frames that made them
        evs = [e for tr in snap.get("device_traces", []) for e in tr if e.get("action") == "alloc"]
        evs.sort(key=lambda e: -e["size"])
        for e in evs[:12]:
            fr = [f"{f['filename'].split('/')[-1]}:{f['line']}:{f['name']}" for f in e.get("frames", [])
                  if f["filename"].endswith(".py") and "torch/" not in f["filename"]]
            print(json.dumps({"step_alloc_gb": round(e["size"] / 1e9, 3), "site": " <- ".join(fr[:4])}))
        torch.cuda.memory._record_memory_history(enabled=None)
    # the persistent part: weights, optimizer state, gradient flats, workspaces
    state_b = sum(p.master.numel() * p.master.element_size() for p in ex.params if p.group)
    grads_b = sum(f["grad"].numel() * f["grad"].element_size() for f in ex.flats if torch.is_tensor(f.get("grad")))
    ex.forward(feeds, training=True)
    torch.cuda.synchronize()
    live = torch.cuda.memory_allocated() - base
    seen = {}
    by_saved = collections.Counter()
    by_env = collections.Counter()
    for i, s in enumerate(ex.steps):
        ts = []
        _tensors(ex._saved.get(i), ts)
        for t in ts:
            if not t.is_cuda:
                continue
            k = t.untyped_storage().data_ptr()
            if k not in seen:
                seen[k] = t.untyped_storage().nbytes()
                by_saved[s.op_type] += seen[k]
    for i, s in enumerate(ex.steps):
        for o in s.outputs:
            t = ex._env.get(o)
            if torch.is_tensor(t) and t.is_cuda:
                k = t.untyped_storage().data_ptr()
                if k not in seen:
                    seen[k] = t.untyped_storage().nbytes()
                    by_env[s.op_type] += seen[k]
    (p,) = native.plan_memory(m.pcg, 1, with_blocks=True, weight_bytes_per_param=wbytes, act_elem_bytes=2.0,
                              executor_fusions=True)
    steps = p["steps"]
    fwd_end = steps // 2 - 1
    plan = collections.Counter()
    for blk in p["blocks"]:
        if blk["kind"] == 0 and blk["start"] <= fwd_end <= blk["end"]:
            plan[m.pcg.layer_op(blk["node"]).op_type] += blk["bytes"]
    ops = sorted(set(by_saved) | set(by_env) | set(plan), key=lambda k: -(plan[k] + by_saved[k]))
    rows = [{"op": k, "plan_gb": round(plan[k] / 1e9, 3), "saved_gb": round(by_saved[k] / 1e9, 3),
             "env_only_gb": round(by_env[k] / 1e9, 3)} for k in ops]
    print(json.dumps({"model": name, "batch": b, "allocator_live_after_forward_gb": round(live / 1e9, 3),
                      "distinct_kept_gb": round(sum(seen.values()) / 1e9, 3),
                      "plan_activations_at_forward_end_gb": round(sum(plan.values()) / 1e9, 3),
                      "plan_arena_gb": round(p["arena_bytes"] / 1e9, 3),
                      "plan_weight_gb": round(p["weight_bytes"] / 1e9, 3),
                      "base_allocated_after_step_gb": round(base / 1e9, 3),
                      "step_peak_gb": round(step_peak / 1e9, 3),
                      "step_peak_over_base_gb": round((step_peak - base) / 1e9, 3),
                      "masters_gb": round(state_b / 1e9, 3), "grad_flats_gb": round(grads_b / 1e9, 3),
                      "measured_peak_gb": round(torch.cuda.max_memory_allocated() / 1e9, 3)}))
    for r in rows:
        print(json.dumps(r))


if __name__ == "__main__":
    main()
