"""RCCL on real hardware at world size 1 (FF_DIST_WORLD1=1).

The multi-GPU bench only ever runs on the driver's 8-GPU node, so this test
drives the whole RCCL path on the one GPU a test box has: a ``nccl``
process group (RCCL on ROCm) with one member whose collectives are still
issued -- every DistContext wrapper (all-reduce, reduce-scatter, reduce,
broadcast, all-gather, max), the all-to-all redistribution exchange, and
training steps whose bucketed gradient all-reduce / ZeRO reduce-scatter +
all-gather / parameter-server reduce + broadcast go through RCCL, eagerly and
replayed from hipGraph segments cut at every collective (runtime/graphs.py).
A one-member collective is the identity, so the trained parameters must
equal a run with no process group.

The check runs in a child process (its own process group, torn down when it
exits); reference launch model: tests/multi_gpu_tests.sh:28-74.
"""
import json
import os
import subprocess
import sys
import textwrap

import pytest


ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_CHILD = textwrap.dedent(r'''
    import json, os, sys
    sys.path.insert(0, os.path.join(ROOT, "tests")); sys.path.insert(0, ROOT)
    import torch
    import dist_models as M
    from flexflow_train_amd.core import AdamOptimizer, FFConfig, FFModel, LossType, MetricsType
    from flexflow_train_amd.parallel import comm as C

    def train(model_fn, steps, graphed, **over):
        cfg = FFConfig(); cfg.only_data_parallel = True; cfg.bucket_mb = 0
        for k, v in over.items():
            setattr(cfg, k, v)
        m = FFModel(cfg)
        feeds, labels = model_fn(m)
        m.compile(optimizer=AdamOptimizer(m, alpha=1e-3), loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY,
                  metrics=[MetricsType.METRICS_ACCURACY])
        ex = m.executor
        g = torch.Generator().manual_seed(0)
        for n in sorted(ex.parameter_names()):
            ex.set_parameter(n, torch.randn(ex.get_parameter(n).shape, generator=g) * 0.2)
        dev = ex.cfg.device
        feeds = {k: v.to(dev) for k, v in feeds.items()}; labels = labels.to(dev)
        if graphed:
            step = ex.make_graphed_train_step(feeds, labels, warmup=1)
            for _ in range(steps - 1):
                step()
        else:
            for _ in range(steps):
                ex.train_step(feeds, labels)
        if DEV == "cuda":
            torch.cuda.synchronize()
        return ex, {n: ex.get_parameter(n).float().cpu() for n in sorted(ex.parameter_names())}

    out = {}
    mode = sys.argv[1]
    if mode == "ref":
        for name, over in (("dp", {}), ("zero", {"shard_optimizer": True}), ("ps", {"parameter_sync": "ps"})):
            _, p = train(M.mlp, 4, False, **over)
            torch.save(p, os.path.join(OUT, f"ref_{name}.pt"))
        _, p = train(M.embedding, 4, False)
        torch.save(p, os.path.join(OUT, "ref_emb.pt"))
        print(json.dumps({"ok": True})); sys.exit(0)

    dev = torch.device("cuda", 0) if DEV == "cuda" else torch.device("cpu")
    ctx = C.DistContext.from_env(device=dev)
    out["backend"] = ctx.backend
    out["distributed"] = ctx.distributed
    t = torch.arange(1024, dtype=torch.float32, device=dev)
    ref = t.clone()
    for w in (ctx.all_reduce_(t, [0], async_op=True), ctx.reduce_scatter_(t, [0], async_op=True),
              ctx.reduce_(t, [0], 0, async_op=True), ctx.broadcast_(t, [0], 0, async_op=True)):
        w.wait()
    ctx.all_gather_(t, [0])
    out["wrappers_identity"] = bool(torch.equal(t, ref))
    out["max_scalar"] = ctx.max_scalar(3.5)
    box = ((0, 8), (0, 16))
    plan = C.Plan("all_to_all", {0: [C.Contribution(0, box, box)]}, {0: box}, {0: box}, [])
    x = torch.randn(8, 16, device=dev, dtype=torch.bfloat16 if DEV == "cuda" else torch.float32)
    y = C.execute_plan(plan, x, ctx, (8, 16), x.dtype, dev)
    out["all_to_all_identity"] = bool(torch.equal(x, y))
    out["stats"] = dict(ctx.stats)
    res = {}
    for name, model_fn, over in (("dp", M.mlp, {}), ("zero", M.mlp, {"shard_optimizer": True}),
                                 ("ps", M.mlp, {"parameter_sync": "ps"}), ("emb", M.embedding, {})):
        ref_p = torch.load(os.path.join(OUT, f"ref_{name}.pt"), weights_only=True)
        for graphed in ((False, True) if DEV == "cuda" else (False,)):
            ex, p = train(model_fn, 4, graphed, **over)
            diff = max(float((p[k] - ref_p[k]).abs().max()) for k in ref_p)
            res[f"{name}{'_graph' if graphed else ''}"] = {
                "max_abs_diff": diff, "syncs": dict(ex.dist.stats),
                "segments": list(getattr(ex, "graph_segments", ()) or ()),
                "native_replay": getattr(ex, "native_replay", None)}
    out["train"] = res
    import torch.distributed as dist
    dist.destroy_process_group()
    print(json.dumps(out))
''')


def _run(tmp_path, mode, extra_env, dev="cuda"):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "FF_DIST_BACKEND"):
        env.pop(k, None)
    env.update(extra_env)
    env["HSA_ENABLE_IPC_MODE_LEGACY"] = "0"
    if dev == "cpu":
        env["CUDA_VISIBLE_DEVICES"] = ""
        env["HIP_VISIBLE_DEVICES"] = ""
    code = f"ROOT = {ROOT!r}\nOUT = {str(tmp_path)!r}\nDEV = {dev!r}\n" + _CHILD
    p = subprocess.run([sys.executable, "-c", code, mode], env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    return json.loads(p.stdout.strip().splitlines()[-1])


def _check(out, backend):
    assert out["backend"] == backend and out["distributed"]
    assert out["wrappers_identity"] and out["all_to_all_identity"]
    assert out["max_scalar"] == 3.5
    assert out["stats"]["all_to_all"] == 1 and out["stats"]["all_reduce"] == 1
    for name, r in out["train"].items():
        assert r["max_abs_diff"] < 1e-5, (name, r)
        s = r["syncs"]
        if name.startswith("zero"):
            assert s.get("reduce_scatter", 0) > 0 and s["all_gather"] > 0, (name, s)
        elif name.startswith("ps"):
            assert s.get("reduce", 0) > 0 and s.get("broadcast", 0) > 0, (name, s)
        else:
            assert s["all_reduce"] > 0, (name, s)
        if name.endswith("_graph"):
            assert r["segments"] and r["segments"][1] > 0, (name, r)
            if backend == "nccl":   # the segment chain replays from C++ (csrc/runtime/replay.cpp)
                assert r["native_replay"] is True, (name, r)


@pytest.mark.gpu
def test_rccl_world1_collectives_and_training(tmp_path):
    _run(tmp_path, "ref", {"FF_DIST_WORLD1": "0"})
    _check(_run(tmp_path, "rccl", {"FF_DIST_WORLD1": "1"}), "nccl")


def test_gloo_world1_collectives_and_training(tmp_path):
    """The same harness on the CPU (gloo): runs in the CPU tier."""
    _run(tmp_path, "ref", {"FF_DIST_WORLD1": "0"}, dev="cpu")
    _check(_run(tmp_path, "rccl", {"FF_DIST_WORLD1": "1"}, dev="cpu"), "gloo")
