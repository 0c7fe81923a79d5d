"""Piecewise hipGraph capture of a distributed training step
(runtime/graphs.py): 2 ranks share the one GPU over gloo (RCCL needs a GPU
per rank; the segments and the re-issued collectives are the same code), and
a captured-then-replayed step must equal eager steps parameter by parameter,
for data parallelism (bucketed async gradient all-reduces) and for a
Megatron-style tensor-parallel MLP (a synchronous Reduction all-reduce in
the forward pass and its backward)."""
import os
import tempfile

import pytest
import torch
import torch.multiprocessing as mp

import dist_models as M
from dist_util import free_port, write_strategy

pytestmark = pytest.mark.gpu


def _compile(model_fn, strategy):
    from flexflow_train_amd.core import FFConfig, FFModel, LossType, MetricsType, SGDOptimizer

    cfg = FFConfig()
    if strategy:
        cfg.import_strategy_file = strategy
    else:
        cfg.only_data_parallel = True
    cfg.bucket_mb = 0   # one bucket per parameter: many segments
    m = FFModel(cfg)
    feeds, labels = model_fn(m)
    # SGD + momentum: the eager and replayed steps differ only by the order of
    # atomic gradient sums, and SGD keeps that at rounding size (Adam
    # normalises a near-zero gradient whose sign flips into a full lr-sized
    # step, which the parameter comparison below would read as a mismatch)
    m.compile(optimizer=SGDOptimizer(m, lr=0.05, momentum=0.9),
              loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY,
              metrics=[MetricsType.METRICS_SPARSE_CATEGORICAL_CROSSENTROPY])
    ex = m.executor
    g = torch.Generator().manual_seed(0)
    for n in sorted(ex.parameter_names()):
        ex.set_parameter(n, torch.randn(ex.get_parameter(n).shape, generator=g) * 0.2)
    dev = ex.cfg.device
    return ex, {k: v.to(dev) for k, v in feeds.items()}, labels.to(dev)


def _worker(rank, world, port, model_name, strategy, out_path):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "FF_DIST_BACKEND": "gloo"})
    model_fn = getattr(M, model_name)
    a, feeds, labels = _compile(model_fn, strategy)
    b, _, _ = _compile(model_fn, strategy)
    for _ in range(3):
        a.train_step(feeds, labels)
    step = b.make_graphed_train_step(feeds, labels, warmup=2)
    step()
    torch.cuda.synchronize()
    pa = {n: a.get_parameter(n).float().cpu() for n in sorted(a.parameter_names())}
    pb = {n: b.get_parameter(n).float().cpu() for n in sorted(b.parameter_names())}
    # replays keep training
    b.zero_metrics()
    for _ in range(10):
        step()
    first = b.perf_metrics().loss
    b.zero_metrics()
    for _ in range(5):
        step()
    last = b.perf_metrics().loss
    if rank == 0:
        torch.save({"a": pa, "b": pb, "segments": list(b.graph_segments), "first": first, "last": last,
                    "native": bool(getattr(b, "native_replay", False)), "stats": dict(b.dist.stats)}, out_path)
    import torch.distributed as dist

    dist.barrier()
    dist.destroy_process_group()


def _run(model_name, strategy=None, world=2):
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "out.pt")
        mp.start_processes(_worker, args=(world, free_port(), model_name, strategy, out), nprocs=world,
                           join=True, start_method="spawn")
        return torch.load(out, weights_only=True)


def _check(res):
    for n in res["a"]:
        torch.testing.assert_close(res["b"][n], res["a"][n], rtol=2e-2, atol=2e-3)
    n_graphs, n_coll = res["segments"]
    assert n_coll >= 1 and n_graphs >= n_coll + 1, res["segments"]
    assert res["last"] < res["first"]


def test_segmented_graph_data_parallel():
    res = _run("bert_tiny")
    assert res["segments"][1] >= 2, res["segments"]   # several gradient buckets
    _check(res)


def test_segmented_graph_tensor_parallel(tmp_path):
    path = str(tmp_path / "tp.json")
    write_strategy(M.mlp, 2, {"fc0": {"batch": 1, "model": 2, "kind": "column"},
                              "fc1": {"batch": 1, "model": 2, "kind": "row"}}, path)
    _check(_run("mlp", path))


def test_segmented_graph_stage_boundary(tmp_path):
    """Two placement stages (fc0 on rank 0, the rest on rank 1): the stage
    boundary is a matched send / recv plan (comm.py), captured as a
    collective item of the segmented graph and replayed natively; the
    replayed step equals eager steps.  Two gloo ranks share the one GPU here,
    and gloo moves device tensors only through collectives, so the pair runs
    as the sub-group all_to_all form (RCCL ranks send / recv)."""
    import json as _json

    from flexflow_train_amd import _ffcore as C
    from flexflow_train_amd.core import FFConfig, FFModel
    from flexflow_train_amd.search.strategy import export_strategy

    m = FFModel(FFConfig())
    M.mlp(m)
    s = _json.loads(C.data_parallel_strategy(m.cg, 2))
    for k in s:
        s[k]["batch"] = 1
    pcg = C.lower_strategy(m.cg, _json.dumps(s), 2)[0]
    views = {}
    for n in pcg.topo_order():
        name = pcg.layer_name(n).split(".")[0]
        views[n] = (0,) if name in ("x", "fc0") else (1,)
    path = str(tmp_path / "stages.json")
    export_strategy(path, pcg, views, {"world": 2, "source": "test"})
    res = _run("mlp", path)
    _check(res)
    assert res["stats"].get("all_to_all", 0) + res["stats"].get("send_recv", 0) > 0, res["stats"]
    assert res["native"], "the segmented step was not replayed natively"
