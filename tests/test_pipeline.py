"""Pipeline parallelism (GPipe micro-batching, Executor.train_step_pipelined):
the MLP's layers split over two pipeline stages (machine views on rank 0 and
rank 1, 2 gloo ranks) and trained on 2 micro-batches must match one
single-process step on the whole batch; on one rank the same call is plain
gradient accumulation."""
import json
import os
import tempfile

import pytest
import torch
import torch.multiprocessing as mp

import dist_models as M
from dist_util import assert_params_close, free_port, run_single
from flexflow_train_amd.core import ActiMode, DataType


def mlp8(m):
    x = m.create_tensor([8, 32], DataType.DT_FLOAT, name="x")
    t = m.dense(x, 64, ActiMode.AC_MODE_RELU, name="fc0")
    t = m.dense(t, 48, name="fc1")
    t = m.relu(t, name="act1")
    t = m.dense(t, 8, name="out")
    m.softmax(t, name="sm")


def _micro():
    feeds, labels = _full()
    return [{"x": feeds["x"][:8]}, {"x": feeds["x"][8:]}], [labels[:8], labels[8:]]


def _full():
    g = torch.Generator().manual_seed(7)
    return {"x": torch.randn(16, 32, generator=g)}, torch.randint(0, 8, (16,), generator=g)


def _build(strategy_file=None, seed=0):
    from flexflow_train_amd.core import FFConfig, FFModel, LossType, MetricsType, SGDOptimizer

    cfg = FFConfig()
    cfg.seed = seed
    if strategy_file:
        cfg.import_strategy_file = strategy_file
    else:
        cfg.only_data_parallel = True
    model = FFModel(cfg)
    mlp8(model)
    model.compile(optimizer=SGDOptimizer(model, lr=0.05), loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY,
                  metrics=[MetricsType.METRICS_ACCURACY])
    ex = model.executor
    g = torch.Generator().manual_seed(seed)
    for name in sorted(ex.parameter_names()):
        ex.set_parameter(name, torch.randn(ex.get_parameter(name).shape, generator=g) * 0.2)
    return ex


def _train(ex, steps=2, schedule="1f1b"):
    feeds, labels = _micro()
    for _ in range(steps):
        ex.train_step_pipelined(feeds, labels, schedule=schedule)
    return {n: ex.get_parameter(n).detach().cpu().clone() for n in sorted(ex.parameter_names())}


def _stage_strategy(path):
    """Every layer unsharded; x, fc0, fc1 (and their weights) on rank 0, the rest on rank 1."""
    from flexflow_train_amd import _ffcore as C
    from flexflow_train_amd.core import FFConfig, FFModel
    from flexflow_train_amd.search.strategy import export_strategy

    m = FFModel(FFConfig())
    mlp8(m)
    s = json.loads(C.data_parallel_strategy(m.cg, 2))
    for v in s.values():
        v["batch"] = 1
    pcg, _, _ = C.lower_strategy(m.cg, json.dumps(s), 2)
    views = {}
    for n in pcg.topo_order():
        name = pcg.layer_name(n).split(".")[0]
        views[n] = (0,) if name in ("x", "fc0", "fc1") else (1,)
    export_strategy(path, pcg, views, {"world": 2, "source": "test"})


def _worker(rank, world, port, strategy, out, schedule="1f1b"):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    torch.set_num_threads(1)
    ex = _build(strategy)
    params = _train(ex, schedule=schedule)
    if rank == 0:
        torch.save({"params": params, "stats": dict(ex.dist.stats), "stages": ex.pipeline_stages(),
                    "peak": ex.peak_live_micro_batches}, out)
    import torch.distributed as dist

    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("schedule", ["gpipe", "1f1b"])
def test_gradient_accumulation_matches_full_batch(schedule):
    ref = run_single(M.mlp)
    ex = _build()
    got = _train(ex, schedule=schedule)
    assert_params_close(got, ref["params"], rtol=1e-4, atol=1e-5)
    # one stage: 1F1B keeps one micro-batch live, GPipe all of them
    assert ex.peak_live_micro_batches == (1 if schedule == "1f1b" else 2)


@pytest.mark.parametrize("schedule", ["gpipe", "1f1b"])
def test_two_stage_pipeline_matches_full_batch(schedule):
    ref = run_single(M.mlp)
    with tempfile.TemporaryDirectory() as d:
        strat = os.path.join(d, "pp.json")
        _stage_strategy(strat)
        out = os.path.join(d, "out.pt")
        mp.start_processes(_worker, args=(2, free_port(), strat, out, schedule), nprocs=2, join=True,
                           start_method="spawn")
        res = torch.load(out, weights_only=True)
    assert_params_close(res["params"], ref["params"], rtol=1e-4, atol=1e-5)
    assert res["stages"] == 2 and res["peak"] == 2
    # the stage boundary moved activations / gradients between the ranks as
    # matched send / recv pairs (comm.py _exchange_send_recv), no all_to_all
    assert res["stats"].get("send_recv", 0) > 0, res["stats"]
    assert res["stats"].get("all_to_all", 0) == 0, res["stats"]


# ---------------------------------------------------------------- searched stages
def deep(m, batch=8, width=1024, layers=4):
    """Weight-heavy, activation-light: its gradient all-reduce outweighs the
    compute, so splitting it into stages (no gradient sync) beats DP."""
    t = m.create_tensor([batch, width], DataType.DT_FLOAT, name="x")
    for i in range(layers):
        t = m.dense(t, width, ActiMode.AC_MODE_RELU, name=f"fc{i}")
    m.softmax(m.dense(t, 8, name="out"), name="sm")


def _search(world, micro_batches, **kw):
    from flexflow_train_amd import _ffcore as C
    from flexflow_train_amd.core import FFConfig, FFModel
    from flexflow_train_amd.search import native

    m = FFModel(FFConfig())
    deep(m, **kw)
    cfg = {"world": world, "budget": 10, "time_limit": 20, "micro_batches": micro_batches,
           "enable_parameter_parallel": True}
    pcg, rep, views = C.graph_optimize(m.cg, native.cost_model(use_profiles=False), json.dumps(cfg))
    return pcg, json.loads(rep), views


def test_search_prices_pipeline_candidates():
    """graph_optimize prices every S | world stage split next to the Unity /
    MCMC winner at equal work (m micro-batches per step): a deep weight-heavy
    MLP on 4 devices with 4 micro-batches goes to 4 data-parallel-free stages;
    the bubble is (S - 1) / (m + S - 1); stage placements are disjoint blocks."""
    _, rep, views = _search(4, 4, width=2048)
    assert rep["micro_batches"] == 4
    cands = {c["stages"]: c for c in rep["pipeline_candidates"]}
    assert set(cands) == {2, 4}
    for s, c in cands.items():
        assert abs(c["bubble_fraction"] - (s - 1) / (4 + s - 1)) < 1e-9
        assert len(c["stage_time"]) == s
    assert rep["algorithm"].endswith("+pipeline") and rep["pipeline_stages"] == 4, rep["algorithm"]
    assert rep["cost"] < rep["data_parallel_cost"]
    # four stages, one device each, in topological order
    assert sorted({tuple(v) for v in views.values()}) == [(0,), (1,), (2,), (3,)]


def test_micro_batches_change_the_winner():
    """With one micro-batch a pipeline is pure bubble on 4 devices for the
    shallow model; with 4 the stages overlap and win."""
    _, r1, _ = _search(4, 1)
    _, r4, _ = _search(4, 4)
    assert not r1["algorithm"].endswith("+pipeline"), r1["algorithm"]
    assert r4["algorithm"].endswith("+pipeline"), r4["algorithm"]


def _fit_worker(rank, world, port, out):
    if world > 1:
        os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                           "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    else:
        for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
            os.environ.pop(k, None)
    torch.set_num_threads(1)
    import numpy as np
    from flexflow_train_amd.core import FFConfig, FFModel, LossType, MetricsType, SGDOptimizer

    cfg = FFConfig()
    cfg.micro_batches = 2
    cfg.search_budget = 10
    cfg.search_time_limit = 20
    cfg.print_freq = 0
    cfg.batch_size = 8
    if world == 1:
        cfg.only_data_parallel = True
    m = FFModel(cfg)
    deep(m, width=256)
    m.compile(optimizer=SGDOptimizer(m, lr=0.05), loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY,
              metrics=[MetricsType.METRICS_ACCURACY])
    ex = m.executor
    g = torch.Generator().manual_seed(3)
    for name in sorted(ex.parameter_names()):
        ex.set_parameter(name, torch.randn(ex.get_parameter(name).shape, generator=g) * 0.05)
    x = torch.randn(32, 256, generator=g).numpy().astype(np.float32)
    y = torch.randint(0, 8, (32, 1), generator=g).numpy().astype(np.int32)
    m.fit(x=x, y=y, batch_size=8, epochs=1)
    params = {n: ex.get_parameter(n).detach().cpu().clone() for n in sorted(ex.parameter_names())}
    if rank == 0:
        torch.save({"params": params, "algorithm": m.search_report.get("algorithm", ""),
                    "stats": dict(ex.dist.stats)}, out)
    if world > 1:
        import torch.distributed as dist

        dist.barrier()
        dist.destroy_process_group()


def test_fit_with_micro_batches_on_searched_pipeline(tmp_path):
    """FFConfig.micro_batches=2: the search on 2 gloo ranks picks a
    two-stage pipeline for the weight-heavy MLP, fit() trains it in GPipe
    order (2 micro-batches per update), and the parameters equal one process
    accumulating the same 2 micro-batches per step."""
    ref = str(tmp_path / "ref.pt")
    out = str(tmp_path / "pp.pt")
    _fit_worker(0, 1, 0, ref)
    mp.start_processes(_fit_worker, args=(2, free_port(), out), nprocs=2, join=True, start_method="spawn")
    a = torch.load(ref, weights_only=True)
    b = torch.load(out, weights_only=True)
    assert b["algorithm"].endswith("+pipeline"), b["algorithm"]
    assert b["stats"].get("send_recv", 0) > 0, b["stats"]   # stage boundaries: matched send / recv pairs
    assert_params_close(b["params"], a["params"], rtol=1e-4, atol=1e-5)
