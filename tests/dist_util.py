"""Multi-process CPU harness: run the same model under a strategy on W gloo
ranks and compare against the single-process run (reference: the CI's
multi_gpu_tests.sh ran examples under DP / searched strategies and checked
they train; here numerics are compared parameter by parameter)."""
from __future__ import annotations

import json
import os
import socket
import tempfile
from typing import Callable, Dict, Optional

import torch
import torch.multiprocessing as mp


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _train(model_fn: Callable, strategy_file: Optional[str], steps: int, seed: int, optimizer: str = "sgd",
           cfg_over: Optional[Dict] = None):
    from flexflow_train_amd.core import (AdamOptimizer, FFConfig, FFModel, LossType, MetricsType, SGDOptimizer)

    cfg = FFConfig()
    cfg.seed = seed
    for k, v in (cfg_over or {}).items():
        setattr(cfg, k, v)
    if strategy_file:
        cfg.import_strategy_file = strategy_file
    else:
        cfg.only_data_parallel = True
    model = FFModel(cfg)
    feeds, labels = model_fn(model)
    opt = SGDOptimizer(model, lr=0.05) if optimizer == "sgd" else AdamOptimizer(model, alpha=1e-3)
    model.compile(optimizer=opt, loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY,
                  metrics=[MetricsType.METRICS_ACCURACY])
    ex = model.executor
    g = torch.Generator().manual_seed(seed)
    for name in sorted(ex.parameter_names()):
        full = ex.get_parameter(name)
        ex.set_parameter(name, torch.randn(full.shape, generator=g) * 0.2)
    losses = []
    for _ in range(steps):
        ex.train_step(feeds, labels)
        losses.append(float(ex.perf_metrics().loss) if hasattr(ex.perf_metrics(), "loss") else 0.0)
    params = {n: ex.get_parameter(n).detach().cpu().clone() for n in sorted(ex.parameter_names())}
    return params, ex


def _worker(rank, world, port, model_fn, strategy_file, steps, seed, out_path, optimizer, cfg_over=None):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    torch.set_num_threads(1)
    params, ex = _train(model_fn, strategy_file, steps, seed, optimizer, cfg_over)
    if rank == 0:
        torch.save({"params": params, "stats": dict(ex.dist.stats)}, out_path)
    import torch.distributed as dist

    dist.barrier()
    dist.destroy_process_group()


def run_distributed(model_fn: Callable, world: int, strategy_file: Optional[str] = None, steps: int = 2,
                    seed: int = 0, optimizer: str = "sgd", cfg_over: Optional[Dict] = None) -> Dict:
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "out.pt")
        mp.start_processes(_worker, args=(world, free_port(), model_fn, strategy_file, steps, seed, out, optimizer, cfg_over),
                           nprocs=world, join=True, start_method="spawn")
        return torch.load(out, weights_only=True)


def run_single(model_fn: Callable, steps: int = 2, seed: int = 0, optimizer: str = "sgd") -> Dict:
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        os.environ.pop(k, None)
    params, ex = _train(model_fn, None, steps, seed, optimizer)
    return {"params": params}


def write_strategy(model_fn: Callable, world: int, overrides: Dict[str, dict], path: str):
    """Lower the data-parallel strategy with per-layer overrides and export
    it as a strategy file the FFModel can --import."""
    from flexflow_train_amd import _ffcore as C
    from flexflow_train_amd.core import FFConfig, FFModel
    from flexflow_train_amd.search.strategy import export_strategy

    m = FFModel(FFConfig())
    model_fn(m)
    s = json.loads(C.data_parallel_strategy(m.cg, world))
    for k, v in overrides.items():
        assert k in s, f"no layer {k}: {sorted(s)}"
        s[k] = v
    pcg, mapping, n = C.lower_strategy(m.cg, json.dumps(s), world)
    export_strategy(path, pcg, {}, {"world": world, "source": "test"})
    return pcg


def assert_params_close(a: Dict, b: Dict, rtol=2e-4, atol=2e-5):
    assert sorted(a) == sorted(b), (sorted(a), sorted(b))
    for k in a:
        torch.testing.assert_close(a[k], b[k], rtol=rtol, atol=atol, msg=lambda m: f"{k}: {m}")


def _recompile_worker(rank, world, port, model_fn, strategy_file, before, after, out_path):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    torch.set_num_threads(1)
    from flexflow_train_amd.core import (AdamOptimizer, FFConfig, FFModel, LossType, MetricsType, RecompileState)

    cfg = FFConfig()
    cfg.seed = 0
    cfg.only_data_parallel = True
    model = FFModel(cfg)
    feeds, labels = model_fn(model)
    model.compile(optimizer=AdamOptimizer(model, alpha=1e-3), loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY,
                  metrics=[MetricsType.METRICS_ACCURACY])
    ex = model.executor
    g = torch.Generator().manual_seed(0)
    for name in sorted(ex.parameter_names()):
        full = ex.get_parameter(name)
        ex.set_parameter(name, torch.randn(full.shape, generator=g) * 0.2)
    state = {"it": 0}

    def alter(ff):
        ff.ffconfig.only_data_parallel = False
        ff.ffconfig.import_strategy_file = strategy_file

    r = RecompileState(lambda ff: state["it"] == before, alter, model)
    for it in range(before + after):
        state["it"] = it
        model.recompile_on_condition(r)
        model.executor.train_step(feeds, labels)
    ex = model.executor
    params = {n: ex.get_parameter(n).detach().cpu().clone() for n in sorted(ex.parameter_names())}
    if rank == 0:
        torch.save({"params": params, "recompilations": r.recompilations}, out_path)
    import torch.distributed as dist

    dist.barrier()
    dist.destroy_process_group()


def run_recompile(model_fn, world, strategy_file, steps_before=2, steps_after=2):
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "out.pt")
        mp.start_processes(_recompile_worker, args=(world, free_port(), model_fn, strategy_file, steps_before,
                                                    steps_after, out), nprocs=world, join=True, start_method="spawn")
        return torch.load(out, weights_only=True)


def _ckpt_worker(rank, world, port, model_fn, strategy_file, steps, seed, ckpt_dir, mode, out_path, optimizer):
    """Train ``steps`` steps and save a checkpoint (mode "save", weights drawn
    like _train), or load one (possibly written under another world /
    strategy) and train ``steps`` more (mode "load")."""
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    torch.set_num_threads(1)
    from flexflow_train_amd.core import (AdamOptimizer, FFConfig, FFModel, LossType, MetricsType, SGDOptimizer)
    from flexflow_train_amd.utils.checkpoint import load_checkpoint, save_checkpoint

    cfg = FFConfig()
    cfg.seed = seed
    if strategy_file:
        cfg.import_strategy_file = strategy_file
    else:
        cfg.only_data_parallel = True
    model = FFModel(cfg)
    feeds, labels = model_fn(model)
    opt = SGDOptimizer(model, lr=0.05, momentum=0.9) if optimizer == "sgd" else AdamOptimizer(model, alpha=1e-3)
    model.compile(optimizer=opt, loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY,
                  metrics=[MetricsType.METRICS_ACCURACY])
    ex = model.executor
    meta = {}
    if mode == "save":
        g = torch.Generator().manual_seed(seed)
        for name in sorted(ex.parameter_names()):
            ex.set_parameter(name, torch.randn(ex.get_parameter(name).shape, generator=g) * 0.2)
    else:
        meta = load_checkpoint(model, ckpt_dir)
    for _ in range(steps):
        ex.train_step(feeds, labels)
    if mode == "save":
        save_checkpoint(model, ckpt_dir)
    params = {n: ex.get_parameter(n).detach().cpu().clone() for n in sorted(ex.parameter_names())}
    if rank == 0:
        torch.save({"params": params, "meta": {k: v for k, v in meta.items() if isinstance(v, (bool, int, str))}},
                   out_path)
    import torch.distributed as dist

    dist.barrier()
    dist.destroy_process_group()


def run_checkpointed(model_fn, ckpt_dir: str, save_world: int, load_world: int, save_strategy: Optional[str] = None,
                     load_strategy: Optional[str] = None, steps_before: int = 2, steps_after: int = 2, seed: int = 0,
                     optimizer: str = "adam") -> Dict:
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "out.pt")
        mp.start_processes(_ckpt_worker, args=(save_world, free_port(), model_fn, save_strategy, steps_before, seed,
                                               ckpt_dir, "save", out, optimizer),
                           nprocs=save_world, join=True, start_method="spawn")
        mp.start_processes(_ckpt_worker, args=(load_world, free_port(), model_fn, load_strategy, steps_after, seed,
                                               ckpt_dir, "load", out, optimizer),
                           nprocs=load_world, join=True, start_method="spawn")
        return torch.load(out, weights_only=True)
