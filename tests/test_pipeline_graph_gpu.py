"""The pipelined step (Executor.train_step_pipelined: 2 stages on rank 0 /
rank 1, 2 micro-batches, 1F1B) captured as hipGraph segments cut at every
stage-boundary transfer and gradient collective (make_graphed_train_step with
lists of micro-batches), replayed natively: the replayed steps equal eager
pipelined steps parameter by parameter.  2 gloo ranks share the one GPU
(RCCL needs a GPU per rank; the segments and the re-issued transfers are the
same code)."""
import os
import tempfile

import pytest
import torch
import torch.multiprocessing as mp

from dist_util import assert_params_close, free_port
import test_pipeline as P

pytestmark = pytest.mark.gpu


def _worker(rank, world, port, strategy, out):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "FF_DIST_BACKEND": "gloo"})
    a = P._build(strategy)
    b = P._build(strategy)
    dev = a.cfg.device
    feeds, labels = P._micro()
    feeds = [{k: v.to(dev) for k, v in f.items()} for f in feeds]
    labels = [y.to(dev) for y in labels]
    for _ in range(3):
        a.train_step_pipelined(feeds, labels)
    step = b.make_graphed_train_step(feeds, labels, warmup=2)
    step()
    torch.cuda.synchronize()
    pa = {n: a.get_parameter(n).float().cpu() for n in sorted(a.parameter_names())}
    pb = {n: b.get_parameter(n).float().cpu() for n in sorted(b.parameter_names())}
    if rank == 0:
        torch.save({"a": pa, "b": pb, "segments": list(b.graph_segments), "native": bool(b.native_replay),
                    "stages": b.pipeline_stages()}, out)
    import torch.distributed as dist

    dist.barrier()
    dist.destroy_process_group()


def test_pipelined_step_graph_capture(tmp_path):
    strat = str(tmp_path / "pp.json")
    P._stage_strategy(strat)
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "out.pt")
        mp.start_processes(_worker, args=(2, free_port(), strat, out), nprocs=2, join=True, start_method="spawn")
        res = torch.load(out, weights_only=True)
    assert res["stages"] == 2
    n_graphs, n_coll = res["segments"]
    assert n_coll >= 2 and n_graphs >= n_coll, res["segments"]   # boundary transfers cut the step
    assert res["native"]
    assert_params_close(res["b"], res["a"], rtol=1e-4, atol=1e-5)
