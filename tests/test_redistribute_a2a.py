"""Resharding through one all_to_all (parallel/comm.py): dim-0 shards ->
dim-1 shards, partial sums -> shards, and a reshard onto a sub-block, on 2
and 4 gloo ranks, checked element for element against the full tensor, and
the same plans through the point-to-point fallback."""
import os

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from dist_util import free_port
from flexflow_train_amd.parallel.comm import DistContext, Redistributor, make_plan
from flexflow_train_amd.parallel.layout import Layout, rel_slices


def _cases(world):
    """(src, dst, the plan kind the engine must pick; None = not checked)."""
    S = (8, 12, 4)
    cases = [
        (Layout(S, (world, 1, 1), block=world), Layout(S, (1, world if 12 % world == 0 else 1, 1), block=world),
         None),
        # partial sums -> batch shards: one reduce_scatter_tensor
        (Layout(S, (1, 1, 1), a_deg=world, block=world), Layout(S, (world, 1, 1), block=world), "reduce_scatter"),
        # partial sums -> shards of an inner dim (packed once, then reduce-scattered)
        (Layout(S, (1, 1, 1), a_deg=2, block=2), Layout(S, (1, 2, 1), block=2), "reduce_scatter"),
        (Layout(S, (1, 2, 1), block=world), Layout(S, (2, 1, 1), block=2, start=world - 2), None),
        # shards -> replicated: all_gather_into_tensor, outermost and inner dims
        (Layout(S, (world, 1, 1), block=world), Layout(S, (1, 1, 1), block=world), "all_gather"),
        (Layout(S, (1, 2, 1), block=2), Layout(S, (1, 1, 1), block=2), "all_gather"),
    ]
    if world >= 4:
        # a stage boundary that involves 3 of 4 ranks: a sub-group all_to_all
        cases.append((Layout(S, (2, 1, 1), block=2, start=0), Layout(S, (1, 1, 1), block=1, start=2), "all_to_all"))
        # replicated on [0, 1] -> 2-way shards on [1, 2]: rank 1 keeps its own
        # piece while another rank exchanges (it must not come back zero
        # whether or not it is a member of the exchange)
        cases.append((Layout(S, (1, 1, 1), block=2, start=0), Layout(S, (2, 1, 1), block=2, start=1), None))
    return cases


def _worker(rank, world, port, p2p, errs):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    if p2p:
        os.environ["FF_REDIST_P2P"] = "1"
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ctx = DistContext(rank, world, torch.device("cpu"))
        red = Redistributor(ctx)
        g = torch.Generator().manual_seed(0)
        for src, dst, kind in _cases(world):
            if kind is not None and not p2p:
                assert make_plan(src, dst, world).kind == kind, (src, dst, make_plan(src, dst, world).kind)
            full = torch.randn(src.sizes, generator=g)
            cs = src.coord(rank)
            x = None
            if cs is not None:
                x = full[rel_slices(src.box(cs.shard), tuple((0, s) for s in src.sizes))].clone()
                if src.sum_degree > 1:   # partial sums: piece i holds full/deg
                    x = x / src.sum_degree
            y = red(x, src, dst, torch.float32, torch.device("cpu"))
            cd = dst.coord(rank)
            if cd is None:
                assert y is None
                continue
            want = full[rel_slices(dst.box(cd.shard), tuple((0, s) for s in dst.sizes))]
            torch.testing.assert_close(y, want)
        key = "p2p" if p2p else "all_to_all"
        assert ctx.stats[key] > 0, ctx.stats
        if not p2p:
            assert ctx.stats.get("reduce_scatter", 0) >= 1 and ctx.stats["all_gather"] >= 1, ctx.stats
            if world >= 4:
                assert ctx.stats.get("all_to_all_subgroup", 0) >= 1 or rank == 3, ctx.stats
    except BaseException as e:  # noqa: BLE001
        errs.put(repr(e))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
@pytest.mark.parametrize("p2p", [False, True])
def test_reshard_matches_full_tensor(world, p2p):
    errs = mp.get_context("spawn").SimpleQueue()
    mp.start_processes(_worker, args=(world, free_port(), p2p, errs), nprocs=world, join=True, start_method="spawn")
    assert errs.empty()


def test_plan_kinds():
    S = (8, 12, 4)
    assert make_plan(Layout(S, (4, 1, 1), block=4), Layout(S, (1, 4, 1), block=4), 4).kind == "all_to_all"
    assert make_plan(Layout(S, (1, 1, 1), a_deg=4, block=4), Layout(S, (1, 1, 1), block=4), 4).kind == "all_reduce"
    assert make_plan(Layout(S, (4, 1, 1), block=4), Layout(S, (1, 1, 1), block=4), 4).kind == "all_gather"
