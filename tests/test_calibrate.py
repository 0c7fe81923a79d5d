"""Collective cost-model calibration (parallel/calibrate.py): the fit
recovers known latency / bandwidth from a fake clock, the calibrated
MachineSpecification prices those collectives as measured, and on 2 gloo
ranks a trained step's message sizes are found, measured (real collectives)
and summarised with the simulator's predicted step time -- the plumbing
bench.py runs on N > 1 GPUs."""
import os

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from flexflow_train_amd import _ffcore as C
from flexflow_train_amd.parallel import calibrate

ALPHA, BW = 12e-6, 180e9


def fake_clock(kind, nbytes, p):
    """A link with latency ALPHA per collective (all-reduce: the cost model's
    2 (p - 1) / 4 + 1 alpha terms) and bus bandwidth BW (all-to-all half)."""
    bw = BW / 2 if kind == "all_to_all" else BW
    a = ALPHA * (2.0 * (p - 1) / 4.0 + 1.0) if kind == "all_reduce" else ALPHA
    return (a + calibrate._factor(kind, p) * nbytes / bw) * 1e3


class FakeCtx:
    world = 8
    rank = 0


def test_fit_recovers_latency_and_bandwidth():
    sizes = {k: [1 << 20, 16 << 20, 64 << 20] for k in calibrate.KINDS}
    samples = calibrate.measure(FakeCtx(), sizes, torch.device("cpu"), timer=fake_clock)
    fits = calibrate.fit(samples)
    assert set(fits) == set(calibrate.KINDS)
    assert fits["all_reduce"]["bw_bytes_per_s"] == pytest.approx(BW, rel=1e-6)
    assert fits["all_to_all"]["bw_bytes_per_s"] == pytest.approx(BW / 2, rel=1e-6)
    assert fits["all_gather"]["latency_s"] == pytest.approx(ALPHA, rel=1e-6)
    nominal = C.MachineSpecification.mi355x()
    cal = calibrate.calibrated_spec(nominal, fits)
    assert cal.collective_latency == pytest.approx(ALPHA, rel=1e-6)
    assert cal.collective_bw[8] == pytest.approx(BW, rel=1e-6) and cal.all_to_all_bw[8] == pytest.approx(BW / 2)
    rows = calibrate.comparison(samples, nominal, cal)
    for r in rows:   # after calibration the model reproduces every measurement
        assert r["calibrated_ms"] == pytest.approx(r["measured_ms"], rel=1e-3, abs=1e-4), r
    # the nominal (uncalibrated) model is off somewhere: the calibration matters
    assert any(abs(r["simulated_ms"] - r["measured_ms"]) > 0.05 * r["measured_ms"] for r in rows)


def _worker(rank, world, port, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    torch.set_num_threads(1)
    try:
        import dist_models as M
        from flexflow_train_amd.core import FFConfig, FFModel, LossType, MetricsType, SGDOptimizer

        cfg = FFConfig()
        cfg.only_data_parallel = True
        m = FFModel(cfg)
        feeds, labels = M.mlp(m)
        m.compile(optimizer=SGDOptimizer(m, lr=0.05), loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY,
                  metrics=[MetricsType.METRICS_ACCURACY])
        ex = m.executor
        ex.train_step(feeds, labels)
        used = calibrate.step_message_sizes(ex)
        assert used.get("all_reduce"), used        # the DP gradient buckets
        cal = calibrate.calibrate_for_step(ex, iters=2)   # real gloo collectives
        kinds = {s["kind"] for s in cal["samples"]}
        assert kinds == set(calibrate.KINDS), kinds
        summ = calibrate.summary(cal, m.pcg, m.views, world, measured_ms=5.0, ffconfig=m.ffconfig)
        assert "predicted_ms_calibrated" in summ and "predicted_ms_nominal" in summ, summ
        assert summ["comm"] and all("measured_ms" in r and "simulated_ms" in r for r in summ["comm"])
        if rank == 0:
            q.put("ok")
    except BaseException as e:  # noqa: BLE001
        q.put(repr(e))
        raise
    finally:
        dist.destroy_process_group()


def test_calibrate_step_on_two_gloo_ranks():
    from dist_util import free_port
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    mp.start_processes(_worker, args=(2, free_port(), q), nprocs=2, join=True, start_method="spawn")
    assert q.get() == "ok"
