"""Failure recovery (SURVEY §5.3 / §5.4 — the reference has no checkpoint /
resume and no failure handling): fit() writes atomic step checkpoints
(FFConfig.checkpoint_dir / checkpoint_every); a run killed mid-training by an
injected fault (FF_FAULT_INJECT_STEP) and started again resumes from the
newest complete checkpoint at the recorded iteration and ends with exactly the
weights of an uninterrupted run — on one process and on 2 gloo ranks."""
import os

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from dist_util import free_port

EPOCHS, N, B = 2, 96, 16          # 6 iterations per epoch, 12 steps


def _data():
    rng = np.random.default_rng(0)
    x = rng.standard_normal((N, 20)).astype(np.float32)
    y = rng.integers(0, 5, (N,)).astype(np.int32)
    return x, y


def _fit(ckpt_dir, every, native=True, fault=None, world=1):
    from flexflow_train_amd.core import (ActiMode, DataType, FFConfig, FFModel, LossType, MetricsType,
                                         SGDOptimizer)

    cfg = FFConfig()
    cfg.batch_size = B
    cfg.print_freq = 0
    cfg.seed = 7
    cfg.native_data_loader = native
    cfg.checkpoint_dir = ckpt_dir or ""
    cfg.checkpoint_every = every
    cfg.keep_checkpoints = 2
    m = FFModel(cfg)
    t = m.create_tensor([B, 20], DataType.DT_FLOAT)
    h = m.dense(t, 32, ActiMode.AC_MODE_RELU)
    m.softmax(m.dense(h, 5))
    m.compile(optimizer=SGDOptimizer(m, lr=0.05, momentum=0.9), loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY,
              metrics=[MetricsType.METRICS_ACCURACY])
    x, y = _data()
    if fault is not None:
        os.environ["FF_FAULT_INJECT_STEP"] = str(fault)
    try:
        m.fit(x=x, y=y, epochs=EPOCHS)
    finally:
        os.environ.pop("FF_FAULT_INJECT_STEP", None)
    ex = m.executor
    return {n: ex.get_parameter(n).detach().clone() for n in sorted(ex.parameter_names())}, ex.step_num


@pytest.mark.parametrize("native", [True, False], ids=["native-loader", "python-loader"])
def test_resume_after_injected_fault_matches_uninterrupted(tmp_path, native):
    ref, steps = _fit(None, 0, native)
    assert steps == EPOCHS * N // B
    d = str(tmp_path / "ckpt")
    with pytest.raises(RuntimeError, match="injected fault"):
        _fit(d, 4, native, fault=9)        # dies after step 9; checkpoints at steps 4 and 8
    done = sorted(os.listdir(d))
    assert done == ["step-4", "step-8"], done
    got, steps2 = _fit(d, 4, native)        # restart: resumes at step 8 (epoch 1, iteration 2)
    assert steps2 == steps
    for n in ref:
        torch.testing.assert_close(got[n], ref[n], rtol=0, atol=0)
    # only the newest keep_checkpoints complete checkpoints remain
    assert sorted(os.listdir(d)) == ["step-12", "step-8"]


def test_incomplete_checkpoint_is_ignored(tmp_path):
    from flexflow_train_amd.utils.checkpoint import latest_checkpoint

    d = tmp_path / "c"
    (d / "step-3").mkdir(parents=True)
    (d / "step-3" / "meta.json").write_text("{}")
    (d / "step-5").mkdir()                  # a rank died while writing: no meta.json
    (d / "step-5" / "rank0.pt").write_bytes(b"")
    assert latest_checkpoint(str(d)) == str(d / "step-3")
    assert latest_checkpoint(str(tmp_path / "none")) is None


def test_pruning_counts_only_complete_checkpoints(tmp_path):
    """A stale higher-numbered incomplete directory (a crashed save) neither
    counts towards keep_checkpoints nor survives the next save."""
    d = tmp_path / "ckpt"
    (d / "step-50").mkdir(parents=True)          # no meta.json: a crashed save
    (d / "step-50" / "rank0.pt").write_bytes(b"")
    _fit(str(d), 4, True)
    assert sorted(os.listdir(d)) == ["step-12", "step-8"]


def test_resume_with_other_epoch_size_restores_nothing(tmp_path):
    """A checkpoint recorded with a different iterations-per-epoch is not
    resumed: its weights are not loaded, and the step counter continues past
    its step so later checkpoints sort after it."""
    import json
    d = str(tmp_path / "ckpt")
    _fit(d, 4, True)
    meta_f = os.path.join(d, "step-12", "meta.json")
    meta = json.load(open(meta_f))
    meta["progress"]["iters_per_epoch"] = 99
    json.dump(meta, open(meta_f, "w"))
    os.remove(os.path.join(d, "step-8", "meta.json"))
    ref, steps = _fit(None, 0, True)
    with pytest.warns(UserWarning, match="not resuming"):
        got, steps2 = _fit(d, 0, True)
    assert steps2 == 12 + steps
    for n in ref:
        torch.testing.assert_close(got[n], ref[n], rtol=0, atol=0)


def test_saves_after_a_non_resumed_start_survive(tmp_path):
    """After a mismatched checkpoint is skipped, the run's own checkpoints are
    numbered after it, survive the keep-newest rotation, and are what a
    restart resumes from."""
    import json
    from flexflow_train_amd.utils.checkpoint import latest_checkpoint, read_checkpoint_meta
    d = str(tmp_path / "ckpt")
    _fit(d, 4, True)
    meta_f = os.path.join(d, "step-12", "meta.json")
    meta = json.load(open(meta_f))
    meta["progress"]["iters_per_epoch"] = 99
    json.dump(meta, open(meta_f, "w"))
    with pytest.warns(UserWarning, match="not resuming"):
        _fit(d, 4, True)                     # steps 13..24, checkpoints at 16, 20, 24
    assert sorted(os.listdir(d)) == ["step-20", "step-24"]
    last = latest_checkpoint(d)
    assert last.endswith("step-24")
    assert read_checkpoint_meta(last)["progress"]["iters_per_epoch"] == N // B


def _rank(rank, world, port, d, fault, out):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    torch.set_num_threads(1)
    import torch.distributed as dist
    try:
        params, _ = _fit(d, 4, True, fault=fault if rank == 1 else None)
        if rank == 0:
            torch.save(params, out)
    except RuntimeError as e:
        if "injected fault" not in str(e):
            raise
        os._exit(3)   # the failed rank: the peer's next collective times out / errors
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def _launch(world, d, fault, out):
    port = free_port()
    ctx = mp.get_context("spawn")
    env_t = os.environ.get("FF_DIST_TIMEOUT_S")
    os.environ["FF_DIST_TIMEOUT_S"] = "20"
    try:
        procs = [ctx.Process(target=_rank, args=(r, world, port, d, fault, out)) for r in range(world)]
        for p in procs:
            p.start()
        for p in procs:
            p.join(120)
        codes = [p.exitcode for p in procs]
        for p in procs:
            if p.is_alive():
                p.kill()
        return codes
    finally:
        if env_t is None:
            os.environ.pop("FF_DIST_TIMEOUT_S", None)
        else:
            os.environ["FF_DIST_TIMEOUT_S"] = env_t


def test_two_rank_job_restarts_from_checkpoint(tmp_path):
    """Rank 1 fails after step 9; the job is restarted (as torchrun
    --max-restarts would) and resumes from step 8 on both ranks."""
    ref_out, out = str(tmp_path / "ref.pt"), str(tmp_path / "got.pt")
    assert _launch(2, str(tmp_path / "ref_ckpt"), None, ref_out) == [0, 0]
    d = str(tmp_path / "ckpt")
    codes = _launch(2, d, 9, out)
    assert codes[1] == 3 and codes[0] != 0, codes
    assert _launch(2, d, None, out) == [0, 0]
    ref, got = torch.load(ref_out, weights_only=True), torch.load(out, weights_only=True)
    for n in ref:
        torch.testing.assert_close(got[n], ref[n], rtol=0, atol=0)
