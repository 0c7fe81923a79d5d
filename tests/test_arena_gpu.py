"""The step's device arena (csrc/runtime/arena.cpp via runtime/arena.py):
tensors allocated inside ``Arena.use()`` come out of the reserved region
(tracked live / high-water bytes, no overflow while it fits, overflow counted
when it does not), freed ranges coalesce, and a training step run out of the
arena -- eager and captured into a hipGraph whose pool is the arena -- gives
the same parameters as the default allocator."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_arena_serves_and_tracks():
    from flexflow_train_amd.runtime.arena import Arena

    a = Arena(torch.device("cuda", 0), 256 << 20)
    s0 = a.stats()
    assert s0["capacity_gb"] >= 0.268
    with a.use():
        xs = [torch.empty(8 << 20, dtype=torch.uint8, device="cuda") for _ in range(4)]
    s1 = a.stats()
    assert s1["segments"] > s0["segments"] and s1["high_water_gb"] > 0 and s1["overflow_segments"] == 0
    del xs
    torch.cuda.synchronize()
    torch.cuda.empty_cache()      # the block cache hands the segments back: ranges coalesce
    with a.use():
        big = torch.empty(200 << 20, dtype=torch.uint8, device="cuda")   # needs the coalesced range
    s2 = a.stats()
    assert s2["overflow_segments"] == 0, s2
    with a.use():
        huge = torch.empty(512 << 20, dtype=torch.uint8, device="cuda")  # does not fit: hipMalloc, counted
    s3 = a.stats()
    assert s3["overflow_segments"] >= 1 and s3["overflow_high_gb"] > 0.5
    del big, huge


def _bert(arena_bytes):
    import numpy as np
    from flexflow_train_amd import models as Z
    from flexflow_train_amd.core import AdamOptimizer, FFConfig, FFModel, LossType, MetricsType

    torch.manual_seed(0)
    m = FFModel(FFConfig())
    inputs, out, mc = Z.build("bert", m, batch_size=4, hidden_size=256, num_encoder_layers=2, num_heads=4,
                              dim_feedforward=1024, sequence_length=64, vocab_size=512)
    m.compile(optimizer=AdamOptimizer(m, alpha=1e-3), loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY,
              metrics=[MetricsType.METRICS_ACCURACY])
    ex = m.executor
    g = torch.Generator().manual_seed(0)
    for n in sorted(ex.parameter_names()):
        ex.set_parameter(n, torch.randn(ex.get_parameter(n).shape, generator=g) * 0.05)
    fn, ln = Z.synthetic("bert", mc, inputs, np.random.default_rng(0))
    feeds = {k: ex._local_piece(k, torch.as_tensor(v)) for k, v in fn.items()}
    labels = ex.local_labels(torch.as_tensor(ln))
    if arena_bytes:
        ex.enable_arena(arena_bytes)
    for _ in range(2):
        ex.train_step(feeds, labels)
    ex._eager_arena = ex.arena.stats() if arena_bytes else None
    step = ex.make_graphed_train_step(feeds, labels, warmup=1)
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    return ex, {n: ex.get_parameter(n).float().cpu() for n in sorted(ex.parameter_names())}


def test_training_step_out_of_the_arena():
    ex_a, pa = _bert(1 << 30)
    st = ex_a.arena.stats()
    assert st["segments"] > 0 and st["overflow_segments"] == 0, st
    # the one-device step replays through the native replayer (csrc/runtime/replay.cpp)
    assert ex_a.native_replay is True
    # the capture reuses the blocks the eager steps left in the pool (same
    # stream) instead of taking fresh segments next to them
    eager = ex_a._eager_arena
    assert st["high_water_gb"] <= 1.25 * eager["high_water_gb"] + 0.05, (eager, st)
    _, pb = _bert(0)
    for n in pa:
        torch.testing.assert_close(pa[n], pb[n], rtol=2e-2, atol=2e-3)


def test_ffconfig_device_arena():
    """FFConfig.device_arena: compile() sizes the arena from the liveness plan
    and the model's training steps (eager and graphed) allocate from it."""
    import numpy as np
    from flexflow_train_amd import models as Z
    from flexflow_train_amd.core import AdamOptimizer, FFConfig, FFModel, LossType, MetricsType

    cfg = FFConfig()
    cfg.device_arena = True
    m = FFModel(cfg)
    inputs, out, mc = Z.build("bert", m, batch_size=4, hidden_size=256, num_encoder_layers=2, num_heads=4,
                              dim_feedforward=1024, sequence_length=64, vocab_size=512)
    m.compile(optimizer=AdamOptimizer(m, alpha=1e-3), loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY,
              metrics=[MetricsType.METRICS_ACCURACY])
    ex = m.executor
    assert ex.arena is not None
    fn, ln = Z.synthetic("bert", mc, inputs, np.random.default_rng(0))
    feeds = {k: ex._local_piece(k, torch.as_tensor(v)) for k, v in fn.items()}
    labels = ex.local_labels(torch.as_tensor(ln))
    ex.train_step(feeds, labels)
    step = ex.make_graphed_train_step(feeds, labels, warmup=1)
    step()
    torch.cuda.synchronize()
    st = ex.arena.stats()
    assert st["capacity_gb"] > 0 and st["segments"] > 0 and st["overflow_segments"] == 0, st
