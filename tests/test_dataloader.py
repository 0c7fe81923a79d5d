"""Native batch prefetcher (csrc/ffcore/src/dataloader.cc) and the rank-local
loader over it: row selection, shuffling, slot recycling, and fit() through it
matching fit() through the host loaders."""
import numpy as np
import pytest
import torch

from flexflow_train_amd import _ffcore as C


def _drain(pf, n, arrs_slots):
    out = []
    for _ in range(n):
        slot, b = pf.next()
        out.append((b, [t.clone() for t in arrs_slots[slot]]))
        pf.release(slot)
    return out


def _make(arrays, rows, batch, shuffle=False, seed=0, depth=3, workers=2):
    pf = C.BatchPrefetcher(arrays, rows, batch, shuffle, seed, depth, workers)
    slots = []
    for s in range(pf.depth):
        sl = []
        for i, a in enumerate(arrays):
            lo, hi = rows[i]
            t = torch.empty((hi - lo,) + a.shape[1:], dtype=torch.from_numpy(a[:1]).dtype)
            pf.set_slot(s, i, t.data_ptr())
            sl.append(t)
        slots.append(sl)
    return pf, slots


def test_prefetcher_rows_in_order():
    x = np.arange(40 * 3, dtype=np.float32).reshape(40, 3)
    y = np.arange(40, dtype=np.int64)
    pf, slots = _make([x, y], [(2, 6), (2, 6)], batch=8)
    assert pf.iters_per_epoch == 5
    pf.start()
    got = _drain(pf, 12, slots)  # crosses two epoch boundaries
    pf.stop()
    for b, (xs, ys) in got:
        i = b % 5
        np.testing.assert_array_equal(ys.numpy(), y[i * 8 + 2:i * 8 + 6])
        np.testing.assert_array_equal(xs.numpy(), x[i * 8 + 2:i * 8 + 6])
    assert [b for b, _ in got] == list(range(12))


def test_prefetcher_shuffle_is_a_permutation_per_epoch():
    y = np.arange(64, dtype=np.int64)
    pf, slots = _make([y], [(0, 16)], batch=16, shuffle=True, seed=7, depth=4, workers=3)
    pf.start()
    got = _drain(pf, 8, slots)
    pf.stop()
    e0 = np.concatenate([t[0].numpy() for _, t in got[:4]])
    e1 = np.concatenate([t[0].numpy() for _, t in got[4:]])
    assert sorted(e0) == list(range(64)) and sorted(e1) == list(range(64))
    assert not np.array_equal(e0, np.arange(64)) and not np.array_equal(e0, e1)
    # the prefetcher reports the same permutation it staged
    assert pf.sample_of(1, 3) == got[1][1][0][3].item()


def test_prefetcher_rejects_bad_input():
    with pytest.raises(ValueError):
        C.BatchPrefetcher([np.zeros((4, 2), np.float32)], [(0, 9)], 8, False, 0, 2, 1)
    with pytest.raises(ValueError):
        C.BatchPrefetcher([np.zeros((10, 2), np.float32), np.zeros(9, np.int64)], [(0, 4), (0, 4)], 4, False, 0,
                          2, 1)


def test_fit_native_matches_host_loader():
    from flexflow_train_amd.core import ActiMode, DataType, FFConfig, FFModel, LossType, MetricsType, SGDOptimizer

    rng = np.random.default_rng(0)
    X = rng.standard_normal((256, 32)).astype(np.float32)
    Y = rng.integers(0, 10, (256, 1)).astype(np.int32)

    def run(native):
        cfg = FFConfig()
        cfg.batch_size = 32
        cfg.print_freq = 0
        cfg.native_data_loader = native
        m = FFModel(cfg)
        x = m.create_tensor([32, 32], DataType.DT_FLOAT, name="x")
        t = m.dense(x, 64, ActiMode.AC_MODE_RELU, name="d1")
        m.softmax(m.dense(t, 10, name="d2"))
        m.compile(optimizer=SGDOptimizer(m, lr=0.05), loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY,
                  metrics=[MetricsType.METRICS_ACCURACY])
        assert (m._native_loader([X], Y, 32) is not None) == native
        for n in m.executor.parameter_names():
            m.executor.set_parameter(n, torch.linspace(-0.1, 0.1, m.executor.get_parameter(n).numel())
                                     .reshape(m.executor.get_parameter(n).shape))
        m.fit(x=X, y=Y, epochs=2)
        return {n: m.executor.get_parameter(n) for n in m.executor.parameter_names()}

    a, b = run(True), run(False)
    for n in a:
        torch.testing.assert_close(a[n], b[n], rtol=1e-5, atol=1e-6)
