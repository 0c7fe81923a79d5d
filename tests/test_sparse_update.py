"""Row-sparse SGD update of embedding tables (runtime/executor.py
_sparse_sgd): with plain SGD it must reproduce the dense update exactly,
including repeated and out-of-range ids and bag (sum) aggregation."""
import torch

from flexflow_train_amd.core import AggrMode, DataType, FFConfig, FFModel, LossType, SGDOptimizer


def _run(sparse: bool, steps=3):
    m = FFModel(FFConfig())
    ids = m.create_tensor([8, 3], DataType.DT_INT64, name="ids")
    e = m.embedding(ids, 50, 16, AggrMode.AGGR_MODE_SUM, name="emb")
    t = m.dense(e, 8, name="fc")
    m.softmax(t, name="sm")
    m.compile(optimizer=SGDOptimizer(m, lr=0.1), loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY)
    ex = m.executor
    ex.cfg.sparse_embedding_update = sparse
    if not sparse:  # rebuild the flats without the sparse split
        for p in ex.params:
            p.sparse = False
        for f in ex.flats:
            f["sparse"] = False
    g = torch.Generator().manual_seed(3)
    for n in sorted(ex.parameter_names()):
        ex.set_parameter(n, torch.randn(ex.get_parameter(n).shape, generator=g) * 0.3)
    x = torch.randint(0, 50, (8, 3), generator=g)
    x[0, 0] = x[0, 1] = x[1, 2]          # repeated rows
    x[2, 1] = 77                          # out of range: contributes nothing
    y = torch.randint(0, 8, (8,), generator=g)
    for _ in range(steps):
        ex.train_step({"ids": x}, y)
    return ex, {n: ex.get_parameter(n).clone() for n in sorted(ex.parameter_names())}


def test_sparse_matches_dense():
    ex, sp = _run(True)
    assert any(f["sparse"] for f in ex.flats), "embedding table not on the sparse path"
    _, dn = _run(False)
    for n in dn:
        torch.testing.assert_close(sp[n], dn[n], rtol=1e-6, atol=1e-6)
