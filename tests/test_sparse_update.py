"""Row-sparse SGD update of embedding tables (runtime/executor.py
_sparse_sgd): with plain SGD it must reproduce the dense update exactly,
including repeated and out-of-range ids and bag (sum) aggregation.

The CPU test runs the torch fallback; the gpu-marked tests run the path the
DLRM bench uses: the HIP embedding kernels (wave-per-row backward with
privatized copies), the bf16 compute copy refreshed by index_copy_, and the
update inside a hipGraph capture / replay."""
import pytest
import torch

from flexflow_train_amd.core import AggrMode, DataType, FFConfig, FFModel, LossType, SGDOptimizer


def _build(sparse: bool, rows=50, dim=16, batch=8, bag=3):
    m = FFModel(FFConfig())
    ids = m.create_tensor([batch, bag], DataType.DT_INT64, name="ids")
    e = m.embedding(ids, rows, dim, AggrMode.AGGR_MODE_SUM, name="emb")
    t = m.dense(e, 8, name="fc")
    m.softmax(t, name="sm")
    m.compile(optimizer=SGDOptimizer(m, lr=0.1), loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY)
    ex = m.executor
    ex.cfg.sparse_embedding_update = sparse
    if not sparse:  # keep the flats, take the dense optimizer path
        for p in ex.params:
            p.sparse = False
        for f in ex.flats:
            f["sparse"] = False
    g = torch.Generator().manual_seed(3)
    for n in sorted(ex.parameter_names()):
        ex.set_parameter(n, torch.randn(ex.get_parameter(n).shape, generator=g) * 0.3)
    x = torch.randint(0, rows, (batch, bag), generator=g)
    x[0, 0] = x[0, 1] = x[1, 2]          # repeated rows
    x[2, 1] = rows + 27                   # out of range: reads a zero row, gets no gradient
    y = torch.randint(0, 8, (batch,), generator=g)
    return m, ex, x, y


def _params(ex):
    return {n: ex.get_parameter(n).float().cpu().clone() for n in sorted(ex.parameter_names())}


def _run(sparse: bool, steps=3):
    _, ex, x, y = _build(sparse)
    for _ in range(steps):
        ex.train_step({"ids": x}, y)
    return ex, _params(ex)


def test_sparse_matches_dense():
    ex, sp = _run(True)
    assert any(f["sparse"] for f in ex.flats), "embedding table not on the sparse path"
    _, dn = _run(False)
    for n in dn:
        torch.testing.assert_close(sp[n], dn[n], rtol=1e-6, atol=1e-6)


def test_backward_without_update_does_not_leak_rows():
    """Repeated backward() with no update(), then zero_gradients(): no stale
    touched-row lists and no stale gradient rows survive into the next step."""
    m, ex, x, y = _build(True)
    emb_steps = [s for s in ex.steps if s.op_type == "EMBEDDING"]
    for _ in range(3):
        ex.forward({"ids": x}, training=True)
        ex.backward(ex.compute_loss(y))
    assert len(emb_steps[0].ctx.extra.get("touched_rows", [])) == 1
    m.zero_gradients()
    assert not emb_steps[0].ctx.extra.get("touched_rows")
    for f in ex.flats:
        assert float(f["grad"].float().abs().sum()) == 0.0
    # dense-cleared run: the flag follows the flat, nothing is recorded
    _, ex2, x2, y2 = _build(False)
    ex2.train_step({"ids": x2}, y2)
    assert not [s for s in ex2.steps if s.op_type == "EMBEDDING"][0].ctx.extra.get("touched_rows")


def test_out_of_range_forward_reads_zero_row():
    m = FFModel(FFConfig())
    ids = m.create_tensor([4, 2], DataType.DT_INT64, name="ids")
    e = m.embedding(ids, 10, 8, AggrMode.AGGR_MODE_SUM, name="emb")
    from flexflow_train_amd.ops.embedding import EmbeddingOp

    W = torch.randn(10, 8)
    idx = torch.tensor([[1, 12], [3, -1], [9, 9], [10, 0]])

    class _Ctx:
        extra = {}

        def a(self, k, d=None):
            return "sum" if k == "aggr" else d

    (out,), _ = EmbeddingOp().forward(_Ctx(), [idx], [W])
    ref = torch.stack([W[1], W[3], 2 * W[9], W[0]])
    torch.testing.assert_close(out, ref)


def _gpu_pair(steps_eager=2, replays=3, rows=4096, dim=64, batch=256, bag=4):
    out = {}
    for sparse in (True, False):
        torch.manual_seed(0)
        _, ex, x, y = _build(sparse, rows=rows, dim=dim, batch=batch, bag=bag)
        assert ex.cfg.compute_dtype == torch.bfloat16
        for _ in range(steps_eager):
            ex.train_step({"ids": x}, y)
        torch.cuda.synchronize()
        eager = _params(ex)
        step = ex.make_graphed_train_step({"ids": x}, y, warmup=0)
        for _ in range(replays):
            step({"ids": x}, y)
        torch.cuda.synchronize()
        out[sparse] = (ex, eager, _params(ex))
    return out


@pytest.mark.gpu
def test_sparse_matches_dense_gpu_eager_and_graphed():
    from flexflow_train_amd import kernels as K

    n0 = K.STATS["sparse_sgd"]
    out = _gpu_pair()
    assert K.STATS["sparse_sgd"] > n0, "the native row-sparse SGD did not run"
    ex_s = out[True][0]
    assert any(f["sparse"] for f in ex_s.flats), "embedding table not on the sparse path"
    assert ex_s.cfg.device.type == "cuda"
    for phase in (1, 2):
        sp, dn = out[True][phase], out[False][phase]
        for n in dn:
            # fp32 atomics in the embedding backward: summation order differs run to run
            torch.testing.assert_close(sp[n], dn[n], rtol=1e-5, atol=1e-5)
    # the bf16 compute copy of the table follows the fp32 master
    f = next(f for f in ex_s.flats if f["sparse"])
    p = f["params"][0]
    torch.testing.assert_close(p.compute.float(), p.master.to(torch.bfloat16).float())


@pytest.mark.gpu
@pytest.mark.parametrize("gdt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("idt", [torch.int32, torch.int64])
def test_sparse_sgd_rows_kernel(gdt, idt):
    """The native two-launch row update against the framework formula: two
    tables of different widths, repeated ids and ids outside the table."""
    from flexflow_train_amd import kernels as K

    dev = "cuda"
    g = torch.Generator(device="cpu").manual_seed(5)
    tabs, refs = [], []
    for rows, dim, n in ((1000, 64, 700), (37, 16, 90)):
        m = torch.randn(rows, dim, generator=g).to(dev)
        gr = torch.randn(rows, dim, generator=g).to(dev, gdt)
        c = m.to(torch.bfloat16)
        idx = torch.randint(-3, rows + 5, (n,), generator=g)
        idx[:10] = idx[10:20]
        idx = idx.to(dev, idt)
        r = idx.long().clamp(0, rows - 1)
        want = m.clone()
        want[r] = m[r] - 0.05 * gr[r].float()
        wg = gr.clone()
        wg[r] = 0
        tabs.append((m, gr, c, idx))
        refs.append((want, wg))
    n0 = K.STATS["sparse_sgd"]
    assert K.sparse_sgd_rows(tabs, 0.05)
    assert K.STATS["sparse_sgd"] == n0 + 1
    for (m, gr, c, _), (want, wg) in zip(tabs, refs):
        torch.testing.assert_close(m, want, rtol=1e-6, atol=1e-6)  # the kernel may fuse the multiply-add
        torch.testing.assert_close(c, m.to(torch.bfloat16), rtol=0, atol=0)
        torch.testing.assert_close(gr, wg, rtol=0, atol=0)
