"""Parallel shape inference, op by op (reference: lib/op-attrs/test/src/
op-attrs/ops/*.cc — the same cases, expressed as tables over the C++ core's
infer_parallel_output_shapes / infer_parallel_weight_shapes).

Notation: P(dims, shard degrees, sum degree, discard-copy degree); an
expected shape is (shard degrees, sum degree, discard-copy degree)."""
import pytest

from flexflow_train_amd import _ffcore as C


def P(dims, degs=None, s=1, c=1):
    return C.ParallelTensorShape(list(dims), list(degs or [1] * len(dims)), s, c)


def sig(ps):
    return (list(ps.shard_degrees()), ps.sum_degree, ps.discard_copy_degree)


def outs(op, ins):
    return [sig(x) for x in C.infer_parallel_output_shapes(op, ins)]


def weights(op, ins):
    return [sig(x) for x in C.infer_parallel_weight_shapes(op, ins)]


# ---------------------------------------------------------------- LINEAR
# reference ops/linear.cc test: input [12, 16, 32] -> out_channels 16, bias
LIN = dict(out_channels=16, use_bias=True)
LINEAR_CASES = [
    # name, input (degs, sum, copy), output, projection, bias
    ("data parallel + input partial sums", ([4, 8, 1], 2, 1),
     ([4, 8, 1], 2, 1), ([1, 1], 1, 2 * 4 * 8), ([1], 2, 4 * 8)),
    ("reduction parallel", ([1, 1, 4], 2, 1),
     ([1, 1, 1], 2 * 4, 1), ([4, 1], 1, 2), ([1], 2 * 4, 1)),
    ("output-channel parallel", ([1, 1, 1], 2, 4),
     ([1, 1, 4], 2, 1), ([1, 4], 1, 2), ([4], 2, 1)),
    ("column parallel, no input sums", ([1, 1, 1], 1, 4),
     ([1, 1, 4], 1, 1), ([1, 4], 1, 1), ([4], 1, 1)),
]


@pytest.mark.parametrize("name,inp,out,proj,bias", LINEAR_CASES, ids=[c[0] for c in LINEAR_CASES])
def test_linear(name, inp, out, proj, bias):
    op = C.OpAttrs("LINEAR", **LIN)
    x = P([12, 16, 32], *inp)
    assert outs(op, [x]) == [out]
    assert weights(op, [x]) == [proj, bias]


def test_linear_serial_shapes():
    op = C.OpAttrs("LINEAR", **LIN)
    (o,) = C.infer_output_shapes(op, [C.TensorShape([12, 16, 32], C.DataType.FLOAT)])
    assert list(o.dims) == [12, 16, 16]
    w = C.infer_weight_shapes(op, [C.TensorShape([12, 16, 32], C.DataType.FLOAT)])
    assert [list(t.dims) for t in w] == [[32, 16], [16]]


def test_linear_activation_rejects_partial_sums():
    op = C.OpAttrs("LINEAR", out_channels=16, activation="relu")
    with pytest.raises(Exception):
        C.infer_parallel_output_shapes(op, [P([12, 16, 32], [1, 1, 4])])


# ---------------------------------------------------------------- EMBEDDING
# reference ops/embedding.cc test: bag (SUM) over the feature dim
EMB_CASES = [
    ("data parallel", ([2, 1], 1, 1), ([2, 1], 1, 1), ([1, 1], 1, 2)),
    ("input features parallel", ([1, 4], 1, 1), ([1, 1], 4, 1), ([1, 1], 1, 4)),
    ("output-channel parallel", ([1, 1], 1, 4), ([1, 4], 1, 1), ([1, 4], 1, 1)),
]


@pytest.mark.parametrize("name,inp,out,w", EMB_CASES, ids=[c[0] for c in EMB_CASES])
def test_embedding_bag(name, inp, out, w):
    op = C.OpAttrs("EMBEDDING", num_entries=100, out_channels=32, aggr="sum")
    x = P([8, 16], *inp)
    assert outs(op, [x]) == [out]
    assert weights(op, [x]) == [w]


def test_embedding_lookup_keeps_sequence_shards():
    # no aggregation: [B, S] -> [B, S, C]; a sharded S stays a shard
    op = C.OpAttrs("EMBEDDING", num_entries=100, out_channels=32, aggr="none")
    assert outs(op, [P([8, 16], [1, 2])]) == [([1, 2, 1], 1, 1)]
    assert outs(op, [P([8, 16], [1, 1], 1, 4)]) == [([1, 1, 4], 1, 1)]


# ---------------------------------------------------------------- ATTENTION
def test_attention_batch_and_head_parallel():
    op = C.OpAttrs("MULTIHEAD_ATTENTION", embed_dim=32, num_heads=4)
    dp = P([8, 16, 32], [2, 1, 1])
    assert outs(op, [dp] * 3) == [([2, 1, 1], 1, 1)]
    # weights replicated over the batch shards (discard copies)
    assert [w[2] for w in weights(op, [dp] * 3)] == [2, 2, 2]
    # head parallel: q/k/v discard copies -> weights sharded on heads, output partial sums
    hp = P([8, 16, 32], [1, 1, 1], 1, 2)
    assert outs(op, [hp] * 3) == [([1, 1, 1], 2, 1)]
    w = weights(op, [hp] * 3)
    assert w[0] == ([1, 2], 1, 1)


@pytest.mark.parametrize("bad", [P([8, 16, 32], [1, 1, 2]), P([8, 16, 32], None, 2, 1)],
                         ids=["feature-dim sharded", "partial-sum input"])
def test_attention_rejects(bad):
    op = C.OpAttrs("MULTIHEAD_ATTENTION", embed_dim=32, num_heads=4)
    with pytest.raises(Exception):
        C.infer_parallel_output_shapes(op, [bad] * 3)


# ---------------------------------------------------------------- CONV2D / POOL / BN
def test_conv2d_parallel_rules():
    op = C.OpAttrs("CONV2D", out_channels=8, kernel_h=3, kernel_w=3, stride_h=1, stride_w=1, padding_h=1,
                   padding_w=1, groups=1)
    assert outs(op, [P([4, 3, 8, 8], [2, 1, 1, 1])]) == [([2, 1, 1, 1], 1, 1)]
    assert weights(op, [P([4, 3, 8, 8], [2, 1, 1, 1])]) == [([1, 1, 1, 1], 1, 2), ([1], 1, 2)]
    # input-channel shards -> partial sums; output channels via discard copies
    assert outs(op, [P([4, 4, 8, 8], [1, 2, 1, 1])]) == [([1, 1, 1, 1], 2, 1)]
    assert outs(op, [P([4, 3, 8, 8], None, 1, 2)]) == [([1, 2, 1, 1], 1, 1)]
    assert weights(op, [P([4, 3, 8, 8], None, 1, 2)]) == [([2, 1, 1, 1], 1, 1), ([2], 1, 1)]
    # attribute parallelism: H bands (halo exchange, parallel/halo.py); the
    # weights are replicated over the bands
    assert outs(op, [P([4, 3, 8, 8], [1, 1, 2, 1])]) == [([1, 1, 2, 1], 1, 1)]
    assert weights(op, [P([4, 3, 8, 8], [2, 1, 2, 1])]) == [([1, 1, 1, 1], 1, 4), ([1], 1, 4)]
    with pytest.raises(Exception):   # W stays whole
        C.infer_parallel_output_shapes(op, [P([4, 3, 8, 8], [1, 1, 1, 2])])
    wide = C.OpAttrs("CONV2D", out_channels=8, kernel_h=7, kernel_w=3, stride_h=1, stride_w=1, padding_h=3,
                     padding_w=1, groups=1)
    with pytest.raises(Exception):   # 1-row bands cannot supply a 3-row halo
        C.infer_parallel_output_shapes(wide, [P([4, 3, 8, 8], [1, 1, 8, 1])])


def test_pool_and_batchnorm():
    pool = C.OpAttrs("POOL2D", kernel_h=2, kernel_w=2, stride_h=2, stride_w=2, padding_h=0, padding_w=0,
                     pool_type="max")
    assert outs(pool, [P([4, 3, 8, 8], [2, 1, 1, 1])]) == [([2, 1, 1, 1], 1, 1)]
    (o,) = C.infer_output_shapes(pool, [C.TensorShape([4, 3, 8, 8], C.DataType.FLOAT)])
    assert list(o.dims) == [4, 3, 4, 4]
    # H bands (2x2 stride 2 windows never cross a band edge: no halo)
    assert outs(pool, [P([4, 3, 8, 8], [1, 1, 2, 1])]) == [([1, 1, 2, 1], 1, 1)]
    with pytest.raises(Exception):
        C.infer_parallel_output_shapes(pool, [P([4, 3, 8, 8], [1, 1, 1, 2])])
    bn = C.OpAttrs("BATCHNORM", relu=False)
    # H bands would normalise with local statistics: rejected (a Combine first)
    with pytest.raises(Exception):
        C.infer_parallel_output_shapes(bn, [P([4, 4, 8, 8], [1, 1, 2, 1])])
    assert weights(bn, [P([4, 4, 8, 8], [1, 2, 1, 1])]) == [([2], 1, 1), ([2], 1, 1)]
    assert weights(bn, [P([4, 4, 8, 8], [2, 1, 1, 1])]) == [([1], 1, 2), ([1], 1, 2)]


# ---------------------------------------------------------------- NORMS / SOFTMAX / ELEMENTWISE
def test_layernorm_rules():
    op = C.OpAttrs("LAYERNORM", axes=[-1], elementwise_affine=True, eps=1e-5)
    assert outs(op, [P([8, 16, 32], [2, 2, 1])]) == [([2, 2, 1], 1, 1)]
    assert weights(op, [P([8, 16, 32], [2, 2, 1])]) == [([1], 1, 4), ([1], 1, 4)]
    for bad in (P([8, 16, 32], [1, 1, 2]), P([8, 16, 32], None, 2, 1)):
        with pytest.raises(Exception):
            C.infer_parallel_output_shapes(op, [bad])


def test_softmax_rules():
    op = C.OpAttrs("SOFTMAX", dim=-1)
    assert outs(op, [P([8, 10], [2, 1])]) == [([2, 1], 1, 1)]
    for bad in (P([8, 10], [1, 2]), P([8, 10], None, 2, 1)):
        with pytest.raises(Exception):
            C.infer_parallel_output_shapes(op, [bad])


def test_elementwise_rules():
    add = C.OpAttrs("EW_ADD")
    assert outs(add, [P([4, 8], [2, 1])] * 2) == [([2, 1], 1, 1)]
    assert outs(add, [P([4, 8], None, 2, 1)] * 2) == [([1, 1], 2, 1)]   # linear: sums pass through
    with pytest.raises(Exception):
        C.infer_parallel_output_shapes(add, [P([4, 8], [2, 1]), P([4, 8], [1, 1])])
    with pytest.raises(Exception):   # nonlinear ops need whole values
        C.infer_parallel_output_shapes(C.OpAttrs("DROPOUT", rate=0.1), [P([4, 8], None, 2, 1)])
    assert outs(C.OpAttrs("CAST", dtype="half"), [P([4, 8], [2, 2])]) == [([2, 2], 1, 1)]


def test_batch_matmul_rules():
    op = C.OpAttrs("BATCHMATMUL")
    assert outs(op, [P([4, 8, 16], [2, 1, 1]), P([4, 16, 8], [2, 1, 1])]) == [([2, 1, 1], 1, 1)]
    # contraction dim sharded on both sides -> partial sums
    assert outs(op, [P([4, 8, 16], [1, 1, 2]), P([4, 16, 8], [1, 2, 1])]) == [([1, 1, 1], 2, 1)]


def test_concat_and_flat():
    cat = C.OpAttrs("CONCAT", axis=1)
    assert outs(cat, [P([4, 8], [2, 1]), P([4, 6], [2, 1])]) == [([2, 1], 1, 1)]
    with pytest.raises(Exception):
        C.infer_parallel_output_shapes(cat, [P([4, 8], [1, 2]), P([4, 6], [1, 2])])
    fl = C.OpAttrs("FLAT")
    assert outs(fl, [P([4, 3, 2, 2], [2, 1, 1, 1])]) == [([2, 1], 1, 1)]
    assert outs(fl, [P([4, 3, 2, 2], [1, 3, 1, 1])]) == [([1, 3], 1, 1)]


# ---------------------------------------------------------------- PARALLEL OPS
def test_parallel_ops_degrees():
    x = P([8, 16])
    assert outs(C.OpAttrs("REPARTITION", dim=0, degree=4), [x]) == [([4, 1], 1, 1)]
    assert outs(C.OpAttrs("COMBINE", dim=0, degree=2), [P([8, 16], [4, 1])]) == [([2, 1], 1, 1)]
    assert outs(C.OpAttrs("REPLICATE", degree=3), [x]) == [([1, 1], 1, 3)]
    assert outs(C.OpAttrs("REDUCTION", degree=2), [P([8, 16], None, 4, 1)]) == [([1, 1], 2, 1)]


@pytest.mark.parametrize("kind,kw,x", [
    ("REPARTITION", dict(dim=0, degree=3), P([8, 4])),              # 8 not divisible by 3
    ("COMBINE", dict(dim=0, degree=3), P([8, 4], [4, 1])),          # 3 does not divide 4
    ("REDUCTION", dict(degree=3), P([8, 4], None, 4, 1)),           # 3 does not divide the sum degree
], ids=["repartition", "combine", "reduction"])
def test_parallel_ops_divisibility(kind, kw, x):
    with pytest.raises(Exception):
        C.infer_parallel_output_shapes(C.OpAttrs(kind, **kw), [x])


def test_total_parallel_degree_and_piece_shape():
    x = P([8, 16, 32], [2, 1, 4], 3, 5)
    # degree = product(shard degrees) x sum x discard copies (parallel_tensor_shape.cc:36-38)
    assert x.total_parallel_degree() == 2 * 4 * 3 * 5
    assert list(x.piece_shape().dims) == [4, 16, 8]
    assert list(x.reduced_shape().dims) == [8, 16, 32]
