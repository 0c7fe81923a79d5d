"""The reference's op-attrs shape-inference cases with the reference's own
dimensions (lib/op-attrs/test/src/op-attrs/ops/{attention,conv_2d,embedding,
linear,softmax,dropout,element_unary,element_binary,cast,layer_norm,batch_norm,
batch_matmul,concat,flat,pool_2d,combine,reduction,repartition,replicate}.cc),
serial and parallel, against the C++ core.

Deliberate deviations, each asserted below so they stay visible:
* attention input bias: per-head [2k+v, heads] (q / k / v bias of every head,
  PyTorch's in_proj_bias split by head) where the reference has one [3 *
  embed_dim] vector; under head parallelism it is sharded with the heads
  instead of replicated.
* attention output bias under head parallelism: a partial-sum weight (added
  on replica 0 of the partial sums, like the reference's own LINEAR bias under
  reduction parallelism) where the reference replicates it.
* shard degrees must divide the dimension (the reference's conv test lifts 7
  samples to batch degree 2).
* LINEAR with a fused activation rejects partial-sum inputs (the reference's
  test uses RELU with partial sums; act(a) + act(b) != act(a + b)).
* discard-copy (replicated) inputs propagate through element-wise ops,
  softmax, dropout, layer / batch norm and concat (the reference rejects
  them): the replicated activations of a tensor-parallel region flow through
  these ops on every replica instead of forcing a re-partition.
* LAYERNORM gamma / beta span the normalized axes (PyTorch, and the
  reference's own layer_norm_kernels.cu per-column affine) where the
  reference's op-attrs gives the non-normalized dims; they are replicated
  (copy = product of the input's shard degrees) instead of sharded.
* BATCHMATMUL rejects partial-sum operands: with the executor's canonical
  replica placement the cross terms of two partial operands do not meet on
  one device.
* FLAT's end_dim is inclusive (PyTorch flatten); an empty range is the
  identity, as in the reference.
* POOL2D: the H (attribute) dim may be sharded (halo exchange); W stays
  unpartitioned.  BATCHNORM keeps the reference's rule (no spatial degrees):
  a band would normalise with its own statistics."""
import pytest

from flexflow_train_amd import _ffcore as C

F = C.DataType.FLOAT


def P(dims, degs=None, s=1, c=1):
    return C.ParallelTensorShape(list(dims), list(degs or [1] * len(dims)), s, c)


def sig(ps):
    return (list(ps.shard_degrees()), ps.sum_degree, ps.discard_copy_degree)


def serial(op, ins):
    shapes = [C.TensorShape(list(d), F) for d in ins]
    return ([list(t.dims) for t in C.infer_output_shapes(op, shapes)],
            [list(t.dims) for t in C.infer_weight_shapes(op, shapes)])


def par(op, ins):
    return ([sig(t) for t in C.infer_parallel_output_shapes(op, ins)],
            [sig(t) for t in C.infer_parallel_weight_shapes(op, ins)])


# ------------------------------------------------------------------ attention
# attention.cc: embed 32, heads 10, kdim = vdim = 32, bias; q/k/v [40, 48, 36]
ATT = dict(embed_dim=32, num_heads=10, kdim=32, vdim=32, bias=True)
QKV = [40, 48, 36]


def test_attention_serial_shapes():
    o, w = serial(C.OpAttrs("MULTIHEAD_ATTENTION", **ATT), [QKV] * 3)
    assert o == [[40, 48, 32]]
    assert w[0] == [36 * 32 * 3 + 32 * 32, 10]          # the reference's weights shape
    assert w[2] == [32]                                  # output bias
    assert w[1] == [3 * 32, 10]                          # deviation: per-head input bias


@pytest.mark.parametrize("name,inp,out,wts", [
    ("data parallelism", ([4, 1, 1], 1, 1),
     ([4, 1, 1], 1, 1), [([1, 1], 1, 4), ([1, 1], 1, 4), ([1], 1, 4)]),
    ("attention head parallelism", ([1, 1, 1], 1, 2),
     ([1, 1, 1], 2, 1), [([1, 2], 1, 1), ([1, 2], 1, 1), ([1], 2, 1)]),
    ("combined data & attention head parallelism", ([4, 1, 1], 1, 2),
     ([4, 1, 1], 2, 1), [([1, 2], 1, 4), ([1, 2], 1, 4), ([1], 2, 4)]),
], ids=lambda v: v if isinstance(v, str) else None)
def test_attention_parallel(name, inp, out, wts):
    x = P(QKV, *inp)
    o, w = par(C.OpAttrs("MULTIHEAD_ATTENTION", **ATT), [x] * 3)
    assert o == [out]
    assert w[0] == wts[0]          # weights: the reference's values in all three cases
    assert w[1:] == wts[1:]


# ------------------------------------------------------------------ conv2d
# conv_2d.cc: out 4, kernel 3x2, stride 2x2, padding 1x1, groups 1, bias;
# input [7, 4, 11, 15] -> [7, 4, 6, 8]
CONV = dict(out_channels=4, kernel_h=3, kernel_w=2, stride_h=2, stride_w=2, padding_h=1, padding_w=1, groups=1,
            use_bias=True)
IMG = [7, 4, 11, 15]


def test_conv2d_serial_shapes():
    o, w = serial(C.OpAttrs("CONV2D", **CONV), [IMG])
    assert o == [[7, 4, 6, 8]]
    assert w == [[4, 4, 3, 2], [4]]
    _, w_nb = serial(C.OpAttrs("CONV2D", **dict(CONV, use_bias=False)), [IMG])
    assert w_nb == [[4, 4, 3, 2]]        # incoming roles: input, kernel (no bias)


@pytest.mark.parametrize("name,inp,out,kernel,bias", [
    ("data parallelism", ([2, 1, 1, 1], 1, 1), ([2, 1, 1, 1], 1, 1), ([1, 1, 1, 1], 1, 2), ([1], 1, 2)),
    ("input channel parallelism", ([1, 2, 1, 1], 1, 1), ([1, 1, 1, 1], 2, 1), ([1, 2, 1, 1], 1, 1), ([1], 2, 1)),
    ("output channel parallelism", ([1, 1, 1, 1], 1, 2), ([1, 2, 1, 1], 1, 1), ([2, 1, 1, 1], 1, 1), ([2], 1, 1)),
    ("propagating sum degree", ([1, 1, 1, 1], 2, 1), ([1, 1, 1, 1], 2, 1), ([1, 1, 1, 1], 1, 2), ([1], 2, 1)),
], ids=lambda v: v if isinstance(v, str) else None)
def test_conv2d_parallel(name, inp, out, kernel, bias):
    # the reference lifts its 7-sample input to batch degree 2; pieces here
    # must divide evenly, so the parallel cases use 8 samples
    o, w = par(C.OpAttrs("CONV2D", **CONV), [P([8] + IMG[1:], *inp)])
    assert o == [out] and w == [kernel, bias]


# ------------------------------------------------------------------ embedding
# embedding.cc: 1024 entries, 128 channels, SUM; input [48, 56]
EMB = dict(num_entries=1024, out_channels=128, aggr="sum")


def test_embedding_serial_shapes():
    o, w = serial(C.OpAttrs("EMBEDDING", **EMB), [[48, 56]])
    assert o == [[48, 128]] and w == [[1024, 128]]


@pytest.mark.parametrize("name,inp,out,wt", [
    ("data parallelism", ([4, 1], 1, 1), ([4, 1], 1, 1), ([1, 1], 1, 4)),
    ("input features parallelism", ([1, 4], 1, 1), ([1, 1], 4, 1), ([1, 1], 1, 4)),
    ("output channel shard parallelism", ([1, 1], 1, 4), ([1, 4], 1, 1), ([1, 4], 1, 1)),
], ids=lambda v: v if isinstance(v, str) else None)
def test_embedding_parallel(name, inp, out, wt):
    o, w = par(C.OpAttrs("EMBEDDING", **EMB), [P([48, 56], *inp)])
    assert o == [out] and w == [wt]


# ------------------------------------------------------------------ linear
# linear.cc: out 16, bias; input [12, 16, 8]
LIN = dict(out_channels=16, use_bias=True)


def test_linear_serial_shapes_and_roles():
    o, w = serial(C.OpAttrs("LINEAR", **LIN), [[12, 16, 8]])
    assert o == [[12, 16, 16]] and w == [[8, 16], [16]]
    _, w_nb = serial(C.OpAttrs("LINEAR", out_channels=16, use_bias=False), [[12, 16, 8]])
    assert w_nb == [[8, 16]]


@pytest.mark.parametrize("name,inp,out,proj,bias", [
    ("data parallelism", ([4, 8, 1], 2, 1), ([4, 8, 1], 2, 1), ([1, 1], 1, 2 * 4 * 8), ([1], 2, 4 * 8)),
    ("reduction parallelism", ([1, 1, 4], 2, 1), ([1, 1, 1], 8, 1), ([4, 1], 1, 2), ([1], 8, 1)),
    ("output channel parallelism", ([1, 1, 1], 2, 4), ([1, 1, 4], 2, 1), ([1, 4], 1, 2), ([4], 2, 1)),
], ids=lambda v: v if isinstance(v, str) else None)
def test_linear_parallel(name, inp, out, proj, bias):
    o, w = par(C.OpAttrs("LINEAR", **LIN), [P([12, 16, 8], *inp)])
    assert o == [out] and w == [proj, bias]


def err(fn, *a):
    """None if the call raises (the reference's tl::expected error)"""
    try:
        return fn(*a)
    except Exception:
        return None


def pout(op, ins):
    return err(lambda: [sig(t) for t in C.infer_parallel_output_shapes(op, ins)])


def pwts(op, ins):
    return err(lambda: [sig(t) for t in C.infer_parallel_weight_shapes(op, ins)])


def sout(op, ins):
    return err(lambda: serial(op, ins)[0])


# ------------------------------------------------------------------ softmax / dropout / unary / cast
# softmax.cc: input [12, 14, 16]
def test_softmax():
    assert sout(C.OpAttrs("SOFTMAX", dim=1), [[12, 14, 16]]) == [[12, 14, 16]]
    assert sout(C.OpAttrs("SOFTMAX", dim=4), [[12, 14, 16]]) is None
    sm = C.OpAttrs("SOFTMAX", dim=1)
    assert pout(sm, [P([12, 14, 16], [2, 1, 4])]) == [([2, 1, 4], 1, 1)]
    assert pout(C.OpAttrs("SOFTMAX", dim=4), [P([12, 14, 16], [2, 1, 4])]) is None
    assert pout(sm, [P([12, 14, 16], [1, 2, 1])]) is None        # sharded softmax dim
    assert pout(sm, [P([12, 14, 16], [1, 1, 1], 2)]) is None     # partial sums
    assert pout(sm, [P([12, 14, 16], [1, 1, 1], 1, 2)]) == [([1, 1, 1], 1, 2)]   # deviation: copies propagate


@pytest.mark.parametrize("op", [C.OpAttrs("DROPOUT", rate=0.5, seed=1), C.OpAttrs("RELU")], ids=["dropout", "relu"])
def test_dropout_and_unary(op):
    # dropout.cc: [12, 14, 16] (2, 1, 4); element_unary.cc: [16, 32, 24] (4, 1, 8)
    assert sout(op, [[16, 32, 24]]) == [[16, 32, 24]]
    assert pout(op, [P([16, 32, 24], [4, 1, 8])]) == [([4, 1, 8], 1, 1)]
    assert pout(op, [P([16, 32, 24], [1, 1, 1], 2)]) is None
    assert pout(op, [P([16, 32, 24], [1, 1, 1], 1, 2)]) == [([1, 1, 1], 1, 2)]   # deviation


def test_cast():
    # cast.cc: [12, 16], degrees (4, 8), sum 2, copy 3 -> everything carried over
    op = C.OpAttrs("CAST", dtype="double")
    out = C.infer_output_shapes(op, [C.TensorShape([12, 16], F)])[0]
    assert list(out.dims) == [12, 16] and out.dtype == C.DataType.DOUBLE
    assert pout(op, [P([12, 16], [4, 8], 2, 3)]) == [([4, 8], 2, 3)]


# ------------------------------------------------------------------ element binary
# element_binary.cc: EW_ADD on [16, 32, 24]
def test_element_binary():
    add, A = C.OpAttrs("EW_ADD"), [16, 32, 24]
    assert sout(add, [A, A]) == [A]
    assert sout(add, [A, [17, 32, 24]]) is None
    assert pout(add, [P(A, [4, 1, 1]), P(A, [4, 1, 1])]) == [([4, 1, 1], 1, 1)]
    assert pout(add, [P(A, [1, 1, 1], 4), P(A, [1, 1, 1], 4)]) == [([1, 1, 1], 4, 1)]
    assert pout(add, [P(A, [1, 4, 1]), P(A, [1, 1, 4])]) is None   # mismatched degrees
    assert pout(add, [P(A, [1, 1, 1], 1, 4), P(A, [1, 1, 1], 1, 4)]) == [([1, 1, 1], 1, 4)]   # deviation


# ------------------------------------------------------------------ layer norm
# layer_norm.cc: axes {1, 3}, input [12, 14, 16, 18]
def test_layer_norm():
    ln = C.OpAttrs("LAYERNORM", axes=[1, 3], elementwise_affine=True, eps=0.1)
    ln_na = C.OpAttrs("LAYERNORM", axes=[1, 3], elementwise_affine=False, eps=0.1)
    I = [12, 14, 16, 18]
    o, w = serial(ln, [I])
    assert o == [I] and w == [[14, 18], [14, 18]]       # deviation: normalized axes
    assert serial(ln_na, [I])[1] == []                   # no gamma / beta without affine
    x = P(I, [2, 1, 2, 1])                               # partitioned outside the axes
    assert pout(ln, [x]) == [([2, 1, 2, 1], 1, 1)]
    assert pwts(ln, [x]) == [([1, 1], 1, 4), ([1, 1], 1, 4)]
    assert pwts(ln_na, [x]) == []
    assert pout(ln, [P(I, [1, 2, 4, 1])]) is None       # partitioned inside the axes
    assert pout(ln, [P(I, [1, 1, 1, 1], 2)]) is None    # partial sums


# ------------------------------------------------------------------ batch norm
# batch_norm.cc: input [12, 14, 16, 18], channels = dim 1
def test_batch_norm():
    bn = C.OpAttrs("BATCHNORM", affine=True, relu=False, eps=1.0, momentum=0.1)
    bn_na = C.OpAttrs("BATCHNORM", affine=False, relu=False, eps=1.0, momentum=0.1)
    I = [12, 14, 16, 18]
    o, w = serial(bn, [I])
    assert o == [I] and w == [[14], [14]]
    assert serial(bn_na, [I])[1] == []
    x = P(I, [1, 2, 1, 1])
    assert pout(bn, [x]) == [([1, 2, 1, 1], 1, 1)]
    assert pwts(bn, [x]) == [([2], 1, 1), ([2], 1, 1)]
    assert pwts(bn_na, [x]) == []
    assert pout(C.OpAttrs("BATCHNORM", affine=True, relu=True, eps=1.0, momentum=0.1), [x]) == [([1, 2, 1, 1], 1, 1)]
    assert pout(bn, [P(I, [1, 1, 1, 1], 2)]) is None                  # partial sums
    assert pout(bn, [P(I, [1, 1, 1, 2])]) is None                     # W sharded
    assert pout(bn, [P(I, [1, 1, 2, 1])]) is None                     # H sharded: bands would use local statistics


# ------------------------------------------------------------------ batch matmul
# batch_matmul.cc: lhs [b, n, m] x rhs [b, m, p], b 4 / 2, m 9 / 3, n 25 / 5, p 49 / 7
_B, _M, _N, _P = 4, 9, 25, 49


def _lhs(s, c, ob, on, om):
    return P([_B, _N, _M], [ob, on, om], s, c)


def _rhs(s, c, ob, om, op):
    return P([_B, _M, _P], [ob, om, op], s, c)


def test_batch_matmul_serial():
    bm = C.OpAttrs("BATCHMATMUL")
    assert sout(bm, [[4, 8, 6], [4, 6, 10]]) == [[4, 8, 10]]
    assert sout(bm, [[4, 8, 6], [5, 6, 10]]) is None
    assert sout(bm, [[4, 8, 6], [4, 7, 10]]) is None


@pytest.mark.parametrize("lhs,rhs,want", [
    ((1, 1, 2, 1, 1), (1, 1, 2, 1, 1), ([2, 1, 1], 1, 1)),        # data parallel
    ((1, 1, 1, 5, 1), (1, 5, 1, 1, 1), ([1, 5, 1], 1, 1)),        # n parallel
    ((1, 7, 1, 1, 1), (1, 1, 1, 1, 7), ([1, 1, 7], 1, 1)),        # p parallel
    ((1, 1, 1, 1, 3), (1, 1, 1, 3, 1), ([1, 1, 1], 3, 1)),        # reduction parallel
    ((11, 1, 1, 1, 1), (11, 1, 1, 1, 1), None),                   # both partial, no copies: invalid
    ((11, 1, 1, 1, 1), (1, 11, 1, 1, 1), None),                   # deviation: reference propagates sum 11
    ((11, 11, 1, 1, 1), (11, 11, 1, 1, 1), None),                 # deviation: reference gives sum 121
], ids=["dp", "n", "p", "reduction", "partial_both_invalid", "propagate_lhs_rejected", "partial_cross_rejected"])
def test_batch_matmul_parallel(lhs, rhs, want):
    got = pout(C.OpAttrs("BATCHMATMUL"), [_lhs(*lhs), _rhs(*rhs)])
    assert got == ([want] if want else None)


# ------------------------------------------------------------------ concat
# concat.cc: axis 1, inputs [12, {14, 16, 18}, 20]
_S = ([12, 14, 20], [12, 16, 20], [12, 18, 20])


def _cat(s, c, d0, d1, d2, degs=None):
    return [P(x, [d0, d1, d2], s, c) for x in _S] if degs is None else degs


def test_concat_serial():
    cc = C.OpAttrs("CONCAT", axis=1)
    assert sout(cc, []) is None
    assert sout(cc, list(_S) + [[12, 20, 20, 1]]) is None
    assert sout(C.OpAttrs("CONCAT", axis=3), list(_S)) is None
    assert sout(cc, list(_S)) == [[12, 48, 20]]


def test_concat_parallel():
    cc = C.OpAttrs("CONCAT", axis=1)
    assert pout(cc, _cat(2, 1, 1, 1, 1)) == [([1, 1, 1], 2, 1)]
    assert pout(cc, [P(_S[0], [1, 1, 1], 2), P(_S[1], [1, 1, 1], 4), P(_S[2], [1, 1, 1], 4)]) is None
    assert pout(cc, _cat(1, 2, 1, 1, 1)) == [([1, 1, 1], 1, 2)]
    assert pout(cc, [P(_S[0], [1, 1, 1], 1, 2), P(_S[1], [1, 1, 1], 1, 2), P(_S[2], [1, 1, 1], 1, 4)]) is None
    assert pout(cc, _cat(1, 1, 1, 2, 1)) is None                      # sharded concat axis
    assert pout(cc, _cat(1, 1, 2, 1, 4)) == [([2, 1, 4], 1, 1)]
    assert pout(cc, [P(_S[0], [2, 1, 4]), P(_S[1], [4, 1, 2]), P(_S[2], [4, 1, 2])]) is None
    assert pout(cc, _cat(3, 5, 2, 1, 4)) == [([2, 1, 4], 3, 5)]


# ------------------------------------------------------------------ flat
# flat.cc: [2, 4, 2, 3]; the reference's exclusive end_dim E is end_dim E - 1 here
@pytest.mark.parametrize("start,end,want", [
    (0, 3, [48]), (2, 3, [2, 4, 6]), (0, 1, [8, 2, 3]), (1, 2, [2, 8, 3]), (2, 1, [2, 4, 2, 3]), (2, 2, [2, 4, 2, 3]),
], ids=["all", "trailing", "leading", "middle", "empty", "single"])
def test_flat_serial(start, end, want):
    assert sout(C.OpAttrs("FLAT", start_dim=start, end_dim=end), [[2, 4, 2, 3]]) == [want]


def test_flat_parallel():
    fl = C.OpAttrs("FLAT", start_dim=1, end_dim=2)
    X = [4, 8, 6, 9]
    assert pout(fl, [P(X, [2, 1, 1, 3])]) == [([2, 1, 3], 1, 1)]
    assert pout(fl, [P(X, [1, 1, 2, 1])]) is None
    assert pout(fl, [P(X, [1, 1, 1, 1], 2)]) == [([1, 1, 1], 2, 1)]
    assert pout(fl, [P(X, [1, 1, 1, 1], 1, 2)]) == [([1, 1, 1], 1, 2)]
    assert pout(fl, [P(X, [2, 1, 1, 3], 7, 5)]) == [([2, 1, 3], 7, 5)]


# ------------------------------------------------------------------ pool2d
# pool_2d.cc: kernel 3x2, stride 2x2, padding 1x1
def _pool(t, act="none"):
    return C.OpAttrs("POOL2D", kernel_h=3, kernel_w=2, stride_h=2, stride_w=2, padding_h=1, padding_w=1, pool_type=t,
                     activation=act)


def test_pool2d():
    assert sout(_pool("max"), [[10, 12, 14]]) is None
    assert sout(_pool("max"), [[11, 13, 12, 6]]) == [[11, 13, 6, 4]]
    X = [16, 13, 12, 6]
    assert pout(_pool("max"), [P(X, [4, 1, 1, 1])]) == [([4, 1, 1, 1], 1, 1)]
    assert pout(_pool("max"), [P(X, [1, 1, 1, 1], 1, 3)]) == [([1, 1, 1, 1], 1, 3)]
    assert pout(_pool("max"), [P(X, [1, 1, 1, 1], 2)]) is None            # max is not linear
    assert pout(_pool("avg"), [P(X, [1, 1, 1, 1], 2)]) == [([1, 1, 1, 1], 2, 1)]
    assert pout(_pool("avg", "relu"), [P(X, [1, 1, 1, 1], 2)]) is None
    assert pout(_pool("max"), [P([16, 14, 20, 12], [4, 2, 5, 6])]) is None   # deviation: W sharded


# ------------------------------------------------------------------ parallel ops
# combine / reduction / repartition.cc: [12/2, 14/1, 48/3, 18/2] sum 3 copy 2
# (the reference's 16-wide dim 2 is 48 here: shard degrees divide the dims)
_X = ([12, 14, 48, 18], [2, 1, 3, 2], 3, 2)


def test_parallel_ops():
    x = P(*_X)
    assert pout(C.OpAttrs("COMBINE", dim=2, degree=3), [x]) == [([2, 1, 1, 2], 3, 2)]
    assert pout(C.OpAttrs("COMBINE", dim=2, degree=4), [x]) is None
    assert pout(C.OpAttrs("REDUCTION", degree=3), [x]) == [([2, 1, 3, 2], 1, 2)]
    assert pout(C.OpAttrs("REDUCTION", degree=4), [x]) is None
    assert pout(C.OpAttrs("REPARTITION", dim=2, degree=4), [x]) == [([2, 1, 12, 2], 3, 2)]
    # replicate.cc: [10/2, 12/1, 14/2, 16/2] sum 3 copy 2, degree 4 -> copy 8
    assert pout(C.OpAttrs("REPLICATE", degree=4), [P([10, 12, 14, 16], [2, 1, 2, 2], 3, 2)]) == [([2, 1, 2, 2], 3, 8)]
