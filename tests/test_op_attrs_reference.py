"""The reference's op-attrs shape-inference cases with the reference's own
dimensions (lib/op-attrs/test/src/op-attrs/ops/{attention,conv_2d,embedding,
linear}.cc), serial and parallel, against the C++ core.

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
  test uses RELU with partial sums; act(a) + act(b) != act(a + b))."""
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
