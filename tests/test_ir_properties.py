"""Property tests of the IR's value semantics (the reference's dtgen contract,
SURVEY §1: every IR type has equality, hashing and a JSON round trip that
preserves both).  Hypothesis generates the values: tensor shapes, parallel
shapes, operator attributes, machine views, layer configs, whole
computation graphs and their lowered PCGs, and substitutions of the bundled
rule corpus."""
import json

import pytest

hypothesis = pytest.importorskip("hypothesis")
from hypothesis import given, settings  # noqa: E402
from hypothesis import strategies as st  # noqa: E402

from flexflow_train_amd import _ffcore as C  # noqa: E402
from flexflow_train_amd.core import ActiMode, DataType, FFConfig, FFModel  # noqa: E402

SET = settings(max_examples=60, deadline=None)
DTYPES = [C.DataType.FLOAT, C.DataType.BFLOAT16, C.DataType.HALF, C.DataType.INT32, C.DataType.INT64]


@st.composite
def tensor_shapes(draw):
    dims = draw(st.lists(st.integers(1, 4096), min_size=1, max_size=5))
    return C.TensorShape(dims, draw(st.sampled_from(DTYPES)))


@st.composite
def parallel_shapes(draw):
    rank = draw(st.integers(1, 4))
    degs = [draw(st.sampled_from([1, 2, 4, 8])) for _ in range(rank)]
    dims = [d * draw(st.integers(1, 64)) for d in degs]
    s = draw(st.sampled_from([1, 2, 4]))
    c = draw(st.sampled_from([1, 2, 8]))
    return C.ParallelTensorShape(dims, degs, s, c, draw(st.sampled_from(DTYPES)))


@given(tensor_shapes())
@SET
def test_tensor_shape_roundtrip(t):
    u = C.TensorShape.from_json(t.to_json())
    assert u == t and hash(u) == hash(t) and u.to_json() == t.to_json()


@given(parallel_shapes())
@SET
def test_parallel_shape_roundtrip(p):
    q = C.ParallelTensorShape.from_json(p.to_json())
    assert q == p and hash(q) == hash(p)
    assert q.piece_shape() == p.piece_shape() and q.total_parallel_degree() == p.total_parallel_degree()


@st.composite
def op_attrs(draw):
    kind = draw(st.sampled_from(["LINEAR", "CONV2D", "EMBEDDING", "SOFTMAX", "MULTIHEAD_ATTENTION", "LAYERNORM",
                                 "POOL2D", "DROPOUT", "SCALAR_MULTIPLY", "CONCAT", "REPARTITION"]))
    acts = ["none", "relu", "sigmoid", "tanh", "gelu"]
    if kind == "LINEAR":
        return C.OpAttrs(kind, out_channels=draw(st.integers(1, 8192)), use_bias=draw(st.booleans()),
                         activation=draw(st.sampled_from(acts)))
    if kind == "CONV2D":
        k = draw(st.integers(1, 7))
        return C.OpAttrs(kind, out_channels=draw(st.integers(1, 512)), kernel_h=k, kernel_w=k,
                         stride_h=draw(st.integers(1, 3)), stride_w=draw(st.integers(1, 3)),
                         padding_h=draw(st.integers(0, 3)), padding_w=draw(st.integers(0, 3)),
                         groups=draw(st.sampled_from([1, 2, 4])), activation=draw(st.sampled_from(acts)))
    if kind == "EMBEDDING":
        return C.OpAttrs(kind, num_entries=draw(st.integers(1, 10 ** 6)), out_channels=draw(st.integers(1, 1024)),
                         aggr=draw(st.sampled_from(["none", "sum", "avg"])))
    if kind == "SOFTMAX":
        return C.OpAttrs(kind, dim=draw(st.integers(-3, 2)))
    if kind == "MULTIHEAD_ATTENTION":
        h = draw(st.sampled_from([1, 2, 4, 8, 16]))
        return C.OpAttrs(kind, embed_dim=h * draw(st.integers(1, 128)), num_heads=h, causal=draw(st.booleans()),
                         dropout=draw(st.sampled_from([0.0, 0.1])))
    if kind == "LAYERNORM":
        return C.OpAttrs(kind, axes=draw(st.lists(st.integers(-3, -1), min_size=1, max_size=2, unique=True)),
                         elementwise_affine=draw(st.booleans()), eps=draw(st.sampled_from([1e-5, 1e-12])))
    if kind == "POOL2D":
        return C.OpAttrs(kind, kernel_h=draw(st.integers(1, 4)), kernel_w=draw(st.integers(1, 4)),
                         pool_type=draw(st.sampled_from(["max", "avg"])))
    if kind == "DROPOUT":
        return C.OpAttrs(kind, rate=draw(st.sampled_from([0.0, 0.1, 0.5])), seed=draw(st.integers(0, 1 << 30)))
    if kind == "SCALAR_MULTIPLY":
        return C.OpAttrs(kind, scalar=draw(st.floats(-10, 10, allow_nan=False)))
    if kind == "CONCAT":
        return C.OpAttrs(kind, axis=draw(st.integers(-2, 3)))
    return C.OpAttrs(kind, dim=draw(st.integers(0, 3)), degree=draw(st.sampled_from([2, 4, 8])))


@given(op_attrs())
@SET
def test_op_attrs_roundtrip(op):
    q = C.OpAttrs.from_json(op.to_json())
    assert q == op and hash(q) == hash(op) and q.to_json() == op.to_json()


@st.composite
def machine_views(draw):
    nd = draw(st.integers(1, 3))
    return {"start": [draw(st.integers(0, 3)), draw(st.integers(0, 7))],
            "dimensions": [{"stride": draw(st.integers(1, 4)),
                            "projection": draw(st.sampled_from(["INTRA_NODE", "INTER_NODE"]))} for _ in range(nd)]}


@given(machine_views())
@SET
def test_machine_view_roundtrip(v):
    once = C.machine_view_roundtrip(json.dumps(v))
    assert C.machine_view_roundtrip(once) == once
    got = json.loads(once)
    assert got["dimensions"] == v["dimensions"] and got["start"] == v["start"]


@given(st.sampled_from([1, 2, 4, 8]), st.sampled_from([1, 2, 4]), st.sampled_from([1, 2, 4]),
       st.sampled_from(["none", "column", "row", "heads", "experts"]))
@SET
def test_layer_config_roundtrip(b, q, mdeg, kind):
    j = json.dumps({"batch": b, "seq": q, "model": mdeg if kind != "none" else 1, "kind": kind})
    once = C.layer_config_roundtrip(j)
    assert C.layer_config_roundtrip(once) == once
    assert json.loads(once)["batch"] == b


@st.composite
def mlp_graphs(draw):
    m = FFModel(FFConfig())
    batch = draw(st.sampled_from([8, 16, 32]))
    x = m.create_tensor([batch, draw(st.sampled_from([16, 32, 64]))], DataType.DT_FLOAT, name="x")
    t = x
    for i in range(draw(st.integers(1, 5))):
        t = m.dense(t, draw(st.sampled_from([8, 16, 32, 64])), draw(st.sampled_from(
            [ActiMode.AC_MODE_NONE, ActiMode.AC_MODE_RELU, ActiMode.AC_MODE_GELU])), name=f"d{i}")
        if draw(st.booleans()):
            t = m.dropout(t, 0.1, 7, name=f"drop{i}")
    m.softmax(t, name="sm")
    return m.cg, batch


@given(mlp_graphs(), st.sampled_from([1, 2, 4]))
@settings(max_examples=25, deadline=None)
def test_graph_roundtrips(g, world):
    cg, batch = g
    cg2 = C.ComputationGraph.from_json(cg.to_json())
    assert cg2.to_json() == cg.to_json()
    if batch % world:
        return
    pcg = C.data_parallel_pcg(cg, world)
    p2 = C.ParallelComputationGraph.from_json(pcg.to_json())
    assert p2.structurally_equal(pcg) and p2.structural_hash() == pcg.structural_hash()
    assert p2.to_json() == pcg.to_json()


def _corpus():
    from flexflow_train_amd.search.unity import DEFAULT_RULES
    return C.load_substitutions(open(DEFAULT_RULES).read())[0]


@pytest.fixture(scope="module")
def corpus():
    return _corpus()


@given(st.integers(0, 10 ** 6))
@settings(max_examples=40, deadline=None)
def test_substitution_roundtrip(corpus, i):
    s = corpus[i % len(corpus)]
    t = C.substitution_from_json(s.to_json())
    assert t.to_json() == s.to_json()
