"""flexflow.pcg: the Python bindings over the C ABI (libflexflow_c.so)
(reference: bindings/python/python/flexflow/pcg/high_level.py — a cffi
sketch there).  Graphs built through the C library are the same graphs the
pybind core holds: the serialised form loads into _ffcore unchanged, shapes
agree, errors surface as exceptions, and the strategy search runs."""
import json

import pytest

from flexflow.pcg import Activation, ComputationGraph, DataType, FlexFlowError, version
from flexflow_train_amd import _ffcore as C


def _mlp():
    cg = ComputationGraph()
    x = cg.create_tensor([64, 784], DataType.FLOAT, name="x")
    h = cg.dense(x, 512, Activation.RELU, name="fc1")
    y = cg.softmax(cg.dense(h, 10, name="fc2"))
    return cg, x, h, y


def test_build_shapes_and_roundtrip(tmp_path):
    cg, x, h, y = _mlp()
    assert version().startswith("flexflow")
    assert x.dims == (64, 784) and h.dims == (64, 512) and y.dims == (64, 10)
    assert y.datatype == DataType.FLOAT
    s = cg.serialize()
    core = C.ComputationGraph.from_json(s)          # the pybind core reads it as-is
    assert core.to_json() == s
    assert ComputationGraph.deserialize(s).serialize() == s
    cg.save(str(tmp_path / "cg.json"))
    assert ComputationGraph.load(str(tmp_path / "cg.json")).num_layers == cg.num_layers
    assert cg.as_dot().startswith("digraph") and "fc1" in cg.as_dot()


def test_every_builder():
    cg = ComputationGraph()
    img = cg.create_tensor([8, 3, 32, 32], DataType.FLOAT)
    c = cg.conv2d(img, 16, 3, 3, 1, 1, 1, 1, Activation.RELU)
    assert c.dims == (8, 16, 32, 32)
    p = cg.pool2d(c, 2, 2, 2, 2)
    assert p.dims == (8, 16, 16, 16)
    b = cg.batch_norm(p, relu=True)
    f = cg.flat(b)
    assert f.dims == (8, 16 * 16 * 16)
    d = cg.dropout(cg.dense(f, 64), 0.1)
    a, bb = cg.split(d, [32, 32], axis=1)
    assert a.dims == bb.dims == (8, 32)
    cat = cg.concat([a, bb], axis=1)
    z = cg.add(cg.multiply(cat, d), cg.subtract(d, cg.divide(d, cat)))
    z = cg.scalar_add(cg.scalar_multiply(cg.gelu(cg.tanh(cg.sigmoid(cg.relu(z)))), 2.0), 1.0)
    z = cg.rsqrt(cg.exp(cg.identity(z)))
    assert cg.transpose(cg.reshape(z, [8, 4, 16]), [0, 2, 1]).dims == (8, 16, 4)
    tok = cg.create_tensor([4, 16], DataType.INT32)
    e = cg.embedding(tok, 1000, 32)
    assert e.dims == (4, 16, 32)
    ln = cg.layer_norm(e, [-1], True, 1e-5)
    att = cg.multihead_attention(ln, ln, ln, 32, 4, causal=True)
    assert att.dims == (4, 16, 32)
    assert cg.batch_matmul(att, cg.transpose(att, [0, 2, 1])).dims == (4, 16, 16)
    outs = cg.add_op({"op_type": "RELU"}, [att])
    assert len(outs) == 1 and outs[0].dims == att.dims
    C.ComputationGraph.from_json(cg.serialize())


def test_errors_raise():
    cg = ComputationGraph()
    a = cg.create_tensor([4, 8])
    b = cg.create_tensor([4, 9])
    with pytest.raises(FlexFlowError):
        cg.add(a, b)
    with pytest.raises(FlexFlowError):
        ComputationGraph.from_model("no-such-model")
    with pytest.raises(FlexFlowError):
        ComputationGraph.deserialize("{not json")


def test_search_through_the_c_abi():
    cg, x, h, y = _mlp()
    r = cg.optimize({"num_nodes": 1, "num_gpus_per_node": 8}, {"budget": 20})
    assert 0 < r.cost <= r.data_parallel_cost * (1 + 1e-9)
    rep = r.report()
    assert {"cost", "data_parallel_cost"} <= set(rep)
    pcg = r.parallel_computation_graph()
    C.ParallelComputationGraph.from_json(json.dumps(pcg))
    assert r.parallel_layer_for(h) >= 0


def test_model_zoo_through_the_c_abi():
    bert = ComputationGraph.from_model("bert")
    assert bert.num_layers > 100
    assert C.ComputationGraph.from_json(bert.serialize()).to_json() == bert.serialize()
