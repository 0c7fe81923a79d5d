"""IR: tensor shapes, op attrs, serial + parallel shape inference, CG/PCG
JSON round trips (reference: lib/op-attrs/test, lib/pcg/test)."""
import json

import pytest

from flexflow_train_amd import _ffcore as C
from flexflow_train_amd.core import ActiMode, DataType, FFConfig, FFModel

import dist_models as M


def _pts(dims, degs=None, s=1, c=1):
    return C.ParallelTensorShape(list(dims), list(degs or [1] * len(dims)), s, c)


def test_linear_parallel_shape_rules():
    op = C.OpAttrs("LINEAR", out_channels=64, use_bias=True)
    # data parallel: batch shard, weights replicated (copy = batch degree)
    outs = C.infer_parallel_output_shapes(op, [_pts([32, 16], [4, 1])])
    assert outs[0].shard_degrees() == [4, 1]
    ws = C.infer_parallel_weight_shapes(op, [_pts([32, 16], [4, 1])])
    assert ws[0].discard_copy_degree == 4
    # column parallel: input copies -> output last dim sharded
    outs = C.infer_parallel_output_shapes(op, [_pts([32, 16], [1, 1], 1, 2)])
    assert outs[0].shard_degrees() == [1, 2]
    # row parallel: input last dim sharded -> partial sums
    outs = C.infer_parallel_output_shapes(op, [_pts([32, 16], [1, 2])])
    assert outs[0].sum_degree == 2
    with pytest.raises(Exception):
        relu = C.OpAttrs("LINEAR", out_channels=64, activation="relu")
        C.infer_parallel_output_shapes(relu, [_pts([32, 16], [1, 2])])


def test_attention_head_parallel_shapes():
    op = C.OpAttrs("MULTIHEAD_ATTENTION", embed_dim=32, num_heads=4)
    x = _pts([2, 8, 32], [1, 1, 1], 1, 2)
    out = C.infer_parallel_output_shapes(op, [x, x, x])[0]
    assert out.sum_degree == 2
    ws = C.infer_parallel_weight_shapes(op, [x, x, x])
    assert ws[0].shard_degrees() == [1, 2]


def test_softmax_rejects_sharded_axis():
    op = C.OpAttrs("SOFTMAX", dim=-1)
    with pytest.raises(Exception):
        C.infer_parallel_output_shapes(op, [_pts([8, 10], [1, 2])])


def test_parallel_op_shapes():
    x = _pts([8, 16])
    r = C.infer_parallel_output_shapes(C.OpAttrs("REPARTITION", dim=0, degree=4), [x])[0]
    assert r.shard_degrees() == [4, 1]
    c = C.infer_parallel_output_shapes(C.OpAttrs("COMBINE", dim=0, degree=2), [r])[0]
    assert c.shard_degrees() == [2, 1]
    rep = C.infer_parallel_output_shapes(C.OpAttrs("REPLICATE", degree=2), [x])[0]
    assert rep.discard_copy_degree == 2
    red = C.infer_parallel_output_shapes(C.OpAttrs("REDUCTION", degree=2), [_pts([8, 16], None, 2)])[0]
    assert red.sum_degree == 1


def test_cg_json_roundtrip_and_dot():
    m = FFModel(FFConfig())
    M.bert_tiny(m)
    cg = m.cg
    s = cg.to_json()
    cg2 = C.ComputationGraph.from_json(s)
    assert cg2.to_json() == s
    assert "digraph" in cg.as_dot()


def test_pcg_json_roundtrip_preserves_ids():
    m = FFModel(FFConfig())
    M.attention(m)
    pcg = C.data_parallel_pcg(m.cg, 2)
    p2 = C.ParallelComputationGraph.from_json(pcg.to_json())
    assert list(p2.topo_order()) == list(pcg.topo_order())
    assert p2.structural_hash() == pcg.structural_hash()
    for n in pcg.topo_order():
        for k in range(pcg.num_outputs(n)):
            assert str(p2.shape(C.ValueRef(n, k))) == str(pcg.shape(C.ValueRef(n, k)))


def test_fflayers_shape_inference_matches_torch_semantics():
    m = FFModel(FFConfig())
    x = m.create_tensor([4, 3, 8, 8], DataType.DT_FLOAT, name="img")
    t = m.conv2d(x, 6, 3, 3, 1, 1, 1, 1, ActiMode.AC_MODE_RELU, name="c1")
    assert t.dims == (4, 6, 8, 8)
    t = m.pool2d(t, 2, 2, 2, 2, 0, 0, name="p1")
    assert t.dims == (4, 6, 4, 4)
    t = m.flat(t, name="flat")
    assert t.dims == (4, 96)
    a, b = m.split(t, [32, 64], 1, name="sp")
    assert a.dims == (4, 32) and b.dims == (4, 64)
    c = m.concat([a, b], 1, name="cat")
    assert c.dims == (4, 96)
