"""Strategy equivalence on CPU: data parallel, Megatron-style tensor
parallel, attention-head parallel and embedding channel parallel, run on
2 gloo ranks, must match the single-process run parameter for parameter."""
import os

import pytest

import dist_models as M
from dist_util import assert_params_close, run_distributed, run_single, write_strategy


@pytest.fixture(scope="module")
def ref_mlp():
    return run_single(M.mlp)


def test_mlp_data_parallel(ref_mlp):
    out = run_distributed(M.mlp, 2)
    assert_params_close(out["params"], ref_mlp["params"])


def test_mlp_tensor_parallel(tmp_path, ref_mlp):
    path = str(tmp_path / "tp.json")
    write_strategy(M.mlp, 2, {"fc0": {"batch": 1, "model": 2, "kind": "column"},
                              "fc1": {"batch": 1, "model": 2, "kind": "row"}}, path)
    out = run_distributed(M.mlp, 2, path)
    assert_params_close(out["params"], ref_mlp["params"])


def test_mlp_column_then_dp_mix(tmp_path, ref_mlp):
    path = str(tmp_path / "mix.json")
    write_strategy(M.mlp, 2, {"out": {"batch": 1, "model": 2, "kind": "column"}}, path)
    out = run_distributed(M.mlp, 2, path)
    assert_params_close(out["params"], ref_mlp["params"])


def test_attention_head_parallel(tmp_path):
    ref = run_single(M.attention)
    path = str(tmp_path / "heads.json")
    write_strategy(M.attention, 2, {"mha": {"batch": 1, "model": 2, "kind": "heads"}}, path)
    out = run_distributed(M.attention, 2, path)
    assert_params_close(out["params"], ref["params"])
    dp = run_distributed(M.attention, 2)
    assert_params_close(dp["params"], ref["params"])


def test_embedding_channel_parallel(tmp_path):
    ref = run_single(M.embedding)
    path = str(tmp_path / "emb.json")
    write_strategy(M.embedding, 2, {"emb": {"batch": 1, "model": 2, "kind": "column"}}, path)
    out = run_distributed(M.embedding, 2, path)
    assert_params_close(out["params"], ref["params"])


def test_bert_tiny_data_parallel_adam():
    ref = run_single(M.bert_tiny, optimizer="adam")
    out = run_distributed(M.bert_tiny, 2, optimizer="adam")
    assert_params_close(out["params"], ref["params"], rtol=1e-3, atol=1e-4)


@pytest.mark.parametrize("fn", ["attention_ulysses", "attention_ring", "attention_ring_causal",
                                "attention_ring_contiguous_causal", "attention_ulysses_causal"])
def test_attention_sequence_parallel(tmp_path, fn):
    """Sequence-sharded attention (Ulysses all-to-all / ring attention;
    causal ring = zig-zag chunks unless ring_contiguous) matches the
    single-process run."""
    model_fn = getattr(M, fn)
    ref = run_single(model_fn)
    path = str(tmp_path / "seq.json")
    write_strategy(model_fn, 2, {"mha": {"batch": 1, "seq": 2}}, path)
    out = run_distributed(model_fn, 2, path)
    assert_params_close(out["params"], ref["params"])
    kind = "sp_all_to_all" if "ulysses" in fn else "ring_p2p"
    assert out["stats"].get(kind, 0) > 0, out["stats"]
    assert (out["stats"].get("ring_zigzag", 0) > 0) == (fn == "attention_ring_causal"), out["stats"]


@pytest.mark.parametrize("fn", ["attention_ring_causal", "attention_ring_contiguous_causal", "attention_ulysses"])
def test_attention_sequence_parallel_4way(tmp_path, fn):
    model_fn = getattr(M, fn)
    ref = run_single(model_fn)
    path = str(tmp_path / "seq4.json")
    write_strategy(model_fn, 4, {"mha": {"batch": 1, "seq": 4}}, path)
    out = run_distributed(model_fn, 4, path)
    assert_params_close(out["params"], ref["params"])


def test_dp_x_tp_4way(tmp_path):
    """Data parallel x tensor parallel on 4 ranks (2 x 2): column/row
    Linear pairs and head-parallel attention inside DP replicas."""
    ref = run_single(M.mlp)
    path = str(tmp_path / "m.json")
    write_strategy(M.mlp, 4, {"fc0": {"batch": 2, "model": 2, "kind": "column"},
                              "fc1": {"batch": 2, "model": 2, "kind": "row"}}, path)
    out = run_distributed(M.mlp, 4, path)
    assert_params_close(out["params"], ref["params"])
    ref = run_single(M.attention)
    path = str(tmp_path / "h.json")
    write_strategy(M.attention, 4, {"mha": {"batch": 2, "model": 2, "kind": "heads"}}, path)
    out = run_distributed(M.attention, 4, path)
    assert_params_close(out["params"], ref["params"])


@pytest.mark.parametrize("fn,world,cfg", [
    ("moe_replicated", 2, {"batch": 1, "model": 2, "kind": "experts"}),
    ("moe_alltoall", 2, {"batch": 1, "model": 2, "kind": "experts"}),
    ("moe_alltoall", 4, {"batch": 1, "model": 4, "kind": "experts"}),
    ("moe_alltoall", 4, {"batch": 2, "model": 2, "kind": "experts"}),
    ("moe_replicated", 4, {"batch": 2, "model": 2, "kind": "experts"}),
])
def test_moe_expert_parallel(tmp_path, fn, world, cfg):
    """Expert parallelism (replicated tokens + reduction, or all-to-all
    dispatch) matches the single-process MoE."""
    model_fn = getattr(M, fn)
    ref = run_single(model_fn)
    path = str(tmp_path / "ep.json")
    write_strategy(model_fn, world, {"moe.experts": cfg}, path)
    out = run_distributed(model_fn, world, path)
    assert_params_close(out["params"], ref["params"])
    if "alltoall" in fn:
        assert out["stats"].get("ep_all_to_all", 0) > 0, out["stats"]


@pytest.mark.parametrize("world", [2, 4])
def test_sharded_optimizer_matches(world):
    """ZeRO-style sharded Adam (reduce-scatter + shard update + all-gather)
    matches the single-process run."""
    ref = run_single(M.bert_tiny, steps=3, optimizer="adam")
    out = run_distributed(M.bert_tiny, world, steps=3, optimizer="adam",
                          cfg_over={"shard_optimizer": True, "bucket_mb": 0})
    assert_params_close(out["params"], ref["params"], rtol=1e-3, atol=1e-4)
    assert out["stats"].get("reduce_scatter", 0) > 0


def test_sharded_optimizer_regularizer_bf16():
    """ZeRO with bf16 compute and L1/L2 kernel regularizers: only this rank's
    shard of the fp32 master is current, so lambda*W must come from the
    (whole, all-gathered) compute copy -- same trajectory as the unsharded
    2-rank run at the same precision."""
    over = {"compute_dtype": "bfloat16-cpu", "bucket_mb": 0}
    ref = run_distributed(M.mlp_l2, 2, steps=4, optimizer="adam", cfg_over=over)
    out = run_distributed(M.mlp_l2, 2, steps=4, optimizer="adam", cfg_over=dict(over, shard_optimizer=True))
    assert out["stats"].get("reduce_scatter", 0) > 0
    assert_params_close(out["params"], ref["params"], rtol=1e-2, atol=1e-3)


def test_recompile_switches_strategy(tmp_path):
    """RecompileState: after 2 DP steps switch to a tensor-parallel strategy
    (alter = import a strategy file) and continue; the result matches 4
    single-process steps exactly (weights + Adam moments carried over)."""
    from dist_util import run_recompile
    ref = run_single(M.mlp, steps=4, optimizer="adam")
    path = str(tmp_path / "tp.json")
    write_strategy(M.mlp, 2, {"fc0": {"batch": 1, "model": 2, "kind": "column"},
                              "fc1": {"batch": 1, "model": 2, "kind": "row"}}, path)
    out = run_recompile(M.mlp, 2, path, steps_before=2, steps_after=2)
    assert out["recompilations"] == 1
    assert_params_close(out["params"], ref["params"], rtol=1e-3, atol=1e-4)


@pytest.mark.parametrize("optimizer", ["sgd", "adam"])
def test_parameter_server_sync_matches(optimizer):
    """ParamSync::PS (reference config.h:38-42, optimizer_kernel.cu:43-70):
    gradients reduced to the group leader, leader-only update, weights
    broadcast back — same trajectory as the single-process run."""
    ref = run_single(M.mlp, steps=3, optimizer=optimizer)
    out = run_distributed(M.mlp, 2, steps=3, optimizer=optimizer, cfg_over={"parameter_sync": "ps"})
    assert_params_close(out["params"], ref["params"], rtol=1e-4, atol=1e-5)
    assert out["stats"].get("reduce", 0) > 0 and out["stats"].get("broadcast", 0) > 0


def test_cnn_data_parallel():
    """Conv / pool / residual CNN: data parallel on 2 ranks matches 1 process."""
    ref = run_single(M.cnn, steps=2)
    out = run_distributed(M.cnn, 2, steps=2)
    assert_params_close(out["params"], ref["params"], rtol=1e-4, atol=1e-5)


def test_cnn_channel_parallel_conv(tmp_path):
    """Output-channel (model) parallel conv: the weight is split on its out
    channels, the activations re-combined (op-attrs conv_2d.cc:85-142)."""
    ref = run_single(M.cnn, steps=2)
    path = str(tmp_path / "conv_tp.json")
    write_strategy(M.cnn, 2, {"c2": {"batch": 1, "model": 2, "kind": "column"}}, path)
    out = run_distributed(M.cnn, 2, path, steps=2)
    assert_params_close(out["params"], ref["params"], rtol=1e-4, atol=1e-5)


def test_cnn_input_channel_parallel_conv(tmp_path):
    """Input-channel (row) parallel conv: partial-sum outputs reduced by RCCL/gloo."""
    ref = run_single(M.cnn, steps=2)
    path = str(tmp_path / "conv_row.json")
    write_strategy(M.cnn, 2, {"c2": {"batch": 1, "model": 2, "kind": "row"}}, path)
    out = run_distributed(M.cnn, 2, path, steps=2)
    assert_params_close(out["params"], ref["params"], rtol=1e-4, atol=1e-5)


def _const_model(m):
    """A Linear fed x + a constant row (FFModel.create_constant_array): the
    constant has no sample dimension and must stay whole on every rank."""
    import numpy as np
    import torch
    from flexflow_train_amd.core import DataType
    x = m.create_tensor([8, 6], DataType.DT_FLOAT, name="x")
    c = m.create_constant_array(np.linspace(-1, 1, 6, dtype=np.float32).reshape(1, 6), name="row")
    m.softmax(m.dense(m.relu(m.add(x, c)), 4, name="fc"))
    g = torch.Generator().manual_seed(3)
    return {"x": torch.randn(8, 6, generator=g)}, torch.randint(0, 4, (8, 1), generator=g, dtype=torch.int32)


def test_constant_input_replicated_under_data_parallel():
    single = run_single(_const_model, steps=3)
    multi = run_distributed(_const_model, world=2, steps=3)
    assert_params_close(single["params"], multi["params"])


def test_strided_machine_view_placement(tmp_path):
    """Inter-operator placement on STRIDED machine views (reference
    machine_view.cc:45-101, mapper.cc:335-430): on 4 gloo ranks the two
    towers run batch-parallel on devices {0, 2} and {1, 3}; the sum and the
    loss on all four.  Same parameters as the single-process run."""
    import json as _json
    from flexflow_train_amd import _ffcore as C
    from flexflow_train_amd.core import FFConfig, FFModel
    from flexflow_train_amd.search.strategy import export_strategy

    ref = run_single(M.towers, steps=3)
    m = FFModel(FFConfig())
    M.towers(m)
    s = _json.loads(C.data_parallel_strategy(m.cg, 4))
    for k in s:
        s[k]["batch"] = 2
    pcg = C.lower_strategy(m.cg, _json.dumps(s), 4)[0]
    views = {}
    for n in pcg.topo_order():
        name = pcg.layer_name(n).split(".")[0]
        if name in ("a0", "a1"):
            views[n] = (0, 2)
        elif name in ("b0", "b1"):
            views[n] = (1, 3)
    path = str(tmp_path / "strided.json")
    export_strategy(path, pcg, views, {"world": 4, "source": "test"})
    out = run_distributed(M.towers, 4, path, steps=3)
    assert_params_close(out["params"], ref["params"])
    assert out["stats"]["all_to_all"] + out["stats"]["p2p"] + out["stats"]["all_gather"] + out["stats"].get("send_recv", 0) > 0


@pytest.mark.parametrize("world", [2, 4])
def test_attribute_parallel_conv_halo(tmp_path, world):
    """Attribute (spatial) parallelism: conv / pool layers on H bands with
    halo exchange (parallel/halo.py) train exactly like the single process."""
    ref = run_single(M.cnn_spatial)
    path = str(tmp_path / "spatial.json")
    spatial = {"batch": 1, "seq": world}
    pcg = write_strategy(M.cnn_spatial, world, {k: spatial for k in ("c1", "p1", "c2", "res", "r2", "p2")}, path)
    from flexflow_train_amd import _ffcore as C
    degs = {pcg.layer_name(n): list(pcg.shape(C.ValueRef(n, 0)).shard_degrees()) for n in pcg.topo_order()}
    assert degs["c1"] == [1, 1, world, 1] and degs["p2"] == [1, 1, world, 1]
    out = run_distributed(M.cnn_spatial, world, path)
    assert_params_close(out["params"], ref["params"])
    # 4 window ops x (forward extend + backward fold) x 2 steps, minus c1's
    # input gradient (the image needs none)
    assert out["stats"].get("halo", 0) >= 2 * 7, out["stats"]


@pytest.mark.parametrize("optimizer", ["adam", "sgd"])
def test_checkpoint_reshard_2_to_4_ranks_resumes_exactly(tmp_path, optimizer):
    """a 2-rank data-parallel run (Adam / momentum SGD) saved
    after 2 steps resumes on 4 ranks under a different (tensor-parallel)
    strategy -- weights, optimizer state and step counters re-sliced -- and
    after 2 more steps matches the uninterrupted 4-step run to 1e-5."""
    from dist_util import run_checkpointed
    from flexflow_train_amd.utils.checkpoint import read_checkpoint_meta

    # the uninterrupted reference: one process, 4 steps (every strategy is
    # numerically the single-process model)
    if optimizer == "adam":
        ref = run_single(M.mlp, steps=4, optimizer="adam")
    else:   # the worker's SGD has momentum 0.9: a reference with the same
        for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
            os.environ.pop(k, None)
        ref = {"params": _train_momentum(M.mlp, 4)}
    tp4 = str(tmp_path / "tp4.json")
    write_strategy(M.mlp, 4, {"fc0": {"batch": 1, "model": 4, "kind": "column"},
                              "fc1": {"batch": 1, "model": 4, "kind": "row"}}, tp4)
    ck = str(tmp_path / "ck")
    out = run_checkpointed(M.mlp, ck, save_world=2, load_world=4, load_strategy=tp4, optimizer=optimizer)
    meta = read_checkpoint_meta(ck)
    assert meta["world"] == 2 and meta["step"] == 2
    assert os.path.exists(os.path.join(ck, "model.json")) and os.path.exists(os.path.join(ck, "strategy.json"))
    assert out["meta"].get("resharded") is True and out["meta"].get("optimizer_resharded") is True
    assert_params_close(out["params"], ref["params"], rtol=1e-5, atol=1e-5)


def _train_momentum(model_fn, steps):
    from flexflow_train_amd.core import FFConfig, FFModel, LossType, MetricsType, SGDOptimizer
    import torch

    cfg = FFConfig()
    cfg.seed = 0
    cfg.only_data_parallel = True
    model = FFModel(cfg)
    feeds, labels = model_fn(model)
    model.compile(optimizer=SGDOptimizer(model, lr=0.05, momentum=0.9),
                  loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY, metrics=[MetricsType.METRICS_ACCURACY])
    ex = model.executor
    g = torch.Generator().manual_seed(0)
    for name in sorted(ex.parameter_names()):
        ex.set_parameter(name, torch.randn(ex.get_parameter(name).shape, generator=g) * 0.2)
    for _ in range(steps):
        ex.train_step(feeds, labels)
    return {n: ex.get_parameter(n).detach().cpu().clone() for n in sorted(ex.parameter_names())}
