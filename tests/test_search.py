"""Machine model, SP decomposition, lowering, simulator, machine mapping,
substitutions and search (CPU).  Mirrors the reference's compiler tests
(lib/compiler/test/src/compiler/machine_mapping/*, allowed_machine_views.cc,
series_parallel/*, lib/substitutions/test/*)."""
import json
import os

import pytest

from flexflow_train_amd import _ffcore as C
from flexflow_train_amd.core import ActiMode, DataType, FFConfig, FFModel
from flexflow_train_amd.search import native

REF_RULES = "/root/reference/substitutions/graph_subst_3_v2.json"


def mlp_cg(batch=64, hidden=64, layers=3):
    m = FFModel(FFConfig())
    x = m.create_tensor([batch, 32], DataType.DT_FLOAT, name="x")
    t = x
    for i in range(layers - 1):
        t = m.dense(t, hidden, ActiMode.AC_MODE_RELU, name=f"fc{i}")
    t = m.dense(t, 10, name="out")
    m.softmax(t, name="sm")
    return m.cg


def test_machine_spec_json_roundtrip():
    s = C.MachineSpecification.mi355x(2, 8)
    s2 = C.MachineSpecification.from_json(s.to_json())
    assert s2.num_nodes == 2 and s2.num_gpus_per_node == 8 and s2.num_devices() == 16
    assert s2.hbm_capacity == pytest.approx(288e9)


def test_allowed_machine_views_fit_and_injective():
    spec = C.MachineSpecification.mi355x(1, 4)
    views = C.get_allowed_machine_views([2, 1], spec)
    assert views
    for v in views:
        ids = C.get_device_ids([2, 1], v, spec)
        assert len(set(ids)) == 2 and all(0 <= i < 4 for i in ids)
    # stride-1 view starting at device 0 covers {0, 1}; stride 2 covers {0, 2}
    sets = {tuple(sorted(C.get_device_ids([2, 1], v, spec))) for v in views}
    assert (0, 1) in sets and (0, 2) in sets and (2, 3) in sets


def test_block_machine_view_is_canonical():
    spec = C.MachineSpecification.mi355x(1, 8)
    v = C.block_machine_view([2, 1, 2], 0, 8, spec)  # T=4 on 8 devices -> 2 implicit replicas
    ids = C.get_device_ids([2, 1, 2], v, spec)
    # ids in row-major task order; the first task dimension is the fastest
    # machine digit (reference machine_view.cc semantics), replicas interleaved
    assert ids == [0, 4, 2, 6]


def test_resource_splits():
    splits = C.get_resource_splits(0, 8)
    assert ((0, 4), (4, 4)) in splits
    assert ((0, 1), (1, 7)) in splits and ((0, 7), (7, 1)) in splits
    for a, b in splits:
        assert a[1] + b[1] == 8 and a[0] + a[1] == b[0]


def test_collective_costs_monotone():
    s = C.MachineSpecification.mi355x()
    ar2 = C.collective_cost("all_reduce", 1e9, 2, s)
    ar8 = C.collective_cost("all_reduce", 1e9, 8, s)
    assert ar2 > 0 and ar8 > 0
    assert C.collective_cost("all_reduce", 1e9, 1, s) == 0
    assert C.collective_cost("all_gather", 1e9, 8, s) < ar8


def test_sp_decomposition_strict_and_relaxed():
    chain = json.loads(C.digraph_sp_decomposition([(0, 1), (1, 2)], [], True))
    assert chain["type"] == "series" and chain["children"] == [0, 1, 2]
    diamond = json.loads(C.digraph_sp_decomposition([(0, 1), (0, 2), (1, 3), (2, 3)], [], True))
    assert diamond["type"] == "series" and diamond["children"][1]["type"] == "parallel"
    # N graph is not series-parallel
    assert C.digraph_sp_decomposition([(0, 2), (1, 2), (1, 3)], [], True) is None
    relaxed = json.loads(C.digraph_sp_decomposition([(0, 2), (1, 2), (1, 3)], [], False))
    assert relaxed is not None
    # transitive edges don't matter
    t = json.loads(C.digraph_sp_decomposition([(0, 1), (1, 2), (0, 2)], [], True))
    assert t["children"] == [0, 1, 2]


def test_cg_sp_decomposition():
    cg = mlp_cg()
    sp = native.sp_decomposition(cg, strict=True)
    assert sp is not None


def test_candidate_configs_and_dp_lowering():
    cg = mlp_cg()
    fc0 = cg.find_layer("fc0")
    cands = [json.loads(c) for c in C.candidate_configs(cg, fc0, 4)]
    kinds = {(c["batch"], c["model"], c["kind"]) for c in cands}
    assert (4, 1, "none") in kinds and (1, 4, "column") in kinds and (2, 2, "column") in kinds
    assert (1, 4, "row") not in kinds  # fused relu forbids row parallel
    dp = C.data_parallel_strategy(cg, 4)
    pcg, mapping, nops = C.lower_strategy(cg, dp, 4)
    ref = C.data_parallel_pcg(cg, 4)
    assert pcg.num_layers() == ref.num_layers()
    for n in pcg.topo_order():
        if pcg.layer_op(n).op_type == "LINEAR":
            assert pcg.shape(C.ValueRef(n, 0)).shard_degrees()[0] == 4


def test_tensor_parallel_lowering_megatron_pair():
    cg = mlp_cg(layers=3)
    s = json.loads(C.data_parallel_strategy(cg, 4))
    s["fc0"] = {"batch": 2, "seq": 1, "model": 2, "kind": "column"}
    # fc1 has relu -> only column; use 'out' as row-parallel consumer of a sharded input
    s["fc1"] = {"batch": 2, "seq": 1, "model": 2, "kind": "column"}
    s["out"] = {"batch": 2, "seq": 1, "model": 2, "kind": "row"}
    pcg, mapping, nops = C.lower_strategy(cg, json.dumps(s), 4)
    types = [pcg.layer_op(n).op_type for n in pcg.topo_order() if not pcg.is_weight_path(n)]
    assert "REPLICATE" in types and "REDUCTION" in types
    out = mapping[cg.find_layer("out")]
    sh = pcg.shape(C.ValueRef(out, 0))
    assert sh.sum_degree == 2 and sh.shard_degrees()[0] == 2


def test_convert_parallel_shape_chain():
    p = C.ParallelComputationGraph()
    x = p.add_input(C.ParallelTensorShape([8, 16]))
    x = p.parallel_partition(x, 0, 4)
    tgt = C.ParallelTensorShape([8, 16], [2, 1], 1, 2)
    v, n = C.convert_parallel_shape(p, x, tgt)
    assert p.shape(v).shard_degrees() == [2, 1] and p.shape(v).discard_copy_degree == 2 and n == 2


def test_simulator_dp_sync_and_dot():
    cg = mlp_cg(batch=16384, hidden=4096)
    cm = native.cost_model()
    p1 = C.data_parallel_pcg(cg, 1)
    p4 = C.data_parallel_pcg(cg, 4)
    r1 = native.simulate(p1, cm, 1)
    r4 = native.simulate(p4, cm, 4, dot=True)
    assert r1["sync_time"] == 0 and r4["sync_time"] > 0
    assert r4["iteration_time"] < r1["iteration_time"]  # strong-scaled batch 256
    assert r4["dot"].startswith("digraph") and "ALLREDUCE" in r4["dot"]
    assert r4["peak_memory"] < r1["peak_memory"]


def test_simulator_memory_penalty():
    cg = mlp_cg(batch=64, hidden=1024)
    spec = C.MachineSpecification.mi355x()
    spec.hbm_capacity = 1e6
    cm = C.CostModel(spec)
    r = native.simulate(C.data_parallel_pcg(cg, 1), cm, 1)
    assert r["memory_penalty"] > 0


def test_profile_table_overrides_analytic():
    cg = mlp_cg()
    p = C.data_parallel_pcg(cg, 1)
    cm = native.cost_model()
    n = next(n for n in p.topo_order() if p.layer_op(n).op_type == "LINEAR")
    f0, b0, _, _ = cm.pcg_node_cost(p, n, 1)
    ins = [p.shape(v).piece_shape() for v in p.layer_data_inputs(n)]
    outs = [p.shape(C.ValueRef(n, 0)).piece_shape()]
    cm.put_profile(C.CostModel.signature(p.layer_op(n), ins + outs), 5.0, 7.0)
    f1, b1, _, _ = cm.pcg_node_cost(p, n, 1)
    assert f1 == pytest.approx(5e-3) and b1 == pytest.approx(7e-3) and f0 != f1


def test_machine_mapping_parallel_branches():
    # two independent towers -> parallel split can run them concurrently on halves
    m = FFModel(FFConfig())
    x = m.create_tensor([1024, 1024], DataType.DT_FLOAT, name="x")
    a = m.dense(x, 32768, ActiMode.AC_MODE_RELU, name="a0")
    a = m.dense(a, 1024, name="a1")
    b = m.dense(x, 32768, ActiMode.AC_MODE_RELU, name="b0")
    b = m.dense(b, 1024, name="b1")
    m.add(a, b, name="sum")
    cm = native.cost_model()
    pcg = C.data_parallel_pcg(m.cg, 1)  # degree-1 ops: placement matters
    r = native.machine_mapping(pcg, cm, 2)
    assert r["feasible"]
    blocks = {pcg.layer_name(n): r["views"][n] for n in pcg.topo_order() if pcg.layer_name(n) in ("a0", "b0")}
    assert blocks["a0"] != blocks["b0"]
    serial = native.machine_mapping(pcg, cm, 1)
    assert r["runtime"] < serial["runtime"]


def test_substitution_partition_and_cancel():
    cg = mlp_cg()
    pcg, _ = C.pcg_from_computation_graph(cg)
    rules = {r.name: r for r in C.generate_parallelization_substitutions(pcg, 2)}
    part = rules["partition_sample_LINEAR_2"]
    matches = C.find_pattern_matches(part, pcg)
    assert len(matches) == 3
    g = pcg
    for _ in range(2):
        mt = C.find_pattern_matches(part, g)
        # rewrite the first linear that is still unpartitioned
        for nm, im in mt:
            if g.shape(im[0]).shard_degrees()[0] == 1:
                g2 = C.apply_substitution(g, part, nm, im)
                assert g2 is not None
                g = g2
                break
    n_before = sum(1 for n in g.topo_order() if g.layer_op(n).op_type in ("REPARTITION", "COMBINE"))
    cancel = rules["cancel_combine_repartition_d0_2"]
    mt = C.find_pattern_matches(cancel, g)
    assert mt
    g3 = C.apply_substitution(g, cancel, *mt[0])
    n_after = sum(1 for n in g3.topo_order() if g3.layer_op(n).op_type in ("REPARTITION", "COMBINE"))
    assert n_after == n_before - 2
    g3.reinfer_shapes()


def test_substitution_column_parallel_recreates_weights():
    cg = mlp_cg()
    pcg, _ = C.pcg_from_computation_graph(cg)
    rules = {r.name: r for r in C.generate_parallelization_substitutions(pcg, 2)}
    col = rules["column_parallel_LINEAR_2"]
    nm, im = C.find_pattern_matches(col, pcg)[0]
    g = C.apply_substitution(pcg, col, nm, im)
    lin = [n for n in g.topo_order() if g.layer_op(n).op_type == "LINEAR"]
    shards = [g.shape(w).shard_degrees() for n in lin for w in g.layer_weights(n)]
    assert [1, 2] in shards  # kernel sharded on out-channels
    g.reinfer_shapes()


@pytest.mark.skipif(not os.path.exists(REF_RULES), reason="reference rule corpus not present")
def test_legacy_rule_corpus():
    with open(REF_RULES) as f:
        coll = C.load_legacy_rules(f.read())
    assert len(coll) == 640
    dot = coll.to_dot(0)
    assert dot.startswith("digraph") and "OP_PARTITION" in dot
    converted = [coll.to_substitution(i) for i in range(len(coll))]
    ok = [s for s in converted if s is not None]
    assert len(ok) > 100
    # converted rules can be matched against a PCG without error
    pcg, _ = C.pcg_from_computation_graph(mlp_cg())
    for s in ok[:50]:
        C.find_pattern_matches(s, pcg, 16)


def test_mcmc_and_unity_never_worse_than_dp():
    cg = mlp_cg(batch=64, hidden=4096)
    cm = native.cost_model()
    cfg = {"world": 4, "budget": 200, "time_limit": 20, "seed": 3}
    pcg, rep, views = C.mcmc_search(cg, cm, json.dumps(cfg))
    rep = json.loads(rep)
    assert rep["cost"] <= rep["data_parallel_cost"] * 1.0000001
    pcg.reinfer_shapes()
    dp = C.data_parallel_pcg(cg, 4)
    cfg["budget"] = 5
    pcg2, rep2, views2 = C.unity_search(dp, cm, json.dumps(cfg))
    rep2 = json.loads(rep2)
    assert rep2["cost"] <= rep2["data_parallel_cost"] * 1.0000001 and rep2["evaluated"] > 1
    pcg3, rep3, _ = C.graph_optimize(cg, cm, json.dumps(cfg))
    assert json.loads(rep3)["predicted_speedup_over_dp"] >= 0.999


def test_search_prefers_tensor_parallel_for_huge_weights_small_batch():
    # 8 tiny samples through 16k x 16k layers: DP all-reduces ~4 GB of gradients
    m = FFModel(FFConfig())
    x = m.create_tensor([8, 16384], DataType.DT_FLOAT, name="x")
    t = m.dense(x, 16384, ActiMode.AC_MODE_RELU, name="fc0")
    t = m.dense(t, 16384, name="fc1")
    m.softmax(t, name="sm")
    cm = native.cost_model()
    cfg = {"world": 8, "budget": 400, "time_limit": 30, "seed": 1}
    pcg, rep, _ = C.mcmc_search(m.cg, cm, json.dumps(cfg))
    rep = json.loads(rep)
    assert rep["predicted_speedup_over_dp"] > 1.5
    kinds = {v["kind"] for v in rep["strategy"].values()}
    assert kinds & {"column", "row"}


def test_network_model_topologies():
    """Topology-aware network model (reference NetworkedMachineModel +
    routing + ring all-reduce expansion)."""
    from flexflow_train_amd import _ffcore as C
    t = C.NetworkTopology.mi355x_cluster(1)
    assert t.num_devices == 8 and t.num_links() == 56
    nm = C.NetworkModel(t)
    assert nm.routes(0, 5) and len(nm.routes(0, 5)[0]) == 1          # direct xGMI link
    ar = [nm.all_reduce_time(list(range(p)), 256e6) for p in (2, 4, 8)]
    assert ar[0] > ar[1] > ar[2] > 0                                   # more rings over more links
    two = C.NetworkModel(C.NetworkTopology.mi355x_cluster(2))
    assert len(two.routes(0, 9)[0]) == 2                               # via the NIC switch
    assert two.all_reduce_time(list(range(16)), 256e6) > ar[2]          # NIC-bound
    bs = C.NetworkModel(C.NetworkTopology.big_switch(8, 64e9, 1e-6))
    assert len(bs.routes(1, 2)[0]) == 2
    fd = C.NetworkModel(C.NetworkTopology.flat_deg_constraint(8, 3, 64e9, 1e-6, 7))
    assert fd.p2p_time(0, 4, 1e6) > 0
    spec = nm.calibrate(C.MachineSpecification.mi355x(1, 8))
    assert spec.collective_bw[8] > spec.collective_bw[2]
    cm = C.CostModel(spec)
    assert cm is not None
    topo, sp = C.NetworkTopology.from_config_text("num_nodes = 2\nnum_sockets_per_node = 2\nnum_gpus_per_socket = 2\n"
                                                  "nvlink_bandwidth = 18.5\nnic_bandwidth = 10.9\n")
    assert sp.num_nodes == 2 and sp.num_gpus_per_node == 4 and topo.num_devices == 8


def test_machine_spec_from_reference_config(tmp_path):
    from flexflow_train_amd.core import FFConfig
    from flexflow_train_amd.search.native import machine_spec
    p = tmp_path / "machine.cfg"
    p.write_text("num_nodes = 1\nnum_gpus_per_node = 8\nxgmi_bandwidth = 64\n")
    cfg = FFConfig()
    cfg.machine_model_file = str(p)
    spec = machine_spec(cfg, 8)
    assert 8 in spec.collective_bw and spec.collective_bw[8] > 1e11
    cfg2 = FFConfig()
    cfg2.machine_model_version = 1
    assert 4 in machine_spec(cfg2, 8).collective_bw
