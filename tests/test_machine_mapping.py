"""The machine-mapping DP.

The first three cases are the reference's fake-cost-table cases
(lib/compiler/test/src/compiler/machine_mapping/get_optimal_machine_mapping.cc):
the same problem trees, machine specifications, allowed views and cost
tables, with the same expected optima.  The rest exercise the DP on PCGs:
boundary-view constraints at series splits, resource splits with disjoint
devices, strided views, and the placements the executor then runs."""
import json

import pytest

from flexflow_train_amd import _ffcore as C
from flexflow_train_amd.core import ActiMode, DataType, FFConfig, FFModel
from flexflow_train_amd.search import native


def view(stride):
    return {"start": [0, 0], "dimensions": [{"stride": stride, "projection": "INTRA_NODE"}]}


MV1, MV2 = view(1), view(2)
FULL = {"num_nodes": 2, "gpus_per_node": 1}
SPLIT = {"num_nodes": 1, "gpus_per_node": 1}
ALLOWED = json.dumps([{"resource": FULL, "views": [MV1, MV2]}, {"resource": SPLIT, "views": [MV2]}])
# movement1 of the reference test: one tensor whose src / dst view sets are
# empty, so all four of its concretisations are the same key and the first
# entry (0.1) is the one the table keeps; the empty movement costs 0
TABLE = json.dumps({
    "ops": [{"leaf": "k1", "view": MV1, "cost": 1.0}, {"leaf": "k2", "view": MV1, "cost": 2.0},
            {"leaf": "k1", "view": MV2, "cost": 1.5}, {"leaf": "k2", "view": MV2, "cost": 2.5}],
    "movements": [{"tensors": [], "cost": 0.0}] + [{"tensors": [{"src": [], "dst": []}], "cost": c}
                                                   for c in (0.1, 0.2, 0.3, 0.4)]})
MOVEMENT1 = [{"src": [], "dst": []}]


def dp(tree, resources=FULL):
    r = C.machine_mapping_dp(json.dumps(tree), TABLE, ALLOWED, json.dumps(resources))
    return json.loads(r)


def _view_eq(a, b):
    return a["start"] == b["start"] and a["dimensions"] == b["dimensions"]


def test_reference_single_layer():
    r = dp({"leaf": "k1"})
    assert r["runtime"] == pytest.approx(1.0)
    assert list(r["mapping"]) == ["."] or list(r["mapping"]) == [""]
    assert _view_eq(next(iter(r["mapping"].values())), MV1)


def test_reference_pair_in_sequence():
    r = dp({"kind": "series", "movement": MOVEMENT1, "left": {"leaf": "k1"}, "right": {"leaf": "k2"}})
    assert r["runtime"] == pytest.approx(1.0 + 2.0 + 0.1)
    assert set(r["mapping"]) == {"L", "R"}
    assert _view_eq(r["mapping"]["L"], MV1) and _view_eq(r["mapping"]["R"], MV1)


def test_reference_pair_in_parallel():
    r = dp({"kind": "parallel", "left": {"leaf": "k1"}, "right": {"leaf": "k2"}})
    assert r["runtime"] == pytest.approx(2.5)
    assert _view_eq(r["mapping"]["L"], MV2) and _view_eq(r["mapping"]["R"], MV2)


def test_boundary_views_are_enumerated_and_priced():
    """A movement whose src / dst are the boundary leaves: the DP must weigh
    the leaf costs against the concretized movement (k1@mv2 + k2@mv2 + 0
    beats k1@mv1 + k2@mv1 + 5)."""
    table = json.loads(TABLE)
    table["movements"] = [
        {"tensors": [{"src": [MV1], "dst": [MV1]}], "cost": 5.0},
        {"tensors": [{"src": [MV2], "dst": [MV2]}], "cost": 0.0},
        {"tensors": [{"src": [MV1], "dst": [MV2]}], "cost": 5.0},
        {"tensors": [{"src": [MV2], "dst": [MV1]}], "cost": 5.0}]
    tree = {"kind": "series", "movement": [{"src": ["."], "dst": ["."]}], "left": {"leaf": "k1"},
            "right": {"leaf": "k2"}}
    r = json.loads(C.machine_mapping_dp(json.dumps(tree), json.dumps(table), ALLOWED, json.dumps(FULL)))
    assert r["runtime"] == pytest.approx(1.5 + 2.5)
    assert _view_eq(r["mapping"]["L"], MV2) and _view_eq(r["mapping"]["R"], MV2)


def test_nested_constraint_respects_resource_split():
    """series(parallel(a, b), c) with movements a->c, b->c: the boundary views
    fixed for a and b at the series split must lie inside the halves the
    parallel split gives them; otherwise that assignment is infeasible."""
    table = {"ops": [], "movements": []}
    for leaf in ("a", "b"):
        table["ops"] += [{"leaf": leaf, "view": MV1, "cost": 4.0}, {"leaf": leaf, "view": MV2, "cost": 4.0}]
    table["ops"] += [{"leaf": "c", "view": MV1, "cost": 1.0}, {"leaf": "c", "view": MV2, "cost": 1.0}]
    for s1 in (MV1, MV2):
        for s2 in (MV1, MV2):
            for d in (MV1, MV2):
                table["movements"].append({"tensors": [{"src": [s1], "dst": [d]}, {"src": [s2], "dst": [d]}],
                                           "cost": 0.5})
    tree = {"kind": "series", "movement": [{"src": ["L"], "dst": ["."]}, {"src": ["R"], "dst": ["."]}],
            "left": {"kind": "parallel", "left": {"leaf": "a"}, "right": {"leaf": "b"}}, "right": {"leaf": "c"}}
    r = json.loads(C.machine_mapping_dp(json.dumps(tree), json.dumps(table), ALLOWED, json.dumps(FULL)))
    # a and b side by side (4.0) beat in series (8.0): 4 + 0.5 + 1
    assert r["runtime"] == pytest.approx(5.5)


def test_resource_splits_are_disjoint_and_cover():
    for res in ({"num_nodes": 1, "gpus_per_node": 8}, {"num_nodes": 4, "gpus_per_node": 8}):
        splits = json.loads(C.machine_resource_splits(json.dumps(res)))
        assert splits
        for a, b in splits:
            na, nb = a["num_nodes"] * a["gpus_per_node"], b["num_nodes"] * b["gpus_per_node"]
            assert na + nb == res["num_nodes"] * res["gpus_per_node"]
            if a["num_nodes"] != res["num_nodes"]:
                assert b["node_offset"] == a["node_offset"] + a["num_nodes"]
            else:
                assert b["gpu_offset"] == a["gpu_offset"] + a["gpus_per_node"]
    one = json.loads(C.machine_resource_splits(json.dumps({"num_nodes": 1, "gpus_per_node": 8})))
    sizes = sorted((a["gpus_per_node"], b["gpus_per_node"]) for a, b in one)
    assert sizes == [(1, 7), (2, 6), (4, 4), (6, 2), (7, 1)]


def _towers(batch=1024):
    m = FFModel(FFConfig())
    x = m.create_tensor([batch, 1024], DataType.DT_FLOAT, name="x")
    a = m.dense(x, 32768, ActiMode.AC_MODE_RELU, name="a0")
    a = m.dense(a, 1024, name="a1")
    b = m.dense(x, 32768, ActiMode.AC_MODE_RELU, name="b0")
    b = m.dense(b, 1024, name="b1")
    m.add(a, b, name="sum")
    return m


def test_pcg_towers_split_over_devices_with_consistent_views():
    m = _towers()
    pcg = C.data_parallel_pcg(m.cg, 1)
    cm = native.cost_model()
    r2, r1 = native.machine_mapping(pcg, cm, 2), native.machine_mapping(pcg, cm, 1)
    assert r2["feasible"] and r2["runtime"] < r1["runtime"]
    by = {pcg.layer_name(n): v for n, v in r2["views"].items()}
    assert by["a0"] == by["a1"] and by["b0"] == by["b1"] and by["a0"] != by["b0"]
    assert {by["a0"], by["b0"]} == {(0,), (1,)}
    # every view the DP chose is a MachineView of the op's task space
    for n, mv in r2["machine_views"].items():
        ts = C.operator_task_space(pcg.shape(C.ValueRef(n, 0)))
        assert tuple(C.get_device_ids(ts, json.dumps(mv), C.MachineSpecification.mi355x())) == r2["views"][n]
    tree = json.loads(C.machine_mapping_problem_tree(pcg))
    assert tree["parallel"] >= 1 and tree["movements"] >= 4


def test_pcg_strided_views_allowed():
    """Degree-2 operators on 4 devices: strided views (stride 2: devices
    {0, 2} / {1, 3}) are candidates unless contiguous_only."""
    ts = [2, 1, 1]
    spec = C.MachineSpecification.mi355x(1, 4)
    views = C.get_allowed_machine_views(ts, spec)
    sets = {tuple(C.get_device_ids(ts, v, spec)) for v in views}
    assert (0, 2) in sets and (1, 3) in sets and (0, 1) in sets
    m = _towers(batch=64)
    s = json.loads(C.data_parallel_strategy(m.cg, 2))
    pcg = C.lower_strategy(m.cg, json.dumps(s), 2)[0]
    cm = native.cost_model()
    full = native.machine_mapping(pcg, cm, 4)
    cont = native.machine_mapping(pcg, cm, 4, contiguous_only=True)
    assert full["feasible"] and cont["feasible"]
    assert full["runtime"] <= cont["runtime"] + 1e-12
    assert full["cache_entries"] > 0


def test_graph_optimize_runs_final_mapping():
    """graph_optimize prices the machine-mapping DP's placements for its
    final PCG (reported as unmapped_cost vs cost) and keeps them only when
    the simulator finds them faster than whole-world placements."""
    from flexflow_train_amd.core import FFConfig
    from flexflow_train_amd.search import unity
    m = _towers(batch=64)
    cfg = FFConfig()
    cfg.batch_size = 64
    cfg.search_budget = 20
    pcg, views, rep = unity.search(m.cg, cfg, 2)
    if "unmapped_cost" in rep:   # a whole-world winner: the final DP mapping was priced
        assert rep["cost"] <= rep["unmapped_cost"] + 1e-12
        assert bool(views) == rep["algorithm"].endswith("+mapping")
    else:                        # the joint search's winner already carries its mapping
        assert views and rep.get("mapped_states", 0) > 0, rep


@pytest.mark.parametrize("nodes,gpus,want", [
    (1, 1, set()),
    (2, 2, {((2, 1), (2, 1)), ((1, 2), (1, 2))}),
    (8, 1, {((1, 1), (7, 1)), ((2, 1), (6, 1)), ((4, 1), (4, 1)), ((6, 1), (2, 1)), ((7, 1), (1, 1))}),
    (6, 1, {((1, 1), (5, 1)), ((2, 1), (4, 1)), ((4, 1), (2, 1)), ((5, 1), (1, 1))}),
    (1, 8, {((1, 1), (1, 7)), ((1, 2), (1, 6)), ((1, 4), (1, 4)), ((1, 6), (1, 2)), ((1, 7), (1, 1))}),
    (1, 6, {((1, 1), (1, 5)), ((1, 2), (1, 4)), ((1, 4), (1, 2)), ((1, 5), (1, 1))}),
], ids=["none", "2x2", "nodes8", "nodes6", "gpus8", "gpus6"])
def test_resource_splits_reference_cases(nodes, gpus, want):
    """lib/compiler/test/src/compiler/machine_mapping/get_machine_resource_splits.cc:
    power-of-two splits along the node OR the gpu dimension (never both), both
    orders; as (nodes, gpus_per_node) shape pairs."""
    splits = json.loads(C.machine_resource_splits(json.dumps({"num_nodes": nodes, "gpus_per_node": gpus})))
    got = {((a["num_nodes"], a["gpus_per_node"]), (b["num_nodes"], b["gpus_per_node"])) for a, b in splits}
    assert got == want


# ---- machine-mapping result combinators
# (lib/compiler/test/src/compiler/machine_mapping/machine_mapping_result.cc)
_MV0 = {"start": [0, 0], "dimensions": [{"stride": 1, "projection": "INTRA_NODE"}]}
_MV1 = {"start": [0, 0], "dimensions": [{"stride": 2, "projection": "INTRA_NODE"}]}
_PRE = {"runtime": 2.0, "mapping": {"L": _MV0, "R": _MV1}}
_POST = {"runtime": 4.0, "mapping": {"": _MV1}}


def _mm(x):
    return "null" if x is None else json.dumps(x)


def _res(s):
    return json.loads(s)


@pytest.mark.parametrize("pre,post", [(None, _POST), (_PRE, None), (None, None)])
def test_series_combine_infeasible(pre, post):
    for rtl in (False, True):
        assert _res(C.mm_series_combine(3.0, _mm(pre), _mm(post), rtl)) is None


def test_series_combine_feasible():
    lr = _res(C.mm_series_combine(3.0, _mm(_PRE), _mm(_POST), False))
    assert lr == {"runtime": 9.0, "mapping": {"LL": _MV0, "LR": _MV1, "R": _MV1}}
    rl = _res(C.mm_series_combine(3.0, _mm(_PRE), _mm(_POST), True))
    assert rl == {"runtime": 9.0, "mapping": {"RL": _MV0, "RR": _MV1, "L": _MV1}}


def test_parallel_combine():
    for a, b in ((None, _POST), (_PRE, None), (None, None)):
        assert _res(C.mm_parallel_combine(_mm(a), _mm(b))) is None
    assert _res(C.mm_parallel_combine(_mm(_PRE), _mm(_POST))) == \
        {"runtime": 4.0, "mapping": {"LL": _MV0, "LR": _MV1, "R": _MV1}}


def test_minimize_runtime():
    faster = {"runtime": 2.0, "mapping": {"L": _MV0, "R": _MV1}}
    slower = {"runtime": 4.0, "mapping": {"": _MV1}}
    assert _res(C.mm_minimize_runtime(_mm(None), _mm(slower))) == slower
    assert _res(C.mm_minimize_runtime(_mm(slower), _mm(None))) == slower
    assert _res(C.mm_minimize_runtime(_mm(None), _mm(None))) is None
    assert _res(C.mm_minimize_runtime(_mm(faster), _mm(slower))) == faster
    assert _res(C.mm_minimize_runtime(_mm(slower), _mm(faster))) == faster
    assert _res(C.mm_minimize_runtime(_mm(slower), _mm(slower))) == slower


def _towers_wide(batch, hid=32768, width=1024):
    m = FFModel(FFConfig())
    x = m.create_tensor([batch, width], DataType.DT_FLOAT, name="x")
    a = m.dense(x, hid, ActiMode.AC_MODE_RELU, name="a0")
    a = m.dense(a, width, name="a1")
    b = m.dense(x, hid, ActiMode.AC_MODE_RELU, name="b0")
    b = m.dense(b, width, name="b1")
    m.add(a, b, name="sum")
    return m


@pytest.mark.parametrize("batch", [8, 64])
def test_joint_unity_search_beats_substitutions_then_mapping(batch):
    """unity_algorithm.cc:37-90: every state is priced with its own machine
    mapping (one shared, content-keyed mapping cache), so the search can
    keep a graph that only pays off once placed -- two towers of huge
    Linears, each on its own GPU with no gradient sync -- which pricing
    states on whole-world placements and mapping only the winner misses."""
    m = _towers_wide(batch)
    cm = native.cost_model(use_profiles=False)   # the analytic model only: deterministic
    init = C.data_parallel_pcg(m.cg, 1)
    costs = {}
    for joint in (True, False):
        cfg = {"world": 2, "budget": 50, "time_limit": 30, "use_machine_mapping": joint,
               "enable_parameter_parallel": True}
        pcg, rep, views = C.unity_search(init, cm, json.dumps(cfg))
        rep = json.loads(rep)
        c = rep["cost"]
        if joint:
            assert rep["mapped_states"] > 0 and rep["mapping_cache_hits"] > 0, rep
            assert views, "the joint winner is a placed graph"
        else:       # substitutions first, then the DP mapping of the winner
            mm = native.machine_mapping(pcg, cm, 2)
            if mm["feasible"]:
                c = min(c, native.simulate(pcg, cm, 2, mm["views"])["iteration_time"])
        costs[joint] = c
    assert costs[True] < 0.97 * costs[False], costs


def test_mapping_cache_shared_across_graphs_is_keyed_by_content():
    """Two PCGs that differ in one operator's parallelization: mapped through
    one shared cache, the second reuses the first one's unchanged subtrees
    (hits) and gets the same runtime a fresh cache gives."""
    m = _towers_wide(64, hid=4096)
    cm = native.cost_model(use_profiles=False)
    a = C.data_parallel_pcg(m.cg, 1)
    rules = {r.name: r for r in C.generate_parallelization_substitutions(a, 2)}
    b = None
    for name, r in sorted(rules.items()):
        for nm, im in C.find_pattern_matches(r, a):
            b = C.apply_substitution(a, r, nm, im)
            if b is not None:
                break
        if b is not None:
            break
    assert b is not None
    sa, sb = C.mm_subtree_signatures(a), C.mm_subtree_signatures(b)
    assert all(len(s) == 32 for s in sa + sb)
    assert set(sa) & set(sb), "unchanged subtrees keep their content keys"
    assert set(sa) != set(sb)
    seq = C.machine_mapping_sequence([a, b], cm, 2)
    fresh_b = native.machine_mapping(b, cm, 2)["runtime"]
    assert seq[1][0] == pytest.approx(fresh_b, rel=1e-9)
    assert seq[0][0] == pytest.approx(native.machine_mapping(a, cm, 2)["runtime"], rel=1e-9)
    assert seq[1][2] > seq[0][2], "the second graph hit entries the first one stored"
