"""Substitutions end to end: the TASO corpus converted and applied, the
Linear + ReLU fusion case of the reference's substitution test, the rule-set
JSON round trip, and Unity driven by rewrites that MCMC cannot express.

Reference: lib/substitutions/test/src/substitutions/substitution.cc
(evaluate / apply_substitution of a Linear+ReLU -> fused Linear rule, checked
by isomorphism), lib/compiler/src/unity_algorithm.cc:27-91 (best-first over
every substitution at every match), substitutions/graph_subst_3_v2.json."""
import collections
import json
import os

import pytest

from flexflow_train_amd import _ffcore as C
from flexflow_train_amd.core import ActiMode, DataType, FFConfig, FFModel
from flexflow_train_amd.search import native, unity

REF_RULES = "/root/reference/substitutions/graph_subst_3_v2.json"
BUNDLED = unity.DEFAULT_RULES


def _bundled():
    with open(BUNDLED) as f:
        return C.load_substitutions(f.read())[0]


def _ops(g):
    return collections.Counter(g.layer_op(n).op_type for n in g.topo_order() if not g.is_weight_path(n))


def test_bundled_rule_set_covers_the_corpus():
    with open(BUNDLED) as f:
        meta = json.load(f)
    assert meta["rules_in_source"] == 640
    subs = _bundled()
    assert len(subs) >= 595
    names = {s.name for s in subs}
    assert len(names) == len(subs)
    assert sum(n.endswith("_rev") for n in names) > 0          # right-to-left forms
    assert all(n.startswith("legacy_taso_rule_") for n in names)


@pytest.mark.skipif(not os.path.exists(REF_RULES), reason="reference rule corpus not present")
def test_corpus_conversion_matches_bundled_and_explains_the_rest():
    with open(REF_RULES) as f:
        subs, skipped = C.load_substitutions(f.read())
    assert len(subs) + len(skipped) == 640
    assert len(subs) == len(_bundled())
    # every rule left out uses an activation as a Linear weight (docs/TASO_RULES.md)
    for s in skipped:
        assert "weight" in s, s
    coll = C.load_legacy_rules(open(REF_RULES).read())
    why = [coll.conversion_failure(i) for i in range(len(coll))]
    assert sum(1 for w in why if w) == len(skipped) + sum(1 for s in subs if s.name.endswith("_rev"))


def test_substitution_json_round_trip():
    subs = _bundled()
    pcg, _ = C.pcg_from_computation_graph(_mlp3d().cg)
    subs += list(C.generate_parallelization_substitutions(pcg, 2))
    for s in subs:
        j = s.to_json()
        assert C.substitution_from_json(j).to_json() == j


def _mlp3d():
    m = FFModel(FFConfig())
    x = m.create_tensor([8, 16, 64], DataType.DT_FLOAT, name="x")
    t = m.dense(x, 128, name="fc0")
    t = m.relu(t, name="r0")
    t = m.dense(t, 64, name="fc1")
    t = m.add(t, x, name="res")
    t = m.dense(t, 64, ActiMode.AC_MODE_RELU, name="fc2")
    m.softmax(m.dense(t, 10, name="out"))
    return m


@pytest.mark.parametrize("world", [1, 2])
def test_corpus_rules_apply_and_preserve_shapes(world):
    """Converted corpus rules match a data-parallel PCG of 3-D activations;
    every successful rewrite keeps the rewritten outputs' parallel shapes and
    re-infers cleanly, and some fuse the ReLU into its Linear."""
    pcg = C.data_parallel_pcg(_mlp3d().cg, world)
    before = _ops(pcg)
    applied, fused = 0, 0
    for s in _bundled():
        for nm, im in C.find_pattern_matches(s, pcg, 64):
            g = C.apply_substitution(pcg, s, nm, im)
            if g is None:
                continue
            applied += 1
            g.reinfer_shapes()
            outs = [n for n in g.topo_order() if g.layer_op(n).op_type == "SOFTMAX"]
            assert len(outs) == 1
            sm_old = next(n for n in pcg.topo_order() if pcg.layer_op(n).op_type == "SOFTMAX")
            assert g.shape(C.ValueRef(outs[0], 0)) == pcg.shape(C.ValueRef(sm_old, 0))
            if _ops(g)["RELU"] < before["RELU"]:
                fused += 1
    assert applied >= 5 and fused >= 3


def _reference_case(fused: bool):
    """The PCG of the reference test: input [4, 24] with batch degree 2,
    dense 16, gelu, dense 12 (no bias) "mm_match", relu "relu_match",
    dense 8 (relu); ``fused``: dense 12 with the relu inside."""
    m = FFModel(FFConfig())
    x = m.create_tensor([4, 24], DataType.DT_FLOAT, name="x")
    t = m.dense(x, 16, name="d0")
    t = m.gelu(t, name="g")
    if fused:
        t = m.dense(t, 12, ActiMode.AC_MODE_RELU, use_bias=False, name="mm_match")
    else:
        t = m.dense(t, 12, use_bias=False, name="mm_match")
        t = m.relu(t, name="relu_match")
    m.dense(t, 8, ActiMode.AC_MODE_RELU, name="d2")
    return C.data_parallel_pcg(m.cg, 2)


def test_linear_relu_fusion_matches_reference_case():
    pcg = _reference_case(fused=False)
    rules = {r.name: r for r in C.generate_parallelization_substitutions(pcg, 2)}
    rule = rules["fuse_linear_relu"]
    matches = C.find_pattern_matches(rule, pcg)
    # the only Linear(no activation) -> ReLU pair; d0 -> gelu is another activation
    assert len(matches) == 1
    nm, im = matches[0]
    assert [pcg.layer_name(n) for n in nm] == ["mm_match", "relu_match"]
    g = C.apply_substitution(pcg, rule, nm, im)
    assert g is not None
    g.reinfer_shapes()
    correct = _reference_case(fused=True)
    assert g.structural_hash() == correct.structural_hash()
    assert _ops(g)["RELU"] == 0 and _ops(g)["LINEAR"] == 3
    gelu = rules["fuse_linear_gelu"]
    assert len(C.find_pattern_matches(gelu, pcg)) == 1   # d0 -> gelu


def _relu_chain():
    m = FFModel(FFConfig())
    x = m.create_tensor([256, 2048], DataType.DT_FLOAT, name="x")
    t = x
    for i in range(4):
        t = m.dense(t, 2048, name=f"fc{i}")
        t = m.relu(t, name=f"r{i}")
    m.softmax(m.dense(t, 16, name="out"))
    return m.cg


def test_unity_rewrites_beat_mcmc_alone():
    """Separate Linear / ReLU layers: MCMC (per-layer parallel configs)
    cannot remove a ReLU pass; Unity's rewrites (the fusion rules and the
    corpus rules that fuse under parallel operators) can."""
    cg = _relu_chain()
    cm = native.cost_model()
    # pipeline candidates off: this checks the rewrites (a 2-stage split of
    # this sync-bound chain would win on its own)
    cfg = {"world": 2, "budget": 12, "time_limit": 60, "seed": 3, "substitution_path": BUNDLED, "pipeline": False}
    _, mrep, _ = C.mcmc_search(cg, cm, json.dumps(cfg))
    pcg, rep, _ = C.graph_optimize(cg, cm, json.dumps(cfg))
    mrep, rep = json.loads(mrep), json.loads(rep)
    assert rep["algorithm"] == "mcmc+unity"
    assert rep["cost"] < mrep["cost"] * 0.999
    assert rep["rule_set_rules"] >= 595 and rep["rules"] > rep["rule_set_rules"]
    assert rep["best_rules"], rep
    pcg.reinfer_shapes()
    # one device: nothing to parallelize, so the only gains are the fusions
    cfg["world"] = 1
    pcg1, rep1, _ = C.graph_optimize(cg, cm, json.dumps(cfg))
    rep1 = json.loads(rep1)
    assert rep1["cost"] < rep1["data_parallel_cost"] * 0.999
    assert _ops(pcg1)["RELU"] == 0 and len(rep1["best_rules"]) == 4, rep1["best_rules"]


def test_unity_budget_is_the_reference_budget():
    """graph_optimize gives Unity --budget best-first pops (not budget/50)."""
    cg = _relu_chain()
    cm = native.cost_model()
    cfg = {"world": 2, "budget": 6, "time_limit": 120, "seed": 3, "substitution_path": "none_here"}
    cfg.pop("substitution_path")
    d = C.data_parallel_pcg(cg, 2)
    _, rep, _ = C.unity_search(d, cm, json.dumps(cfg))
    assert json.loads(rep)["iterations"] == 6


def test_ffconfig_substitution_path():
    cfg = FFConfig()
    assert unity.substitution_path(cfg) == BUNDLED
    cfg.substitution_json_path = "none"
    assert unity.substitution_path(cfg) == ""
    cfg.substitution_json_path = "/nonexistent/rules.json"
    with pytest.raises(FileNotFoundError):
        unity.substitution_path(cfg)


def test_two_linears_sharing_an_input_match_both_ways():
    """lib/substitutions/test/src/substitutions/pcg_pattern.cc: a pattern of
    two LINEAR nodes reading the same pattern input, on a graph where a feeds
    x_matmul and y_matmul (then add), matches exactly twice, with the two
    pattern nodes swapped, both binding the pattern input to a's value."""
    import json as _json
    m = FFModel(FFConfig())
    a = m.create_tensor([16, 24], DataType.DT_FLOAT, name="a")
    t0 = m.dense(a, 16, use_bias=False, name="x_matmul")
    t1 = m.dense(a, 16, use_bias=False, name="y_matmul")
    m.add(t0, t1, name="add")
    pcg = C.data_parallel_pcg(m.cg, 2)
    lin = {"attrs": {}, "constraints": [], "inputs": [[-1, 0]], "num_outputs": -1, "type": "LINEAR"}
    sub = C.substitution_from_json(_json.dumps({
        "format": "ffmi355x.substitution.v1", "name": "two_linears", "num_pattern_inputs": 1,
        "pattern": [lin, lin], "pattern_outputs": [[0, 0], [1, 0]], "output_graph": [], "output_mapping": []}))
    matches = C.find_pattern_matches(sub, pcg)
    got = sorted(tuple(pcg.layer_name(n) for n in nm) for nm, _ in matches)
    assert got == [("x_matmul", "y_matmul"), ("y_matmul", "x_matmul")]
    feeds = {(v.node, v.idx) for _, im in matches for v in im}
    assert len(feeds) == 1   # the one value that feeds both matmuls
    (node, idx), = feeds
    x = pcg.find_layer("x_matmul") if hasattr(pcg, "find_layer") else None
    if x is not None:
        assert any((v.node, v.idx) == (node, idx) for v in pcg.layer_inputs(x))
