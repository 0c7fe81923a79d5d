"""Native CLIs (export-model-arch, substitution-to-dot, protobuf-to-json)
and the C++ model zoo (reference: bin/*, lib/models/test)."""
import json
import os
import subprocess

import pytest

from flexflow_train_amd import _ffcore as C

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "bin")
REF_SUBST = "/root/reference/substitutions"


@pytest.fixture(scope="module", autouse=True)
def _tools_built():
    if not all(os.path.exists(os.path.join(BIN, b)) for b in
               ("ffc-export-model-arch", "ffc-substitution-to-dot", "ffc-protobuf-to-json", "ffc-ffi-test",
                "ffc-runtime-c-test")):
        from tools.build_native import build

        build(["core", "tools", "ffi"])


def _run(*args):
    return subprocess.run([os.path.join(BIN, args[0])] + list(args[1:]), capture_output=True, text=True, check=True)


@pytest.mark.parametrize("model", ["transformer", "inception_v3", "candle_uno", "bert", "split_test",
                                   "single_operator", "gpt"])
def test_export_model_arch(model):
    r = _run("ffc-export-model-arch", model, "--sp-decomposition", "--config",
             '{"batch_size": 4, "num_encoder_layers": 2, "num_decoder_layers": 1}')
    d = json.loads(r.stdout)
    assert d["sp_decomposition"] is not None
    cg = C.ComputationGraph.from_json(json.dumps(d["computation_graph"]))
    assert cg.num_layers() > 2
    dot = _run("ffc-export-model-arch", model, "--dot").stdout
    assert dot.startswith("digraph")


def test_model_zoo_shapes():
    cg = C.get_model_computation_graph("bert", '{"batch_size": 2, "sequence_length": 16, "num_encoder_layers": 1}')
    out = [n for n in cg.topo_order() if cg.layer_op(n).op_type == "SOFTMAX"][0]
    assert list(cg.shape(C.ValueRef(out, 0)).dims) == [2, 16, 30522]
    inc = C.get_model_computation_graph("inception_v3", '{"batch_size": 2}')
    sm = [n for n in inc.topo_order() if inc.layer_op(n).op_type == "SOFTMAX"][0]
    assert list(inc.shape(C.ValueRef(sm, 0)).dims) == [2, 1000]
    cu = C.get_model_computation_graph("candle_uno", '{"batch_size": 2}')
    assert sum(1 for n in cu.topo_order() if cu.layer_op(n).op_type == "INPUT") == 7
    assert set(C.model_names()) >= {"transformer", "inception_v3", "candle_uno", "bert", "split_test"}


@pytest.mark.skipif(not os.path.exists(os.path.join(REF_SUBST, "graph_subst_3_v2.pb")), reason="no corpus")
def test_protobuf_to_json_matches_reference_json(tmp_path):
    out = str(tmp_path / "r.json")
    _run("ffc-protobuf-to-json", os.path.join(REF_SUBST, "graph_subst_3_v2.pb"), out)
    a = json.load(open(out))["rule"]
    b = json.load(open(os.path.join(REF_SUBST, "graph_subst_3_v2.json")))["rule"]
    assert a == b


@pytest.mark.skipif(not os.path.exists(os.path.join(REF_SUBST, "graph_subst_3_v2.json")), reason="no corpus")
def test_substitution_to_dot():
    path = os.path.join(REF_SUBST, "graph_subst_3_v2.json")
    dot = _run("ffc-substitution-to-dot", path, "taso_rule_7").stdout
    assert "cluster_src" in dot and "cluster_dst" in dot
    lst = _run("ffc-substitution-to-dot", path, "--list").stdout.strip().splitlines()
    assert len(lst) == 640


def test_c_runtime_api():
    """Legacy FFModel runtime C API (csrc/ffi/flexflow_runtime_c.h, the
    reference's python/flexflow_c.h surface): a C host builds an MLP and a
    conv/BN/pool CNN, trains them with SGD / Adam through data loaders and
    reads metrics, weights, gradients and raw pointers back."""
    r = _run("ffc-runtime-c-test")
    assert "PASSED (0 failures)" in r.stdout, r.stdout
    assert "FAIL " not in r.stdout


def test_runtime_c_header_covers_reference_names():
    """Every function the reference's python/flexflow_c.h declares for the
    surface this header implements exists here with the same name."""
    import re
    ref = "/root/reference/python/flexflow_c.h"
    if not os.path.exists(ref):
        pytest.skip("reference checkout not present")
    ours = open(os.path.join(os.path.dirname(BIN), "csrc", "ffi", "flexflow_runtime_c.h")).read()
    declared = set(re.findall(r"\b(flexflow_\w+|flowflow_\w+)\s*\(", ours))
    theirs = set(re.findall(r"\b(flexflow_\w+|flowflow_\w+)\s*\(", open(ref).read()))
    covered = theirs & declared
    assert len(declared) >= 140 and len(covered) >= 130, (len(declared), len(covered))


def test_c_ffi(tmp_path):
    """C ABI (csrc/ffi/flexflow_c.h): build, serialise, search, query from C."""
    r = _run("ffc-ffi-test", str(tmp_path / "cg.json"))
    assert "FFI OK" in r.stdout
    cg = C.ComputationGraph.from_json(open(tmp_path / "cg.json").read()) if hasattr(C.ComputationGraph, "from_json") \
        else None
    if cg is not None:
        assert len(list(cg.topo_order())) >= 5
