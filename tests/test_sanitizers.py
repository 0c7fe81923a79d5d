"""Host-code sanitizers over the C++ core (the reference has no
sanitizer anywhere; ASan + UBSan builds for host code are the recommended
race / memory-error net).  The core library, the C ABI and the native CLIs
are compiled with -fsanitize=address,undefined (tools/build_native.py asan ->
bin/asan/) and driven through the paths the normal suite exercises: model
zoo + SP decomposition + JSON / dot export, the legacy rule corpus (protobuf
decode + rule rendering), and the C ABI's build / serialise / search / query
cycle.  Any heap error, leak or undefined behaviour fails the test."""
import json
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ASAN = os.path.join(ROOT, "bin", "asan")
REF_SUBST = "/root/reference/substitutions"
TOOLS = ("ffc-export-model-arch", "ffc-substitution-to-dot", "ffc-protobuf-to-json", "ffc-ffi-test",
         "ffc-runtime-c-test")
ENV = dict(os.environ,
           ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:halt_on_error=1:exitcode=86",
           UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1:exitcode=87")


@pytest.fixture(scope="module", autouse=True)
def _asan_built():
    # pytest-xdist workers share build/: serialise the ninja run so one worker
    # never links while another is still rewriting the object files
    import fcntl

    os.makedirs(os.path.join(ROOT, "build"), exist_ok=True)
    with open(os.path.join(ROOT, "build", ".asan.lock"), "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        if not all(os.path.exists(os.path.join(ASAN, t)) for t in TOOLS):
            from tools.build_native import build

            build(["asan"])


def _run(*args, timeout=600):
    r = subprocess.run([os.path.join(ASAN, args[0])] + list(args[1:]), capture_output=True, text=True,
                       env=ENV, timeout=timeout)
    assert "ERROR: AddressSanitizer" not in r.stderr, r.stderr[-4000:]
    assert "ERROR: LeakSanitizer" not in r.stderr, r.stderr[-4000:]
    assert "runtime error:" not in r.stderr, r.stderr[-4000:]
    assert r.returncode == 0, (r.returncode, r.stderr[-4000:])
    return r


@pytest.mark.parametrize("model", ["transformer", "inception_v3", "candle_uno", "bert", "split_test",
                                   "single_operator", "gpt"])
def test_export_model_arch_under_sanitizers(model):
    r = _run("ffc-export-model-arch", model, "--sp-decomposition", "--config",
             '{"batch_size": 4, "num_encoder_layers": 2, "num_decoder_layers": 1}')
    assert json.loads(r.stdout)["sp_decomposition"] is not None
    assert _run("ffc-export-model-arch", model, "--dot").stdout.startswith("digraph")


def test_c_abi_search_cycle_under_sanitizers(tmp_path):
    """Build a graph through the C ABI, serialise / deserialise it, run the
    strategy search on an 8-GPU machine and query the result."""
    assert "FFI OK" in _run("ffc-ffi-test", str(tmp_path / "cg.json")).stdout


def test_c_runtime_api_under_sanitizers():
    """The legacy FFModel runtime C API: two models trained from C (host
    local execution of dense / conv / batch norm / pool), handles released."""
    assert "PASSED (0 failures)" in _run("ffc-runtime-c-test").stdout


@pytest.mark.skipif(not os.path.exists(os.path.join(REF_SUBST, "graph_subst_3_v2.pb")), reason="no corpus")
def test_rule_corpus_tools_under_sanitizers(tmp_path):
    out = str(tmp_path / "r.json")
    _run("ffc-protobuf-to-json", os.path.join(REF_SUBST, "graph_subst_3_v2.pb"), out)
    assert len(json.load(open(out))["rule"]) == 640
    path = os.path.join(REF_SUBST, "graph_subst_3_v2.json")
    assert "cluster_src" in _run("ffc-substitution-to-dot", path, "taso_rule_7").stdout
    assert len(_run("ffc-substitution-to-dot", path, "--list").stdout.strip().splitlines()) == 640
