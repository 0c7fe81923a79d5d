"""bench.py's launch contract (the driver's multi-GPU scaling run):
``python bench.py --gpus N`` without a launcher starts N ranks itself, and a
run whose process group does not have N members fails instead of reporting
a 1-GPU number as an N-GPU one.  CPU tier: 2 gloo ranks, tiny BERT."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ARGS = ["--model", "bert-base", "--layers", "2", "--steps", "2", "--warmup", "1", "--batch-per-gpu", "2",
        "--seq", "64", "--no-dp-compare"]


def _env(**over):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "FF_DIST_WORLD1"):
        env.pop(k, None)
    env.update(over)
    env["CUDA_VISIBLE_DEVICES"] = ""
    env["OMP_NUM_THREADS"] = "2"
    return env


def test_bench_self_launches_n_ranks():
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"] + ARGS, env=_env(),
                       capture_output=True, text=True, timeout=600, cwd="/tmp")
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [json.loads(ln) for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout            # rank 0 only
    r = lines[0]
    assert r["n_gpus"] == 2 and r["world_size"] == 2 and r["backend"] == "gloo"
    assert r["config"]["global_batch"] == 4 and r["steps"] == 2 and r["warmup"] == 1


def test_bench_refuses_world_mismatch():
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"] + ARGS,
                       env=_env(WORLD_SIZE="1", RANK="0"), capture_output=True, text=True, timeout=300, cwd="/tmp")
    assert p.returncode != 0
    assert "WORLD_SIZE=1" in p.stderr
    assert not [ln for ln in p.stdout.splitlines() if ln.startswith("{")]


def test_bench_multi_rank_emits_comm_calibration_and_ae():
    """N > 1: the JSON line carries the measured collectives at the step's
    message sizes against the cost model before / after calibration, the
    simulator's predicted step beside the measured one, and (--ae) the
    OSDI'22 AE BERT protocol's searched-vs-DP ratio."""
    args = ["--model", "bert-base", "--layers", "2", "--steps", "2", "--warmup", "1", "--batch-per-gpu", "2",
            "--seq", "64", "--no-dp-compare", "--ae"]
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"] + args, env=_env(),
                       capture_output=True, text=True, timeout=900, cwd="/tmp")
    assert p.returncode == 0, p.stderr[-3000:]
    r = [json.loads(ln) for ln in p.stdout.splitlines() if ln.startswith("{")][0]
    cal = r["config"]["comm_calibration"]
    assert "error" not in cal, cal
    assert cal["comm"] and {"measured_ms", "simulated_ms", "calibrated_ms"} <= set(cal["comm"][0])
    assert cal["sizes_used"]["all_reduce"]
    assert cal["predicted_ms_calibrated"] > 0 and cal["measured_ms"] == r["ms_per_step"]
    ae = r["config"]["ae_bert"]
    assert "error" not in ae, ae
    assert ae["global_batch"] == 8 and ae["layers"] == 12
    assert ae["searched_samples_per_sec"] > 0 and ae["dp_samples_per_sec"] > 0 and ae["speedup_over_dp"] > 0
