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
        "--seq", "64", "--no-dp-compare", "--no-ae"]


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
            "--seq", "64", "--no-dp-compare"]
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
    assert ae["isolated"]          # searched / DP runs as fresh child jobs started by rank 0
    assert ae["searched_samples_per_sec"] > 0 and ae["dp_samples_per_sec"] > 0 and ae["speedup_over_dp"] > 0


def test_bench_eight_ranks_reports_measured_speedups():
    """The driver's 8-GPU line, rehearsed on 8 gloo ranks: the AE protocol runs
    by default at N > 1 (no --ae), and the line carries the measured
    searched-vs-DP ratios (headline and AE config), the collectives'
    calibration and what the search did."""
    args = ["--model", "bert-base", "--layers", "2", "--steps", "2", "--warmup", "1", "--batch-per-gpu", "2",
            "--seq", "64"]
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8"] + args,
                       env=_env(OMP_NUM_THREADS="1"), capture_output=True, text=True, timeout=1500, cwd="/tmp")
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [json.loads(ln) for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    r = lines[0]
    assert r["n_gpus"] == 8 and r["world_size"] == 8
    c = r["config"]
    assert "error" not in c["comm_calibration"], c["comm_calibration"]
    s = c["search"]
    assert s["evaluated"] > 0 and s["s"] > 0 and "time_limited" in s and "mapping_won" in s
    # the headline ratio is measured whenever the search left data parallelism
    if not c["parallelism"].startswith("dp"):
        assert c["dp_samples_per_sec"] > 0 and c["dp_reference"].startswith("measured")
    ae = c["ae_bert"]
    assert "error" not in ae and "skipped" not in ae, ae
    assert ae["searched_samples_per_sec"] > 0 and ae["dp_samples_per_sec"] > 0
    assert c["ae_speedup_over_dp"] == ae["speedup_over_dp"] > 0


def test_bench_deadline_keeps_the_headline():
    """Work after the headline (the DP reference / AE protocol) still running
    at --deadline-s is abandoned: rank 0 prints the line with what finished
    and every rank exits 0 (a hang there never costs the measured number)."""
    args = ["--model", "bert-base", "--layers", "2", "--steps", "2", "--warmup", "1", "--batch-per-gpu", "2",
            "--seq", "64", "--no-calibrate", "--deadline-s", "1"]
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"] + args, env=_env(),
                       capture_output=True, text=True, timeout=900, cwd="/tmp")
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [json.loads(ln) for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    c = lines[0]["config"]
    assert lines[0]["value"] > 0 and "deadline" in c["after_headline"]
    assert "error" in c["ae_bert"]
