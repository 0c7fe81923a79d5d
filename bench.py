#!/usr/bin/env python3
"""Headline benchmark: BERT-large training throughput (samples/s, whole node).

    python bench.py --gpus N --steps K --warmup W
    torchrun --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

With --gpus N > 1 and no launcher environment (no WORLD_SIZE), bench.py is its
own launcher: the parent process -- which never touches HIP -- starts N
ranks through torch.distributed.run on 127.0.0.1 and exits with their status.
Every rank then checks that the process group really has N members (and is
RCCL, backend "nccl", on a GPU) and exits non-zero otherwise, so an N-GPU
number can never silently be a 1-GPU one.

Metric / config from BASELINE.json: "samples/sec (whole node) + speedup-over-
DP after search, BERT-large 8xMI355X".  The model is BERT-large (24 layers,
hidden 1024, 16 heads, FFN 4096, seq 512, vocab 30522 padded to 30528) with
a full MLM head, bf16 compute / fp32 master weights + Adam, random-init
weights and synthetic token ids (no datasets on this pool).  The per-GPU
batch is fixed (weak scaling); the strategy comes from the framework's
compile() (searched, or --strategy dp for the data-parallel baseline).
Each timed step = forward + loss + backward + gradient all-reduce + Adam
update over all parameters.  Rank 0 prints ONE JSON line.

Speedup over data parallelism (the reference's Unity-vs-DP protocol,
scripts/osdi22ae/*.sh): with N > 1 and the searched strategy, the line
carries ``speedup_over_dp`` — 1.0 when the search itself chose pure data
parallelism, else the searched samples/s over a data-parallel run of the
same model and batch measured right after (same K / W, outside the headline
timed region) — plus the search's simulated prediction.

Other BASELINE.json configs run through the same contract with --model:
  resnet50     ResNet-50, synthetic 224x224 ImageNet batches (1000 classes),
               per-GPU batch 256, SGD momentum 0.9
  dlrm         DLRM (8 tables x 1M rows, sparse 64, bot 64-512-512-64,
               top 576-1024-1024-1024-1), per-GPU batch 1024, plain SGD lr 0.01
               (the reference's dlrm.cc:171; row-sparse table update)
  gpt3-medium  GPT-3 medium (24 layers, hidden 1024, 16 heads, seq 2048,
               vocab 50257), per-GPU batch 16, AdamW
"""
import argparse
import collections
import gc
import json
import os
import signal
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
if os.environ.get("FF_PKG_ROOT"):  # same-box A/B against a snapshot of the package (profiles/scripts/*.sh)
    sys.path.insert(0, os.path.abspath(os.environ["FF_PKG_ROOT"]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch-per-gpu", type=int, default=0, help="default: 128 (BERT), 512 (ResNet-50), 1024 (DLRM), "
                                                                   "32 (GPT-3 medium) -- 64 / 256 / 16 before round 6; sized "
                                                                   "for 288 GB of HBM per GPU (profiles/r6/g40_*, "
                                                                   "profiles/batch_sweep_r3.txt)")
    ap.add_argument("--seq", type=int, default=512)
    ap.add_argument("--model", default="bert-large",
                    choices=["bert-large", "bert-base", "resnet50", "resnext50", "inception-v3", "dlrm",
                             "gpt3-medium"])
    ap.add_argument("--no-calibrate", action="store_true",
                    help="N > 1: skip timing the step's RCCL collectives (cost-model calibration, outside the "
                         "timed region)")
    ap.add_argument("--ae", action="store_true",
                    help="(default at N > 1 for BERT) also run the reference's OSDI'22 AE BERT protocol "
                         "(scripts/osdi22ae/bert.sh: 12 layers, hidden 1024, 16 heads, seq 512, global batch 8, "
                         "--budget 30) searched vs data parallel, reported as config.ae_bert (outside the headline "
                         "timed region)")
    ap.add_argument("--no-ae", action="store_true", help="skip the AE protocol at N > 1")
    ap.add_argument("--ae-deadline-s", type=float, default=float(os.environ.get("FF_AE_DEADLINE_S", "300")),
                    help="start the AE protocol only if the run so far took less than this many seconds (keeps the "
                         "whole command inside the driver's bench timeout)")
    ap.add_argument("--deadline-s", type=float, default=float(os.environ.get("FF_BENCH_DEADLINE_S", "540")),
                    help="N > 1: wall-clock budget of the whole command; work after the headline still running at "
                         "this point is abandoned, the line printed with what finished")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "float32"],
                    help="compute dtype (float32: the exact-fp32 MFMA kernels; the headline metric is bf16)")
    ap.add_argument("--layers", type=int, default=None, help="override (debug only; invalidates the metric)")
    ap.add_argument("--strategy", default="search", choices=["search", "dp"])
    ap.add_argument("--no-dp-compare", action="store_true",
                    help="skip the data-parallel reference run behind speedup_over_dp")
    ap.add_argument("--budget", type=int, default=0,
                    help="strategy-search budget (MCMC / Unity iterations); default: BERT / GPT the reference's "
                         "OSDI'22 AE value (scripts/osdi22ae/bert.sh --budget 30), the others 400")
    ap.add_argument("--gemm", default=os.environ.get("FF_GEMM", "auto"))
    ap.add_argument("--profile", action="store_true")
    ap.add_argument("--graph", type=int, default=-1,
                    help="replay the training step from a hipGraph (1) or run eagerly (0); default 1: one graph "
                         "on a single GPU, graph segments cut at every RCCL collective across ranks")
    args = ap.parse_args()

    os.environ["FF_GEMM"] = args.gemm
    t_start = time.time()
    if os.environ.get("FF_HANG_DUMP_S"):
        # diagnostic: every thread's Python stack to stderr every N seconds
        import faulthandler
        faulthandler.dump_traceback_later(float(os.environ["FF_HANG_DUMP_S"]), repeat=True)
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(_self_launch(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world != args.gpus:
        print(f"error: --gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks", file=sys.stderr)
        sys.exit(2)
    runner = _run_bert if args.model in ("bert-large", "bert-base") else _run_zoo

    res = runner(args, world, rank, only_dp=args.strategy == "dp")
    dist_world, backend = _check_world(res["ex"], args.gpus)
    # FF_BENCH_REHEARSE_MULTI=1 (with FF_DIST_WORLD1=1: RCCL at world 1) runs
    # the multi-rank flow after the headline -- calibration, the watchdog,
    # the DP reference and the AE protocol -- on one GPU
    multi = world > 1 or os.environ.get("FF_BENCH_REHEARSE_MULTI") == "1"
    if multi and not args.no_calibrate:
        # after the timed steps: the collectives the step issued, timed at its
        # own message sizes on this process group, fitted into the cost model;
        # the simulator's step prediction before / after against the measured
        # step (lib/runtime/src/simulator.cc:1087-1215, 1684-1795 modelled
        # these links from a config file)
        from flexflow_train_amd.parallel import calibrate
        try:
            cal = calibrate.calibrate_for_step(res["ex"])
            res["config"]["comm_calibration"] = calibrate.summary(cal, res["model"].pcg, res["model"].views, world,
                                                                  res["ms"], res["model"].ffconfig)
        except Exception as e:  # noqa: BLE001 -- never costs the headline
            res["config"]["comm_calibration"] = {"error": f"{type(e).__name__}: {e}"[:300]}
    # everything after the headline (the DP reference run, the AE protocol)
    # runs under a watchdog: if it is still going at the deadline -- a slow
    # search, or a hang in a strategy never run at this scale -- rank 0
    # prints the line with what finished and every rank exits 0, so the
    # headline measured above is never lost to the driver's timeout
    extra = {"speed": {}, "ae": None}
    emitted = threading.Lock()

    def emit(note=None):
        if not emitted.acquire(blocking=False):
            return
        if rank != 0:
            return
        conf = res["config"]
        conf.update(extra["speed"])
        ae = extra["ae"]
        if note:
            conf["after_headline"] = note
        if ae is not None and ae.get("speedup_over_dp") is not None:
            # the measured searched-vs-DP ratio of the reference's AE protocol
            # (the headline's 64 sequences per GPU leave the search nothing to
            # win over DP; at 1 sequence per GPU it picks tensor / head splits)
            conf["ae_speedup_over_dp"] = ae["speedup_over_dp"]
        if ae is not None:
            conf["ae_bert"] = ae
        print(json.dumps({"metric": "samples_per_sec_whole_node", "value": round(res["value"], 2),
                          "unit": "samples/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                          "ms_per_step": round(res["ms"], 3), "higher_is_better": True, "scaling": "weak",
                          "vs_baseline": None, "dtype": args.dtype, "data": res["data"], "config": conf,
                          "world_size": dist_world, "backend": backend}), flush=True)

    done = threading.Event()
    if multi:
        left = args.deadline_s - (time.time() - t_start)

        def watchdog():
            if done.wait(max(1.0, left)):
                return
            child = extra.get("child")
            if child is not None and child.poll() is None:
                try:   # the AE protocol's child ranks go with this process
                    os.killpg(child.pid, signal.SIGKILL)
                except OSError:
                    pass
            if extra["ae"] is None and not args.no_ae and args.model in ("bert-large", "bert-base"):
                extra["ae"] = {"error": f"not finished within the {args.deadline_s:.0f} s command deadline"}
            emit(note=f"stopped at the {args.deadline_s:.0f} s deadline")
            sys.stdout.flush()
            sys.stderr.flush()
            os._exit(0)
        threading.Thread(target=watchdog, daemon=True).start()

    inproc = os.environ.get("FF_AE_INPROCESS") == "1"
    want_ae = multi and not args.no_ae and args.model in ("bert-large", "bert-base")
    want_dp = False
    if multi and args.strategy == "search":
        speed = extra["speed"]
        pred = res["search"].get("predicted_speedup_over_dp")
        if pred is not None:
            speed["predicted_speedup_over_dp"] = round(float(pred), 3)
        if res["config"]["parallelism"].startswith("dp") and world > 1:
            speed["speedup_over_dp"] = 1.0
            kept = res["search"].get("kept_data_parallel")
            speed["dp_reference"] = ("the searched strategy is data parallel"
                                     + (f" (kept: {kept})" if kept else ""))
        else:
            want_dp = not args.no_dp_compare
    if inproc:
        # the reference runs in this process, every rank taking part
        if want_dp:
            speed = extra["speed"]
            sps = res["value"]
            try:
                _release(res)
                dp = runner(args, world, rank, only_dp=True)
                speed["dp_samples_per_sec"] = round(dp["value"], 2)
                speed["speedup_over_dp"] = round(sps / dp["value"], 3)
                speed["dp_reference"] = "measured: data-parallel run of the same model / batch after the timed run"
                _release(dp)
            except Exception as e:  # noqa: BLE001 -- reported, never costs the headline line
                speed["dp_reference"] = {"error": f"{type(e).__name__}: {e}"[:300]}
        if want_ae:
            # every rank decides from rank 0's clock, so all of them take the same branch
            spent = _max_over_ranks(res, time.time() - t_start)
            if spent < args.ae_deadline_s:
                extra["ae"] = _run_ae(args, world, rank, res)
            else:
                extra["ae"] = {"skipped": f"run took {spent:.0f} s before the protocol "
                                          f"(deadline {args.ae_deadline_s:.0f} s)"}
    elif want_dp or want_ae:
        # the DP reference and the AE protocol as fresh jobs started by rank 0
        # (_child_bench); the other ranks release their model and wait on the
        # rendezvous store -- no collective pending on the GPUs (an RCCL kernel
        # waiting in a collective would share the GPUs with the children)
        _release(res)
        if rank == 0:
            try:
                if want_dp:
                    speed = extra["speed"]
                    try:
                        left = args.deadline_s - (time.time() - t_start) - 30.0
                        speed.update(_dp_reference_isolated(args, world, rank, res, extra, left))
                        speed["speedup_over_dp"] = round(res["value"] / speed["dp_samples_per_sec"], 3)
                    except Exception as e:  # noqa: BLE001 -- reported, never costs the headline line
                        speed["dp_reference"] = {"error": f"{type(e).__name__}: {e}"[:300]}
                if want_ae:
                    spent = time.time() - t_start
                    if spent < args.ae_deadline_s:
                        extra["ae"] = _run_ae_isolated(args, world, rank, res, extra, args.ae_deadline_s - spent)
                    else:
                        extra["ae"] = {"skipped": f"run took {spent:.0f} s before the protocol "
                                                  f"(deadline {args.ae_deadline_s:.0f} s)"}
            finally:
                _post_done(world, rank, signal_done=True)
        else:
            _post_done(world, rank, signal_done=False, timeout_s=args.deadline_s)
    done.set()
    emit()
    if rank == 0:
        if os.environ.get("FF_GEMM_REPORT"):
            from flexflow_train_amd.ops.dense import dact_report
            from flexflow_train_amd.ops.gemm import report
            print(report(), file=sys.stderr)
            print(dact_report(), file=sys.stderr)
        if args.profile and res.get("profile"):
            print(json.dumps({"profile_ms_total": res["profile"]}), file=sys.stderr)


def _self_launch(n: int) -> int:
    """Parent of an N-rank run started without a launcher: one rank per GPU
    through torch.distributed.run (the same command the driver uses), as
    child processes -- this process imports no GPU library, so no HIP state
    exists here that a child could inherit."""
    import socket
    import subprocess
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "1")
    return subprocess.call(cmd, env=env)


def _max_over_ranks(res, v: float) -> float:
    """max of v over the ranks (the executor's process group; the DP run may
    have released res["ex"])."""
    import torch
    import torch.distributed as dist
    if not dist.is_initialized():
        return v
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else torch.device("cpu")
    t = torch.tensor([v], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def _check_world(ex, want: int):
    """(world size, backend) of the process group the step ran on; exits
    non-zero when it is not ``want`` ranks, or not RCCL on a GPU."""
    world = ex.dist.world
    backend = ex.dist.backend
    if want > 1:
        import torch.distributed as dist
        ok = dist.is_initialized() and dist.get_world_size() == want
        # FF_BENCH_REHEARSAL=1: gloo ranks sharing one GPU (the multi-rank
        # code path rehearsed on a 1-GPU box); the JSON line says so
        if ok and ex.cfg.device.type == "cuda" and backend != "nccl" and os.environ.get("FF_BENCH_REHEARSAL") != "1":
            ok = False
        if not ok:
            print(f"error: expected a {want}-rank process group (RCCL on GPU), got world={world} "
                  f"backend={backend}", file=sys.stderr)
            sys.exit(3)
    return world, backend


def _release(res):
    """Drop a finished run's model, executor and captured graphs before the
    next one (the DP reference) allocates its own."""
    import torch
    for k in ("model", "ex", "step", "feeds", "labels"):
        res.pop(k, None)
    gc.collect()
    if torch.cuda.is_available():
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
        if os.environ.get("FF_MEM_PHASES") == "1":
            print(f"[mem] released: allocated {torch.cuda.memory_allocated() / 1e9:.2f} GB, "
                  f"reserved {torch.cuda.memory_reserved() / 1e9:.2f} GB", file=sys.stderr, flush=True)


def _memory_record(model, ex, world, bytes_per_param=16.0):
    """This rank's liveness memory plan of the step (csrc/ffcore/src/
    memory_plan.cc) next to the allocator's measured peak, GB."""
    import torch
    try:
        from flexflow_train_amd.search import native
        bf16 = getattr(ex.cfg, "compute_dtype", None) == torch.bfloat16
        plans = native.plan_memory(model.pcg, world, model.views, weight_bytes_per_param=bytes_per_param,
                                   act_elem_bytes=2.0 if bf16 else 0.0, executor_fusions=True)
        p = plans[min(ex.dist.rank, len(plans) - 1)]
        rec = {"planned_arena_gb": round(p["arena_bytes"] / 1e9, 2),
               "planned_peak_live_gb": round(p["peak_live_bytes"] / 1e9, 2),
               "per_op_sum_gb": round(p["naive_bytes"] / 1e9, 2)}
    except Exception as e:  # noqa: BLE001 -- the record must not cost the run
        rec = {"plan_error": f"{type(e).__name__}: {e}"[:160]}
    if ex.cfg.device.type == "cuda":
        # whole run (includes the GEMM autotuner's candidate outputs in step 1)
        rec["measured_peak_gb"] = round(torch.cuda.max_memory_allocated(ex.cfg.device) / 1e9, 2)
        if getattr(ex, "_ff_step_peak", None) is not None:
            # one steady-state eager step after the autotuner settled: what
            # the step itself holds at its peak (the plan's subject)
            rec["measured_step_peak_gb"] = round(ex._ff_step_peak / 1e9, 2)
            planned = rec.get("planned_arena_gb")
            if planned:
                rec["plan_error_pct"] = round(100.0 * (planned - rec["measured_step_peak_gb"])
                                              / rec["measured_step_peak_gb"], 1)
        if getattr(ex, "arena", None) is not None:
            rec["device_arena"] = ex.arena.stats()
    return rec


def _search_record(model, world):
    """What the strategy search did: wall time, states / strategies priced,
    iterations against the budget, whether it ended on its time limit, and
    whether the machine mapping (per-op device placement) won."""
    rep = dict(model.search_report or {})
    if world <= 1 or not rep:
        return None
    cfg = model.ffconfig
    limit = float(getattr(cfg, "search_time_limit", 45.0))
    out = {"s": round(float(rep.get("elapsed", 0.0)), 2), "algorithm": rep.get("algorithm"),
           "evaluated": rep.get("evaluated"), "iterations": rep.get("iterations"),
           "budget": int(cfg.search_budget or 0), "mapped_states": rep.get("mapped_states"),
           "mapping_won": bool(model.views) or "+mapping" in str(rep.get("algorithm", "")),
           "predicted_speedup_over_dp": rep.get("predicted_speedup_over_dp")}
    out["time_limited"] = out["s"] >= 0.98 * limit
    return out


def _arena_bytes(model, ex, world, bytes_per_param):
    """The step's device arena (runtime/arena.plan_bytes): the liveness plan's
    peak minus the resident weights / optimizer state, +15 % and 2 GiB."""
    import torch
    from flexflow_train_amd.runtime.arena import plan_bytes
    return plan_bytes(model.pcg, model.views, world, ex.dist.rank, bytes_per_param,
                      getattr(ex.cfg, "compute_dtype", None) == torch.bfloat16)


def _time_steps(args, ex, feeds, labels, global_batch, model=None, bytes_per_param=16.0):
    """W untimed warm-up steps, then EXACTLY K timed steps bracketed by a
    barrier + device synchronisation on both sides; max over ranks."""
    import torch

    dev = ex.cfg.device
    # the framework's device arena: on by default on one GPU (verified there);
    # FF_ARENA=1 / 0 forces it on / off at any N
    arena_on = os.environ.get("FF_ARENA", "1" if ex.dist.world == 1 else "0") == "1"
    if dev.type == "cuda" and model is not None and not args.profile and arena_on:
        # the step runs out of the framework's device arena, sized by the plan
        try:
            ex.enable_arena(_arena_bytes(model, ex, ex.dist.world, bytes_per_param))
        except Exception as e:  # noqa: BLE001 -- the torch allocator serves the step instead
            print(f"warning: device arena not enabled ({type(e).__name__}: {e})", file=sys.stderr)

    def step():
        ex.train_step(feeds, labels)

    def phase(tag):
        # FF_MEM_PHASES=1: allocated / reserved / arena after each set-up phase (stderr)
        if os.environ.get("FF_MEM_PHASES") == "1" and dev.type == "cuda":
            torch.cuda.synchronize()
            a = getattr(ex, "arena", None)
            print(f"[mem] {tag}: allocated {torch.cuda.memory_allocated(dev) / 1e9:.2f} GB, "
                  f"peak {torch.cuda.max_memory_allocated(dev) / 1e9:.2f} GB, "
                  f"reserved {torch.cuda.memory_reserved(dev) / 1e9:.2f} GB"
                  + (f", arena {a.stats()}" if a is not None else ""), file=sys.stderr, flush=True)

    phase("compiled")
    if dev.type == "cuda" and not args.profile:
        # the step's own memory peak: one eager step to settle the autotuner
        # and the workspaces, then one measured from a reset peak counter
        ex.train_step(feeds, labels)
        phase("eager step 1")
        torch.cuda.synchronize()
        torch.cuda.reset_peak_memory_stats(dev)
        ex.train_step(feeds, labels)
        torch.cuda.synchronize()
        ex._ff_step_peak = torch.cuda.max_memory_allocated(dev)
        phase("eager step 2")
    graphed = False
    use_graph = args.graph if args.graph >= 0 else 1
    if use_graph and dev.type == "cuda" and not args.profile:
        try:
            step = ex.make_graphed_train_step(feeds, labels)
            graphed = True
            phase("captured")
        except Exception as e:  # noqa: BLE001 — fall back to eager execution
            print(f"warning: hipGraph capture failed ({type(e).__name__}: {e}); running eagerly", file=sys.stderr)
    for _ in range(args.warmup):
        step()
    phase("warm-up done")
    if dev.type == "cuda":
        torch.cuda.synchronize()
    ex.dist.barrier()
    if dev.type == "cuda":
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    if os.environ.get("FF_STEP_TIMES") == "1":
        # per-step wall times (stderr), each step synchronised: a diagnostic
        # run, not the headline's timing
        for i in range(args.steps):
            ts = time.perf_counter()
            step()
            if dev.type == "cuda":
                torch.cuda.synchronize()
            print(f"[step] {i}: {1000 * (time.perf_counter() - ts):.1f} ms", file=sys.stderr, flush=True)
    else:
        for _ in range(args.steps):
            step()
    if dev.type == "cuda":
        torch.cuda.synchronize()
    ex.dist.barrier()
    if dev.type == "cuda":
        torch.cuda.synchronize()
    elapsed = ex.dist.max_scalar(time.perf_counter() - t0)
    return {"value": global_batch * args.steps / elapsed, "ms": elapsed / args.steps * 1000.0, "graphed": graphed,
            "step": step}


def _run_bert(args, world, rank, only_dp: bool):
    import torch

    from flexflow_train_amd.core import AdamOptimizer, FFConfig, FFModel, LossType, MetricsType
    from flexflow_train_amd.models.bert import bert_base, bert_large, build_bert
    from flexflow_train_amd.ops.gemm import choices as gemm_choices

    # 128 sequences per GPU (65536 tokens, a 63 GB step): with the step's
    # activations freed as the backward goes (round 6) twice the round-5 batch
    # fits in a quarter of the HBM, 4.5 % more samples/s than 64 on one box
    # and half the collective-to-compute ratio across ranks (profiles/r6/g40_*)
    bpg = args.batch_per_gpu or 128
    global_batch = bpg * world
    mk = bert_large if args.model == "bert-large" else bert_base
    kw = dict(batch_size=global_batch, sequence_length=args.seq)
    if args.layers:
        kw["num_encoder_layers"] = args.layers
    bcfg = mk(**kw)

    cfg = FFConfig()
    cfg.batch_size = global_batch
    cfg.print_freq = 0
    cfg.profiling = args.profile
    cfg.only_data_parallel = only_dp
    cfg.compute_dtype = "float32" if args.dtype == "float32" else "bfloat16"
    cfg.search_budget = args.budget or _AE_BUDGET["bert"]
    model = FFModel(cfg)
    build_bert(model, bcfg)
    t0 = time.time()
    model.compile(optimizer=AdamOptimizer(model, alpha=1e-4, weight_decay=0.01, decoupled=True),
                  loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY,
                  metrics=[MetricsType.METRICS_ACCURACY, MetricsType.METRICS_SPARSE_CATEGORICAL_CROSSENTROPY])
    compile_s = time.time() - t0
    ex = model.executor
    dev = ex.cfg.device

    # synthetic data: this rank's piece of every input, generated on device once
    g = torch.Generator(device=dev).manual_seed(1234 + rank)
    feeds = {}
    for name in ex.inputs:
        shp = ex.local_input_shape(name)
        if name == "input_ids":
            feeds[name] = torch.randint(0, bcfg.vocab_size, shp, generator=g, device=dev, dtype=torch.int32)
        elif name == "position_ids":
            feeds[name] = torch.arange(shp[-1], device=dev, dtype=torch.int32).expand(shp).contiguous()
        else:
            feeds[name] = torch.randint(0, bcfg.type_vocab_size, shp, generator=g, device=dev, dtype=torch.int32)
    lshape = ex._loss_layout().piece_shape[:-1]
    labels = torch.randint(0, bcfg.vocab_size, lshape, generator=g, device=dev, dtype=torch.int64)

    t = _time_steps(args, ex, feeds, labels, global_batch, model, 16.0)
    pm = ex.perf_metrics()
    conf = {
        "model": args.model + ("" if not args.layers else f"-{args.layers}L(debug)"),
        "global_batch": global_batch,
        "batch_per_gpu": bpg,
        "seq_len": args.seq,
        "parallelism": _parallelism(model, world),
        "strategy_source": model.search_report.get("source", ""),
        "layers": bcfg.num_encoder_layers,
        "hidden": bcfg.hidden_size,
        "heads": bcfg.num_heads,
        "vocab": bcfg.vocab_size,
        "optimizer": "adamw",
        "compile_s": round(compile_s, 2),
        "hipgraph": t["graphed"],
        "graph_segments": list(getattr(ex, "graph_segments", ())) or None,
        "native_replay": getattr(ex, "native_replay", None),
        "gemm_choices": dict(collections.Counter(gemm_choices().values())),
        "tokens_per_sec": round(t["value"] * args.seq, 1),
        "final_loss": round(pm.loss, 4),
        "memory": _memory_record(model, ex, world),
        "search": _search_record(model, world),
    }
    prof = None
    if args.profile:
        prof = {k: round(v, 3) for k, v in list(ex.profile_report().items())[:40]}
    return {"value": t["value"], "ms": t["ms"], "config": conf, "search": dict(model.search_report),
            "data": "synthetic token ids, random-init weights", "model": model, "ex": ex, "step": t["step"],
            "profile": prof, "feeds": feeds, "labels": labels}


def _post_done(world: int, rank: int, signal_done: bool, timeout_s: float = 600.0):
    """Rank 0 tells the other ranks (through the rendezvous store, CPU only)
    that the post-headline jobs are done; they wait for it."""
    import datetime
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or world == 1:
        return
    store = dist.distributed_c10d._get_default_store()
    if signal_done:
        store.set("ff_bench_post_done", "1")
    else:
        store.set_timeout(datetime.timedelta(seconds=max(60.0, timeout_s)))
        store.wait(["ff_bench_post_done"])


def _child_env():
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "GROUP_RANK", "GROUP_WORLD_SIZE",
                        "ROLE_RANK", "ROLE_WORLD_SIZE", "ROLE_NAME", "MASTER_ADDR", "MASTER_PORT",
                        "FF_BENCH_REHEARSE_MULTI")
           and not k.startswith("TORCHELASTIC_")}
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return env


def _child_bench(world: int, bench_args, timeout_s: float, extra) -> dict:
    """One fresh N-rank bench job (torch.distributed.run, its own
    communicators) started by rank 0; its JSON line.  Killed with its process
    group at ``timeout_s`` (and by the watchdog at the command deadline)."""
    import socket
    import subprocess
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), "--gpus", str(world),
           "--no-ae", "--no-calibrate", "--no-dp-compare", "--deadline-s", str(max(10.0, timeout_s - 10.0))]
    cmd += [str(a) for a in bench_args]
    child = subprocess.Popen(cmd, env=_child_env(), stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                             start_new_session=True)
    extra["child"] = child
    t_end = time.time() + timeout_s
    try:
        while True:
            # a progress line every 30 s (stderr) while the child job runs;
            # communicate() may be retried after a timeout without losing output
            try:
                so, se = child.communicate(timeout=max(1.0, min(30.0, t_end - time.time())))
                break
            except subprocess.TimeoutExpired:
                if time.time() >= t_end:
                    os.killpg(child.pid, signal.SIGKILL)
                    child.communicate()
                    raise TimeoutError(f"did not finish within {timeout_s:.0f} s")
                print(f"[bench] child job {' '.join(str(a) for a in bench_args[-2:])} running, "
                      f"{t_end - time.time():.0f} s left", file=sys.stderr, flush=True)
    finally:
        extra["child"] = None
    logdir = os.environ.get("FF_BENCH_CHILD_LOG_DIR")
    if logdir:
        os.makedirs(logdir, exist_ok=True)
        tag = "_".join(str(a) for a in bench_args[-2:]).replace("/", "_")
        with open(os.path.join(logdir, f"child_{tag}_{int(time.time())}.err"), "w") as f:
            f.write(se)
    lines = [ln for ln in so.splitlines() if ln.startswith("{")]
    if child.returncode != 0 or not lines:
        raise RuntimeError(f"exited {child.returncode}: {se.strip()[-240:]}")
    return json.loads(lines[-1])


def _dp_reference_isolated(args, world, rank, res, extra, budget_s: float):
    """The data-parallel run of the headline's model / batch as a fresh job
    after this run released its memory (a second model built in the same
    process is not a clean reference: over gloo it ran ~10x slower, and a
    fault in it would cost the headline)."""
    _release(res)
    if rank != 0:
        return {}
    a = ["--model", args.model, "--seq", args.seq, "--dtype", args.dtype, "--steps", args.steps,
         "--warmup", args.warmup, "--strategy", "dp"]
    if args.layers:
        a += ["--layers", args.layers]
    if args.batch_per_gpu:
        a += ["--batch-per-gpu", args.batch_per_gpu]
    d = _child_bench(world, a, budget_s, extra)
    return {"dp_samples_per_sec": round(float(d["value"]), 2),
            "dp_reference": "measured: data-parallel run of the same model / batch as a fresh job after the timed run"}


def _run_ae_isolated(args, world, rank, res, extra, budget_s: float):
    """The AE protocol (see _run_ae) in child processes: rank 0 launches the
    searched and the data-parallel run of the AE configuration as two fresh
    N-rank jobs and reads their JSON lines, so a fault or an abort in a
    strategy never run at this scale costs only the protocol, never the
    headline measured above.  The other ranks release their model and
    finish; the watchdog kills the children's process group at the command
    deadline."""
    _release(res)
    out = {"layers": 12, "hidden": 1024 if args.model == "bert-large" else 768,
           "global_batch": max(1, 8 // world) * world, "seq_len": args.seq, "budget": 30,
           "protocol": "scripts/osdi22ae/bert.sh", "isolated": True}
    if rank != 0:
        return out
    t_end = time.time() + budget_s
    runs = {}
    try:
        for strat in ("search", "dp"):
            left = t_end - time.time()
            if left < 20:
                raise TimeoutError(f"{strat} run: {left:.0f} s left of the protocol's budget")
            runs[strat] = _child_bench(world, ["--model", args.model, "--layers", 12, "--seq", args.seq,
                                               "--batch-per-gpu", max(1, 8 // world), "--budget", 30,
                                               "--dtype", args.dtype, "--steps", min(args.steps, 10),
                                               "--warmup", min(args.warmup, 3), "--strategy", strat], left, extra)
        s, d = runs["search"], runs["dp"]
        out["searched_samples_per_sec"] = round(float(s["value"]), 2)
        out["parallelism"] = s["config"]["parallelism"]
        out["predicted_speedup_over_dp"] = (s["config"].get("search") or {}).get("predicted_speedup_over_dp")
        out["dp_samples_per_sec"] = round(float(d["value"]), 2)
        out["speedup_over_dp"] = round(out["searched_samples_per_sec"] / out["dp_samples_per_sec"], 3)
    except Exception as e:  # noqa: BLE001 -- reported, never costs the headline line
        out["error"] = f"{type(e).__name__}: {e}"[:300]
        if "search" in runs:
            out["searched_samples_per_sec"] = round(float(runs["search"]["value"]), 2)
    return out


def _run_ae(args, world, rank, res):
    """The OSDI'22 AE BERT protocol (scripts/osdi22ae/bert.sh:3-7): a 12-layer
    hidden-1024 BERT at global batch 8, the searched strategy (--budget 30)
    against --only-data-parallel, samples/s of each and their ratio.  At one
    sequence per GPU the search has something to win over DP (tensor / head
    parallelism), unlike the headline's 64 sequences per GPU."""
    import copy
    a = copy.copy(args)
    a.layers, a.batch_per_gpu = 12, max(1, 8 // world)
    a.budget = 30
    a.steps, a.warmup = min(args.steps, 10), min(args.warmup, 3)
    out = {"layers": 12, "hidden": 1024 if args.model == "bert-large" else 768, "global_batch": a.batch_per_gpu * world,
           "seq_len": args.seq, "budget": 30, "protocol": "scripts/osdi22ae/bert.sh"}
    _release(res)
    try:
        s = _run_bert(a, world, rank, only_dp=False)
        out["searched_samples_per_sec"] = round(s["value"], 2)
        out["parallelism"] = s["config"]["parallelism"]
        out["predicted_speedup_over_dp"] = s["search"].get("predicted_speedup_over_dp")
        _release(s)
        d = _run_bert(a, world, rank, only_dp=True)
        out["dp_samples_per_sec"] = round(d["value"], 2)
        _release(d)
        out["speedup_over_dp"] = round(out["searched_samples_per_sec"] / out["dp_samples_per_sec"], 3)
    except Exception as e:  # noqa: BLE001 -- reported, never costs the headline line
        out["error"] = f"{type(e).__name__}: {e}"[:300]
    return out


def _parallelism(model, world: int) -> str:
    """"dpN" when every operator is only batch-sharded (searched or not),
    else a summary of the non-DP degrees the search chose."""
    from flexflow_train_amd import _ffcore as C
    pcg = model.pcg
    other = set()
    for n in pcg.topo_order():
        op = pcg.layer_op(n)
        if op.op_type in ("INPUT", "WEIGHT") or pcg.is_weight_path(n) or C.is_parallel_op(op.type):
            continue
        ps = pcg.shape(C.ValueRef(n, 0))
        deg = list(ps.shard_degrees())
        if deg[1:] and max(deg[1:]) > 1 or ps.sum_degree > 1 or ps.discard_copy_degree > 1 or deg[0] != world:
            other.add(f"{op.op_type.lower()}:{'x'.join(map(str, deg))}/s{ps.sum_degree}/c{ps.discard_copy_degree}")
    src = model.search_report.get("source", "")
    if not other:
        return f"dp{world}"
    return f"hybrid({src}; " + ", ".join(sorted(other)[:6]) + ")"


# strategy-search budgets: the transformer configs use the reference's AE
# value (scripts/osdi22ae/bert.sh:3-7 --budget 30; their search settles on
# data parallelism at any budget, and 400 iterations cost ~50 s per run at 8
# GPUs); DLRM keeps 400 — with 20 iterations the search shards only one of
# the eight tables (predicted 1.13x vs 14.8x over DP at 8 GPUs)
_AE_BUDGET = {"bert": 30, "gpt": 30, "dlrm": 400, "resnet50": 400, "resnext50": 20, "inception_v3": 10}

_ZOO = {
    # bench name -> (zoo name, per-GPU batch, config overrides, optimizer, extra config for the JSON line);
    # ResNet-50 512 images (22 GB step) and GPT-3 medium 32 sequences (66 GB) per GPU since round 6: same
    # box, interleaved, +9 % and +3.4 % over 256 / 16 (profiles/r6/g42_batch_sweep.txt)
    "resnet50": ("resnet50", 512, dict(image_size=224, num_classes=1000), "sgd", {"image_size": 224}),
    # the reference's OSDI'22 AE CNNs (scripts/osdi22ae/resnext-50.sh, inception.sh)
    "resnext50": ("resnext50", 64, dict(image_size=224, num_classes=1000), "sgd", {"image_size": 224}),
    "inception-v3": ("inception_v3", 64, dict(image_size=299, num_classes=1000), "sgd", {"image_size": 299}),
    "dlrm": ("dlrm", 1024, dict(embedding_size=[1000000] * 8, sparse_feature_size=64, mlp_bot=[64, 512, 512, 64],
                                mlp_top=[576, 1024, 1024, 1024, 1]), "sgd", {"tables": "8x1M", "sparse": 64}),
    "gpt3-medium": ("gpt", 32, dict(hidden_size=1024, num_layers=24, num_heads=16, sequence_length=2048),
                    "adamw", {"seq_len": 2048, "layers": 24, "hidden": 1024}),
}


def _run_zoo(args, world, rank, only_dp: bool):
    """The other BASELINE configs: model-zoo network + synthetic data of its
    shape, same timing contract as the BERT path."""
    import dataclasses
    import numpy as np
    import torch

    from flexflow_train_amd import models as Z
    from flexflow_train_amd.core import (AdamOptimizer, FFConfig, FFModel, LossType, MetricsType, SGDOptimizer)

    zname, bpg, over, opt, extra = _ZOO[args.model]
    bpg = args.batch_per_gpu or bpg
    global_batch = bpg * world
    cfg = FFConfig()
    cfg.batch_size = global_batch
    cfg.print_freq = 0
    cfg.profiling = args.profile
    cfg.only_data_parallel = only_dp
    cfg.compute_dtype = "float32" if args.dtype == "float32" else "bfloat16"
    cfg.search_budget = args.budget or _AE_BUDGET.get(zname, 400)
    model = FFModel(cfg)
    inputs, out, mcfg = Z.build(zname, model, batch_size=global_batch, **over)
    ce = Z.loss_of(zname) == Z.LOSS_CE
    optimizer = (SGDOptimizer(model, lr=0.01, momentum=0.9 if zname in ("resnet50", "resnext50", "inception_v3")
                              else 0.0) if opt == "sgd"
                 else AdamOptimizer(model, alpha=1e-4, weight_decay=0.01, decoupled=True))
    t0 = time.time()
    model.compile(optimizer=optimizer,
                  loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY if ce
                  else LossType.LOSS_MEAN_SQUARED_ERROR_AVG_REDUCE,
                  metrics=[MetricsType.METRICS_ACCURACY] if ce else [MetricsType.METRICS_MEAN_SQUARED_ERROR])
    compile_s = time.time() - t0
    ex = model.executor

    # synthetic data of the model's shape, generated at this rank's batch
    first = next(iter(ex.inputs))
    lb = ex.local_input_shape(first)[0]
    rng = np.random.default_rng(1234 + rank)
    feeds_np, labels_np = Z.synthetic(zname, dataclasses.replace(mcfg, batch_size=lb), inputs, rng)
    try:
        feeds = {k: ex._local_piece(k, torch.as_tensor(v)) for k, v in feeds_np.items()}
        labels = ex.local_labels(torch.as_tensor(labels_np))
    except ValueError:  # inputs not batch-sharded under this strategy: global batch, then slice
        feeds_np, labels_np = Z.synthetic(zname, mcfg, inputs, np.random.default_rng(1234))
        feeds = {k: ex._local_piece(k, torch.as_tensor(v)) for k, v in feeds_np.items()}
        labels = ex.local_labels(torch.as_tensor(labels_np))
    del feeds_np, labels_np

    bpp = 16.0 if opt in ("adam", "adamw") else (14.0 if zname in ("resnet50", "resnext50", "inception_v3") else 10.0)
    t = _time_steps(args, ex, feeds, labels, global_batch, model, bpp)
    pm = ex.perf_metrics()
    conf = {"model": args.model, "global_batch": global_batch, "parallelism": _parallelism(model, world),
            "strategy_source": model.search_report.get("source", ""), "optimizer": opt,
            "compile_s": round(compile_s, 2), "hipgraph": t["graphed"],
            "graph_segments": list(getattr(ex, "graph_segments", ())) or None,
            "native_replay": getattr(ex, "native_replay", None), "final_loss": round(pm.loss, 4),
            # resident bytes per parameter: fp32 master + bf16 copy + gradient
            # + optimizer state (Adam m, v: 16; SGD momentum: 14; plain SGD: 10)
            "memory": _memory_record(model, ex, world, bpp),
            "search": _search_record(model, world)}
    conf.update(extra)
    if zname == "gpt":
        conf["tokens_per_sec"] = round(t["value"] * mcfg.sequence_length, 1)
    prof = None
    if args.profile:
        prof = {k: round(v, 3) for k, v in list(ex.profile_report().items())[:40]}
    return {"value": t["value"], "ms": t["ms"], "config": conf, "search": dict(model.search_report),
            "data": "synthetic inputs of the model's shape, random-init weights", "model": model, "ex": ex,
            "step": t["step"], "profile": prof, "feeds": feeds, "labels": labels}


def _write_autotune_report():
    """FF_AUTOTUNE_REPORT=<path>: the GEMM autotuner's per-shape candidate
    times and picks (ops/gemm.py report) written at exit, rank 0."""
    path = os.environ.get("FF_AUTOTUNE_REPORT")
    if not path or int(os.environ.get("RANK", "0")) != 0:
        return
    try:
        from flexflow_train_amd.ops import dense, gemm
        with open(path, "w") as f:
            f.write(gemm.report() + "\n" + dense.dact_report() + "\n")
    except Exception as e:  # noqa: BLE001
        print(f"autotune report: {e}", file=sys.stderr)


def _shutdown():
    """Leave the process group explicitly (every rank, after the line is
    out): left to interpreter teardown, the sub-groups of a searched hybrid
    strategy were destroyed with live worker threads and the ranks aborted
    on exit ("terminate called without an active exception", exit 1)."""
    try:
        import torch.distributed as dist
        if dist.is_available() and dist.is_initialized():
            dist.barrier()
            dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001 -- the measurement is already printed
        print(f"warning: process group shutdown: {type(e).__name__}: {e}", file=sys.stderr)


if __name__ == "__main__":
    import atexit
    atexit.register(_write_autotune_report)
    main()
    _shutdown()
