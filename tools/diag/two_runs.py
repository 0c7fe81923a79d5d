"""Diagnostic: two bench runs in one process (``ORDER=dp,dp`` or
``search,dp``), per-run ms/step and per-step times (FF_STEP_TIMES=1):
whether a second run in the same process is slower, and after which first
run.  Launch under torch.distributed.run like bench.py."""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench  # noqa: E402

order = os.environ.get("ORDER", "dp,dp").split(",")
args = argparse.Namespace(batch_per_gpu=int(os.environ.get("BPG", "64")), model=os.environ.get("MODEL", "bert-large"),
                          seq=512, layers=int(os.environ.get("LAYERS", "0")), profile=False, dtype="bf16", budget=0,
                          graph=-1, steps=3, warmup=1, strategy="search")
world, rank = int(os.environ["WORLD_SIZE"]), int(os.environ["RANK"])
for i, s in enumerate(order):
    t = time.time()
    res = bench._run_bert(args, world, rank, only_dp=(s == "dp"))
    if rank == 0:
        print(f"run {i} {s}: {res['value']:.2f} samples/s {res['ms']:.1f} ms/step {res['config']['parallelism'][:50]} "
              f"({time.time() - t:.1f} s)", file=sys.stderr, flush=True)
    bench._release(res)
