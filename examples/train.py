#!/usr/bin/env python3
"""Train any model-zoo entry with synthetic data (the reference's example
programs: examples/cpp/*, examples/python/native/*).

    python examples/train.py --model dlrm --steps 20
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 examples/train.py --model resnet50 \
        --batch-size 512 --strategy search --export-strategy /tmp/resnet.json

Flags after ``--`` go to FFConfig (reference flag set: -b, -e, --budget,
--alpha, --only-data-parallel, --import-strategy, --export-strategy,
--taskgraph, --profiling, ...).  Prints ``ELAPSED TIME`` / ``THROUGHPUT``
like the reference examples.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from flexflow_train_amd import models as Z  # noqa: E402
from flexflow_train_amd.core import (AdamOptimizer, FFConfig, FFModel, LossType, MetricsType,  # noqa: E402
                                     SGDOptimizer)


def main():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--model", required=True, choices=sorted(Z.MODELS))
    ap.add_argument("--config", default="{}", help="JSON overrides of the model config")
    ap.add_argument("--batch-size", type=int, default=0, help="global batch (default: model config)")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--strategy", default="dp", choices=["dp", "search", "mcmc"])
    ap.add_argument("--optimizer", default="sgd", choices=["sgd", "adam"])
    ap.add_argument("--lr", type=float, default=0.01)
    args, rest = ap.parse_known_args()

    ffcfg = FFConfig()
    ffcfg.parse_args([a for a in rest if a != "--"])
    ffcfg.only_data_parallel = args.strategy == "dp"
    if args.strategy == "mcmc":
        ffcfg.search_algorithm = "mcmc"
    kw = json.loads(args.config)
    if args.batch_size:
        kw["batch_size"] = args.batch_size
    model = FFModel(ffcfg)
    inputs, out, mcfg = Z.build(args.model, model, **kw)
    ce = Z.loss_of(args.model) == Z.LOSS_CE
    opt = SGDOptimizer(model, lr=args.lr) if args.optimizer == "sgd" else AdamOptimizer(model, alpha=args.lr)
    t0 = time.time()
    model.compile(optimizer=opt,
                  loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY if ce
                  else LossType.LOSS_MEAN_SQUARED_ERROR_AVG_REDUCE,
                  metrics=[MetricsType.METRICS_ACCURACY] if ce else [MetricsType.METRICS_MEAN_SQUARED_ERROR])
    ex = model.executor
    rank = ex.rank
    if rank == 0:
        print(f"compiled {args.model} in {time.time() - t0:.1f}s: strategy={model.search_report.get('source')}",
              flush=True)
    feeds, labels = Z.synthetic(args.model, mcfg, inputs, np.random.default_rng(1234))
    dev = ex.cfg.device
    feeds = {k: ex._local_piece(k, torch.as_tensor(v)) for k, v in feeds.items()}
    labels = ex.local_labels(torch.as_tensor(labels))
    for _ in range(args.warmup):
        ex.train_step(feeds, labels)
    if dev.type == "cuda":
        torch.cuda.synchronize()
    ex.dist.barrier()
    ex.zero_metrics()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        ex.train_step(feeds, labels)
    if dev.type == "cuda":
        torch.cuda.synchronize()
    ex.dist.barrier()
    el = ex.dist.max_scalar(time.perf_counter() - t0)
    gb = mcfg.batch_size
    if rank == 0:
        print(f"{ex.perf_metrics()}")
        print(f"ELAPSED TIME = {el:.4f}s, THROUGHPUT = {gb * args.steps / el:.2f} samples/s", flush=True)


if __name__ == "__main__":
    main()
