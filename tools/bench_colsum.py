#!/usr/bin/env python3
"""Bandwidth of the bias-gradient column sum (colsum_act, elementwise.hip) and
the embedding backward (embedding.hip) at BERT-large shapes (16384 tokens)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from flexflow_train_amd import kernels as K  # noqa: E402
from tools.bench_kernels import timeit  # noqa: E402


def main():
    M = 16384
    for N, act in [(1024, "none"), (3072, "none"), (4096, "gelu"), (30528, "none")]:
        dy = torch.randn(M, N, device="cuda").to(torch.bfloat16)
        pre = torch.randn_like(dy) if act != "none" else None
        db = torch.zeros(N, device="cuda")
        wdx = act != "none"
        t = timeit(lambda: K.colsum_act(dy, pre, act, dbias=db, write_dx=wdx))
        nb = dy.numel() * 2 * (3 if wdx else 1)
        db.zero_()
        K.colsum_act(dy, pre, act, dbias=db, write_dx=wdx)
        if pre is None:
            ref = dy.float().sum(0)
        else:
            u = pre.float().requires_grad_(True)
            torch.nn.functional.gelu(u, approximate="tanh").backward(dy.float())
            ref = u.grad.sum(0)
        err = (db - ref).abs().max().item() / (ref.abs().max().item() + 1e-6)
        print(json.dumps({"bench": "colsum_act", "M": M, "N": N, "act": act, "ms": round(t, 4),
                          "GBps": round(nb / t / 1e6, 1), "rel_err": err}), flush=True)
    for n, D in [(30522, 1024), (512, 1024), (2, 1024)]:
        idx = torch.randint(0, n, (M,), device="cuda")
        dout = torch.randn(M, D, device="cuda").to(torch.bfloat16)
        dw = torch.zeros(n, D, device="cuda")
        t = timeit(lambda: K.embedding_bwd(idx, dout, dw))
        dw.zero_()
        K.embedding_bwd(idx, dout, dw)
        ref = torch.zeros(n, D, device="cuda").index_add_(0, idx, dout.float())
        err = (dw - ref).abs().max().item() / (ref.abs().max().item() + 1e-6)
        print(json.dumps({"bench": "embedding_bwd", "rows": M, "entries": n, "D": D, "ms": round(t, 4),
                          "GBps": round(dout.numel() * 2 / t / 1e6, 1), "rel_err": err}), flush=True)


if __name__ == "__main__":
    main()
