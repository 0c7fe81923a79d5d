#!/usr/bin/env python3
"""Interleaved same-process A/B of the GEMM candidates on the transformer
training shapes (guide §5.4 rule 24): hipBLASLt (its heuristic's top pick,
through blaslt_gemm), gemmp (32x32x16 MFMA) and gemmq (gemmp's pipeline on
16x16x32 MFMA), each with the split-K counts the autotuner would try.
Random uniform [-1, 1) operands (rule 25).  Prints one JSON line per shape
with the median time of each candidate over R interleaved rounds and its
error against an fp32 reference.

    python tools/gemm_ab.py [--rounds 5] [--iters 10] [--only fwd,dx,dw]
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from flexflow_train_amd import kernels as K  # noqa: E402

T, H, F, V = 32768, 1024, 4096, 30528   # BERT-large, 64 x 512 tokens per GPU


def shapes(only):
    fw = [("qkv", H, 3 * H), ("out", H, H), ("ffn1", H, F), ("ffn2", F, H), ("head", H, V)]
    out = []
    for name, kin, nout in fw:
        if "fwd" in only:
            out.append((f"fwd_{name}", "fwd", kin, nout))
        if "dx" in only:
            out.append((f"dx_{name}", "dx", kin, nout))
        if "dw" in only:
            out.append((f"dw_{name}", "dw", kin, nout))
    return out


def operands(kind, kin, nout, dev):
    g = torch.Generator(device=dev).manual_seed(0)

    def r(*s):
        return (torch.rand(*s, device=dev, generator=g) * 2 - 1).bfloat16()
    if kind == "fwd":     # Y[T, nout] = X[T, kin] W[kin, nout]
        return r(T, kin), r(kin, nout), False, False
    if kind == "dx":      # dX[T, kin] = dY[T, nout] W[kin, nout]^T
        return r(T, nout), r(kin, nout), False, True
    return r(T, kin), r(T, nout), True, False   # dW[kin, nout] = X^T dY


def timed(fn, iters):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--only", default="fwd,dx,dw")
    ap.add_argument("--shapes", default="")
    ap.add_argument("--cands", default="", help="comma list of candidate prefixes (blaslt,p,q,r,t,u,v,w,n)")
    ap.add_argument("--tokens", type=int, default=T)
    ap.add_argument("--beta", type=float, default=0.0, help="accumulate into C (bf16 out): C = AB + beta C")
    args = ap.parse_args()
    globals()["T"] = args.tokens
    dev = "cuda"
    only = set(args.only.split(","))
    for name, kind, kin, nout in shapes(only):
        if args.shapes and name not in args.shapes.split(","):
            continue
        a, b, ta, tb = operands(kind, kin, nout, dev)
        M, N = (a.shape[1] if ta else a.shape[0]), (b.shape[0] if tb else b.shape[1])
        Kd = a.shape[0] if ta else a.shape[1]
        ref = (a.float().t() if ta else a.float()) @ (b.float().t() if tb else b.float())
        bt = args.beta
        cands = {"blaslt": lambda o: K.blaslt_gemm(a, b, trans_a=ta, trans_b=tb, out=o, beta=bt)}
        splits = [1] if kind != "dw" else [2, 4, 8]
        variants = {"p": 0, "q": 1, "r": 2, "t": 3, "u": 4, "v": 5, "w": 6, "x": 10}
        for sp in splits:
            for pre, var in variants.items():
                cands[f"{pre}{sp}"] = (lambda o, sp=sp, var=var:
                                       K.gemmp(a, b, trans_a=ta, trans_b=tb, out=o, beta=bt, splits=sp, variant=var))
        if tb and not ta:   # the eight-wave NT kernels (gemmn.hip, gemmpp.hip modes 0-3 as y0-y3)
            cands["n1"] = lambda o: K.gemmp(a, b, trans_a=ta, trans_b=tb, out=o, beta=bt, variant=9)
            for md in (1, 2, 5, 6):   # bits 0-1: DMA split (1: A / B by group, 2: A triple-buffered), bit 2: setprio
                cands[f"y{md}"] = (lambda o, md=md:
                                   K.gemmp(a, b, trans_a=ta, trans_b=tb, out=o, beta=bt, variant=11, _dbg=16 | md))
        if args.cands:
            keep = args.cands.split(",")
            cands = {k: v for k, v in cands.items() if k == "blaslt" and "blaslt" in keep
                     or k != "blaslt" and k.rstrip("0123456789") in keep}
        if bt:
            ref = ref + bt * 0.5   # outputs start at 0.5 below
        outs = {k: torch.empty(M, N, device=dev, dtype=torch.bfloat16) for k in cands}
        err = {}
        for k, f in cands.items():
            outs[k].fill_(0.5)
            f(outs[k])
            torch.cuda.synchronize()
            err[k] = ((outs[k].float() - ref).abs().max() / ref.abs().max()).item()
        times = {k: [] for k in cands}
        for _ in range(args.rounds):
            for k, f in cands.items():
                times[k].append(timed(lambda f=f, k=k: f(outs[k]), args.iters))
        fl = 2.0 * M * N * Kd
        res = {"case": name, "M": M, "N": N, "K": Kd, "ta": ta, "tb": tb}
        for k in cands:
            med = statistics.median(times[k])
            res[k] = round(med, 4)
            res[k + "_TF"] = round(fl / med / 1e9, 1)
            res[k + "_err"] = round(err[k], 5)
        best = min(cands, key=lambda k: res[k])
        res["best"] = best
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
