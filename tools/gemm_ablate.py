#!/usr/bin/env python3
"""Sync-cost ablation of the phase-pipelined GEMMs (timing only: with the
waits or barriers removed the results are garbage).  gemmp / gemmq (variants
0 / 1) dbg bits: 1 = no vmcnt waits, 2 = no barriers.  gemmt (variant 3,
NN / NT only, ``--gemmt``): 1 = no global loads in the loop, 2 = no LDS
writes (the loads then die too), 4 = no mid-tile barrier, 8 = no epilogue,
15 = all of them (MFMAs + fragment reads only), 16 = non-temporal epilogue stores, 32 = C staged through
LDS and stored as whole rows (a correct result: its error is reported).  LDS-DMA forms
(GEMMT_ABL_VARIANT=4 or 6): 128 = no wait for the next K-tile's loads (exposed load latency),
8 = no epilogue, 136 = both.  Interleaved rounds in one
process:  [GEMMT_ABL_VARIANT=6 GEMMT_DBG=0,128,8,136] python tools/gemm_ablate.py [--gemmt]"""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from flexflow_train_amd import kernels as K  # noqa: E402
from tools.gemm_ab import operands, timed  # noqa: E402

CASES = [("fwd_qkv", "fwd", 1024, 3072), ("dx_ffn1", "dx", 1024, 4096), ("fwd_ffn2", "fwd", 4096, 1024),
         ("dw_ffn1", "dw", 1024, 4096), ("fwd_ffn1", "fwd", 1024, 4096), ("dx_qkv", "dx", 1024, 3072)]


def main():
    for name, kind, kin, nout in CASES:
        a, b, ta, tb = operands(kind, kin, nout, "cuda")
        M, N = (a.shape[1] if ta else a.shape[0]), (b.shape[0] if tb else b.shape[1])
        Kd = a.shape[0] if ta else a.shape[1]
        sp = 4 if kind == "dw" else 1
        out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        cands = {}
        if "--gemmt" in sys.argv:
            if ta:
                continue
            cands["blaslt"] = lambda: K.blaslt_gemm(a, b, trans_a=ta, trans_b=tb, out=out)
            var = int(os.environ.get("GEMMT_ABL_VARIANT", "3"))
            for dbg in [int(x) for x in os.environ.get("GEMMT_DBG", "0,8,32").split(",")]:
                cands[f"t_d{dbg}"] = lambda dbg=dbg: K.gemmp(a, b, trans_a=ta, trans_b=tb, out=out, splits=sp,
                                                             variant=var, _dbg=dbg)
        else:
            for v in (0, 1):
                for dbg in (0, 1, 2, 3):
                    cands[f"v{v}_d{dbg}"] = lambda v=v, dbg=dbg: K.gemmp(a, b, trans_a=ta, trans_b=tb, out=out,
                                                                         splits=sp, variant=v, _dbg=dbg)
        errs = {}
        if "--gemmt" in sys.argv:
            ref = ((a.float().t() if ta else a.float()) @ (b.float().t() if tb else b.float()))
            for k in ("t_d0", "t_d32", "t_d256"):
                if k in cands:
                    cands[k]()
                    errs[k + "_err"] = round(((out.float() - ref).norm() / ref.norm()).item(), 5)
        times = {k: [] for k in cands}
        for _ in range(5):
            for k, f in cands.items():
                times[k].append(timed(f, 10))
        fl = 2.0 * M * N * Kd
        res = {"case": name, **errs}
        for k in cands:
            res[k + "_TF"] = round(fl / statistics.median(times[k]) / 1e9, 1)
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
