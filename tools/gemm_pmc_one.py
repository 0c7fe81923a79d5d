#!/usr/bin/env python3
"""One GEMM shape through hipBLASLt and gemmp variants (rocprofv3 --pmc
target): python tools/gemm_pmc_one.py M N K ta tb [variant[:splits]...]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from flexflow_train_amd import kernels as K  # noqa: E402

M, N, Kd, ta, tb = (int(x) for x in sys.argv[1:6])
variants = [tuple(int(x) for x in (v.split(":") + ["1"])[:2]) for v in sys.argv[6:]] or [(1, 1), (3, 1)]
a = (torch.rand(*((Kd, M) if ta else (M, Kd)), device="cuda") * 2 - 1).bfloat16()
b = (torch.rand(*((N, Kd) if tb else (Kd, N)), device="cuda") * 2 - 1).bfloat16()
out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
for _ in range(10):
    K.blaslt_gemm(a, b, trans_a=bool(ta), trans_b=bool(tb), out=out)
for v, sp in variants:
    for _ in range(10):
        K.gemmp(a, b, trans_a=bool(ta), trans_b=bool(tb), out=out, variant=v, splits=sp)
torch.cuda.synchronize()
print("done")
