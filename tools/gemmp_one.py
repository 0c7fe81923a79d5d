#!/usr/bin/env python3
"""Run one GEMM shape through gemmp N times (rocprofv3 --pmc target).

    python tools/gemmp_one.py M N K [ta tb variant splits]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from flexflow_train_amd import kernels as K  # noqa: E402

args = sys.argv[1:]
M, N, Kd = (int(x) for x in (args[0:3] if len(args) >= 3 else (16384, 1024, 4096)))
ta, tb = (bool(int(x)) for x in (args[3:5] if len(args) >= 5 else (0, 0)))
variant = int(args[5]) if len(args) > 5 else 0
splits = int(args[6]) if len(args) > 6 else 1
a = (torch.rand(*((Kd, M) if ta else (M, Kd)), device="cuda") * 2 - 1).bfloat16()
b = (torch.rand(*((N, Kd) if tb else (Kd, N)), device="cuda") * 2 - 1).bfloat16()
out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
for _ in range(20):
    K.gemmp(a, b, trans_a=ta, trans_b=tb, out=out, variant=variant, splits=splits)
torch.cuda.synchronize()
print("done")
