#!/usr/bin/env python3
"""Run one GEMM shape through gemmp N times (rocprofv3 --pmc target)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from flexflow_train_amd import kernels as K  # noqa: E402

M, N, Kd = (int(x) for x in (sys.argv[1:4] if len(sys.argv) > 3 else (16384, 1024, 4096)))
a = (torch.rand(M, Kd, device="cuda") * 2 - 1).bfloat16()
b = (torch.rand(Kd, N, device="cuda") * 2 - 1).bfloat16()
out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
for _ in range(20):
    K.gemmp(a, b, out=out)
torch.cuda.synchronize()
print("done")
