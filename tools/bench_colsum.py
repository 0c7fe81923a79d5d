#!/usr/bin/env python3
"""colsum_act (bias-grad / fused act-grad + bias-grad) bandwidth sweep."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from flexflow_train_amd import kernels as K  # noqa: E402
from tools.bench_kernels import timeit  # noqa: E402


def main():
    dev = "cuda"
    for M, N, act in ((16384, 1024, None), (16384, 3072, None), (16384, 4096, "gelu"), (16384, 30528, None)):
        dy = torch.randn(M, N, device=dev, dtype=torch.bfloat16)
        pre = torch.randn(M, N, device=dev, dtype=torch.bfloat16) if act else None
        db = torch.zeros(N, device=dev, dtype=torch.float32)
        fn = lambda: K.colsum_act(dy, pre, act or "none", db, write_dx=act is not None)  # noqa: E731
        ms = timeit(fn)
        nbytes = M * N * 2 * (3 if act else 1)
        ref = dy.float().sum(0) if not act else None
        print(json.dumps({"M": M, "N": N, "act": act, "ms": round(ms, 4), "TBps": round(nbytes / ms / 1e9, 2)}),
              flush=True)
        if ref is not None:
            db.zero_()
            K.colsum_act(dy, None, "none", db, write_dx=False)
            torch.testing.assert_close(db, ref, rtol=1e-3, atol=1e-2)


if __name__ == "__main__":
    main()
