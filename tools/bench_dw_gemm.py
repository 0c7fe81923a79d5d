#!/usr/bin/env python3
"""Weight-gradient GEMM alternatives (dW = X^T dY, K = tokens) on MI355X."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from flexflow_train_amd import kernels as K  # noqa: E402
from tools.bench_kernels import timeit  # noqa: E402


def main():
    dev = "cuda"
    T = 16384
    for name, kin, nout in (("qkv_dw", 1024, 3072), ("o_dw", 1024, 1024), ("fc1_dw", 1024, 4096),
                            ("fc2_dw", 4096, 1024), ("vocab_dw", 1024, 30528)):
        X = torch.randn(T, kin, device=dev, dtype=torch.bfloat16)
        dY = torch.randn(T, nout, device=dev, dtype=torch.bfloat16)
        out = torch.empty(kin, nout, device=dev, dtype=torch.bfloat16)
        res = {"case": name, "M": kin, "N": nout, "K": T}
        res["blaslt_XtdY"] = timeit(lambda: torch.mm(X.t(), dY, out=out))
        res["blaslt_swap_T"] = timeit(lambda: torch.mm(dY.t(), X).t())
        res["hip_kernel"] = timeit(lambda: K.gemm(X, dY, trans_a=True, out=out))
        Xt = X.t().contiguous()
        res["blaslt_pretransposed"] = timeit(lambda: torch.mm(Xt, dY, out=out))
        res["transpose_copy"] = timeit(lambda: X.t().contiguous())
        X2 = X.view(2, T // 2, kin)
        dY2 = dY.view(2, T // 2, nout)
        res["splitk2_bmm"] = timeit(lambda: torch.bmm(X2.transpose(1, 2), dY2).sum(0))
        try:
            torch.backends.cuda.preferred_blas_library("cublas")
            res["rocblas_XtdY"] = timeit(lambda: torch.mm(X.t(), dY, out=out))
        except Exception as e:  # noqa
            res["rocblas_err"] = str(e)[:80]
        finally:
            torch.backends.cuda.preferred_blas_library("cublaslt")
        fl = 2.0 * T * kin * nout
        best = min((v, k) for k, v in res.items() if isinstance(v, float) and k != "transpose_copy")
        res["best"] = best[1]
        res["best_tflops"] = round(fl / best[0] / 1e9, 1)
        for k, v in list(res.items()):
            if isinstance(v, float):
                res[k] = round(v, 4)
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
