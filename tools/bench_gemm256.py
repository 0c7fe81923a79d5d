#!/usr/bin/env python3
"""gemm256 (LDS-DMA, split-K) vs hipBLASLt (torch.mm) vs gemm128 on the
BERT-large training GEMMs (T = 16384 tokens).  Random [-1,1)-scale data."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from flexflow_train_amd import kernels as K  # noqa: E402
from tools.bench_kernels import timeit  # noqa: E402


def run(name, M, N, Kd, ta, tb, splits_list=(None,)):
    dev = "cuda"
    a = (torch.rand(Kd, M, device=dev) * 2 - 1).bfloat16() if ta else (torch.rand(M, Kd, device=dev) * 2 - 1).bfloat16()
    b = (torch.rand(N, Kd, device=dev) * 2 - 1).bfloat16() if tb else (torch.rand(Kd, N, device=dev) * 2 - 1).bfloat16()
    A = a.t() if ta else a
    B = b.t() if tb else b
    out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    fl = 2.0 * M * N * Kd
    res = {"case": name, "M": M, "N": N, "K": Kd, "ta": ta, "tb": tb}
    res["blaslt"] = timeit(lambda: torch.mm(A, B, out=out))
    res["gemm128"] = timeit(lambda: K.gemm(a, b, trans_a=ta, trans_b=tb, out=out))
    for s in splits_list:
        key = f"gemm256_s{s if s else K.default_splits(M, N, Kd)}"
        res[key] = timeit(lambda: K.gemm256(a, b, trans_a=ta, trans_b=tb, out=out, splits=s))
    ref = (A.float() @ B.float())
    K.gemm256(a, b, trans_a=ta, trans_b=tb, out=out)
    res["err"] = float((out.float() - ref).norm() / ref.norm())
    for k in list(res):
        if isinstance(res[k], float) and k != "err":
            res[k + "_TF"] = round(fl / res[k] / 1e9, 1)
            res[k] = round(res[k], 4)
    print(json.dumps(res), flush=True)


def main():
    T = 16384
    # forward: Y[T, out] = X[T, in] W[in, out]
    run("fwd_qkv", T, 3072, 1024, False, False)
    run("fwd_ffn1", T, 4096, 1024, False, False)
    run("fwd_ffn2", T, 1024, 4096, False, False)
    # dX = dY W^T
    run("dx_ffn1", T, 1024, 4096, False, True)
    run("dx_ffn2", T, 4096, 1024, False, True)
    # dW = X^T dY (K = tokens)
    run("dw_qkv", 1024, 3072, T, True, False, (1, 2, 4, 8))
    run("dw_o", 1024, 1024, T, True, False, (4, 8, 16))
    run("dw_ffn1", 1024, 4096, T, True, False, (1, 2, 4, 8))
    run("dw_ffn2", 4096, 1024, T, True, False, (1, 2, 4, 8))
    run("dw_vocab", 1024, 30528, T, True, False, (1, 2))


if __name__ == "__main__":
    main()
