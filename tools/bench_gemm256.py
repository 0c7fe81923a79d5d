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
    res["gemmp"] = timeit(lambda: K.gemmp(a, b, trans_a=ta, trans_b=tb, out=out))
    res["gemmp_stag"] = timeit(lambda: K.gemmp(a, b, trans_a=ta, trans_b=tb, out=out, _dbg=4))
    K.gemmp(a, b, trans_a=ta, trans_b=tb, out=out, _dbg=4)
    res["err_p_stag"] = float((out.float() - (A.float() @ B.float())).norm() / (A.float() @ B.float()).norm())
    if os.environ.get("GEMMP_ABLATE"):
        for d in (1, 2, 3, 4):
            res[f"gemmp_dbg{d}"] = timeit(lambda: K.gemmp(a, b, trans_a=ta, trans_b=tb, out=out, _dbg=d))
    for s in splits_list:
        if s and s > 1:
            res[f"gemmp_s{s}"] = timeit(lambda: K.gemmp(a, b, trans_a=ta, trans_b=tb, out=out, splits=s))
            res[f"gemmp_stag_s{s}"] = timeit(lambda: K.gemmp(a, b, trans_a=ta, trans_b=tb, out=out, splits=s,
                                                              _dbg=4))
    ref = (A.float() @ B.float())
    K.gemmp(a, b, trans_a=ta, trans_b=tb, out=out)
    res["err_p"] = float((out.float() - ref).norm() / ref.norm())
    for s in splits_list:
        if s and s > 1:
            K.gemmp(a, b, trans_a=ta, trans_b=tb, out=out, splits=s)
            res[f"err_p_s{s}"] = float((out.float() - ref).norm() / ref.norm())
    K.gemm256(a, b, trans_a=ta, trans_b=tb, out=out)
    res["err"] = float((out.float() - ref).norm() / ref.norm())
    for k in list(res):
        if isinstance(res[k], float) and not k.startswith("err"):
            res[k + "_TF"] = round(fl / res[k] / 1e9, 1)
            res[k] = round(res[k], 4)
    print(json.dumps(res), flush=True)


def main():
    T = 16384
    # odd shapes: partial edge tiles, a single K-tile, split remainders
    run("edge", 1000, 776, 192, False, False, (None, 2))
    run("edge_tn", 520, 1032, 128, True, False, (None, 2))
    run("edge_nt", 264, 264, 64, False, True)
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


if __name__ == "__main__" and "--epilogues" not in sys.argv:
    main()


def check_epilogues():
    """gemmp fused epilogues against fp32 references (bias+GELU+pre,
    activation-gradient + bias-gradient column sums, beta accumulate)."""
    dev = "cuda"
    torch.manual_seed(0)
    for (M, N, Kd) in ((1024, 768, 512), (1000, 1032, 192)):
        a = (torch.randn(M, Kd, device=dev) * 0.5).bfloat16()
        b = (torch.randn(Kd, N, device=dev) * 0.5).bfloat16()
        bias = torch.randn(N, device=dev).bfloat16()
        ref = a.float() @ b.float()
        pre = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        y = K.gemmp(a, b, bias=bias, act="gelu", pre=pre)
        u = ref + bias.float()
        e1 = float((pre.float() - u).abs().max() / u.abs().max())
        e2 = float((y.float() - torch.nn.functional.gelu(u, approximate="tanh")).abs().max() / u.abs().max())
        aux = torch.randn(M, N, device=dev).bfloat16()
        db = torch.zeros(N, device=dev)
        g = K.gemmp(a, b, act="gelu", aux=aux, act_bwd=True, dbias=db)
        x = aux.float().requires_grad_(True)
        torch.nn.functional.gelu(x, approximate="tanh").backward(torch.ones_like(x))
        gr = ref * x.grad
        e3 = float((g.float() - gr).abs().max() / gr.abs().max())
        e4 = float((db - g.float().sum(0)).abs().max() / g.float().sum(0).abs().max())
        c = torch.randn(M, N, device=dev)
        c0 = c.clone()
        K.gemmp(a, b, out=c, beta=1.0)
        e5 = float((c - (c0 + ref)).abs().max() / ref.abs().max())
        print(json.dumps({"epilogue_check": [M, N, Kd], "pre": e1, "gelu": e2, "dgelu": e3, "dbias": e4,
                          "beta_f32": e5}), flush=True)


if __name__ == "__main__" and "--epilogues" in sys.argv:
    check_epilogues()
