#!/usr/bin/env python3
"""Micro-benchmarks of the gfx950 kernels against the PyTorch-ROCm library
paths (hipBLASLt GEMM, SDPA attention) on the BERT-large / GPT-3-medium
shapes.  Interleaved rounds in one process (guide §5.4 rule 24), random
data (rule 25).  Prints one JSON line per case."""
import json
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from flexflow_train_amd import kernels as K  # noqa: E402


def timeit(fn, iters=20, rounds=3):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    best = float("inf")
    for _ in range(rounds):
        s = torch.cuda.Event(enable_timing=True)
        e = torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        e.synchronize()
        best = min(best, s.elapsed_time(e) / iters)
    return best


def bench_gemm(tokens=16384, hidden=1024, ffn=4096):
    dev = "cuda"
    cases = [
        ("qkv_fwd", tokens, 3 * hidden, hidden, False, False),
        ("out_fwd", tokens, hidden, hidden, False, False),
        ("fc1_fwd", tokens, ffn, hidden, False, False),
        ("fc2_fwd", tokens, hidden, ffn, False, False),
        ("fc1_dx", tokens, hidden, ffn, False, True),
        ("fc1_dw", hidden, ffn, tokens, True, False),
        ("fc2_dw", ffn, hidden, tokens, True, False),
        ("vocab_fwd", tokens, 30528, hidden, False, False),
    ]
    for name, M, N, Kd, ta, tb in cases:
        a = torch.randn((Kd, M) if ta else (M, Kd), device=dev, dtype=torch.bfloat16)
        b = torch.randn((N, Kd) if tb else (Kd, N), device=dev, dtype=torch.bfloat16)
        A = a.t() if ta else a
        B = b.t() if tb else b
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        t_hip = timeit(lambda: K.gemm(a, b, trans_a=ta, trans_b=tb, out=out))
        t_blas = timeit(lambda: torch.mm(A, B))
        fl = 2.0 * M * N * Kd
        print(json.dumps({"bench": "gemm", "case": name, "M": M, "N": N, "K": Kd, "ta": ta, "tb": tb,
                          "hip_ms": round(t_hip, 4), "hipblaslt_ms": round(t_blas, 4),
                          "hip_tflops": round(fl / t_hip / 1e9, 1), "hipblaslt_tflops": round(fl / t_blas / 1e9, 1)}),
              flush=True)


def bench_attention(B=32, S=512, H=16, D=64, causal=False):
    dev = "cuda"
    qkv = torch.randn(B, S, 3, H, D, device=dev, dtype=torch.bfloat16)
    q, k, v = qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]
    o, lse = K.attention_fwd(q, k, v, causal=causal)
    do = torch.randn_like(o)
    dqkv = torch.empty_like(qkv)
    t_fwd = timeit(lambda: K.attention_fwd(q, k, v, causal=causal, out=o))
    t_bwd = timeit(lambda: K.attention_bwd(q, k, v, o, lse, do, dqkv[:, :, 0], dqkv[:, :, 1], dqkv[:, :, 2],
                                           causal=causal))
    qt, kt, vt = (t.transpose(1, 2).contiguous() for t in (q, k, v))
    sdpa = torch.nn.functional.scaled_dot_product_attention
    t_sdpa = timeit(lambda: sdpa(qt, kt, vt, is_causal=causal))
    qr, kr, vr = (t.detach().clone().requires_grad_(True) for t in (qt, kt, vt))
    out = sdpa(qr, kr, vr, is_causal=causal)
    go = torch.randn_like(out)
    t_sdpa_bwd = timeit(lambda: torch.autograd.grad(out, (qr, kr, vr), go, retain_graph=True))
    fl = 4.0 * B * H * S * S * D * (0.5 if causal else 1.0)
    print(json.dumps({"bench": "attention", "B": B, "S": S, "H": H, "D": D, "causal": causal,
                      "fwd_ms": round(t_fwd, 4), "bwd_ms": round(t_bwd, 4),
                      "fwd_tflops": round(fl / t_fwd / 1e9, 1), "bwd_tflops": round(2.5 * fl / t_bwd / 1e9, 1),
                      "sdpa_fwd_ms": round(t_sdpa, 4), "sdpa_bwd_ms": round(t_sdpa_bwd, 4)}), flush=True)


def bench_memory_bound(M=16384, N=1024):
    dev = "cuda"
    x = torch.randn(M, N, device=dev, dtype=torch.bfloat16)
    r = torch.randn(M, N, device=dev, dtype=torch.bfloat16)
    g = torch.ones(N, device=dev, dtype=torch.bfloat16)
    b = torch.zeros(N, device=dev, dtype=torch.bfloat16)
    t = timeit(lambda: K.layernorm_fwd(x, g, b, 1e-12, residual=r))
    tt = timeit(lambda: torch.nn.functional.layer_norm(x + r, (N,), g, b, 1e-12))
    byts = 4 * M * N * 2
    print(json.dumps({"bench": "add_layernorm_fwd", "M": M, "N": N, "ms": round(t, 4), "torch_ms": round(tt, 4),
                      "GBps": round(byts / t / 1e6, 1)}), flush=True)
    y, s, mean, rstd = K.layernorm_fwd(x, g, b, 1e-12, residual=r)
    dg = torch.zeros(N, device=dev)
    db = torch.zeros(N, device=dev)
    t = timeit(lambda: K.layernorm_bwd(x, s, mean, rstd, g, dg, db))
    print(json.dumps({"bench": "layernorm_bwd", "M": M, "N": N, "ms": round(t, 4),
                      "GBps": round(3 * M * N * 2 / t / 1e6, 1)}), flush=True)
    V = 30528
    logits = torch.randn(M, V, device=dev, dtype=torch.bfloat16)
    labels = torch.randint(0, 30522, (M,), device=dev)
    t = timeit(lambda: K.softmax_ce(logits, labels, 1.0 / M, valid_cols=30522), iters=5)
    print(json.dumps({"bench": "softmax_ce", "M": M, "V": V, "ms": round(t, 4),
                      "GBps": round(3 * M * V * 2 / t / 1e6, 1)}), flush=True)
    n = 335_000_000 // 4 * 4
    w = torch.randn(n, device=dev)
    gg = torch.randn(n, device=dev)
    m = torch.zeros(n, device=dev)
    v = torch.zeros(n, device=dev)
    wb = torch.empty(n, device=dev, dtype=torch.bfloat16)
    t = timeit(lambda: K.adam_step(w, gg, m, v, wb, 1e-4, 0.9, 0.999, 1e-8, 0.01, 1), iters=5)
    print(json.dumps({"bench": "adam_flat", "n": n, "ms": round(t, 4), "GBps": round(n * 22 / t / 1e6, 1)}),
          flush=True)


if __name__ == "__main__":
    which = sys.argv[1:] or ["gemm", "attention", "mem"]
    if "gemm" in which:
        bench_gemm()
    if "attention" in which:
        bench_attention()
        bench_attention(B=8, S=2048, H=16, D=64, causal=True)
        bench_attention(B=4, S=2048, H=16, D=128, causal=True)
    if "mem" in which:
        bench_memory_bound()
