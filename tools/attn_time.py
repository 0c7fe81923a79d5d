#!/usr/bin/env python3
"""Time the flash-attention forward and backward (HIP events) on the BERT-large
and GPT-3-medium shapes; FF_PKG_ROOT selects the package tree (same-box A/B of
two builds: FF_PKG_ROOT=ab_prev python tools/attn_time.py).

    python tools/attn_time.py [iters]
    python tools/attn_time.py --pipe-ab | --delta-ab   (same-process A/B of a kernel switch)
"""
import json
import os
import sys

sys.path.insert(0, os.environ.get("FF_PKG_ROOT") or os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from flexflow_train_amd import kernels as K  # noqa: E402

SHAPES = {"bert-large": (64, 512, 16, 64, False), "gpt3-medium": (16, 2048, 16, 64, True)}   # bench batches


def _time(fn, iters):
    for _ in range(3):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters


def env_ab(var, which, iters, rounds=5):
    """Interleaved same-process A/B of one kernel switch (env `var` 0 vs 1,
    read per launch by attention.hip) on the forward or the backward."""
    import statistics
    for name, (B, S, H, D, causal) in SHAPES.items():
        g = torch.Generator(device="cuda").manual_seed(0)
        qkv = torch.randn(B, S, 3, H, D, device="cuda", dtype=torch.bfloat16, generator=g)
        q, k, v = qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]
        do = torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16, generator=g)
        dqkv = torch.empty_like(qkv)
        o, lse = K.attention_fwd(q, k, v, causal=causal)
        if which == "fwd":
            fn = lambda: K.attention_fwd(q, k, v, causal=causal, out=o)  # noqa: E731
        else:
            fn = lambda: K.attention_bwd(q, k, v, o, lse, do, dqkv[:, :, 0], dqkv[:, :, 1],  # noqa: E731
                                         dqkv[:, :, 2], causal=causal)
        t = {0: [], 1: []}
        for _ in range(rounds):
            for p in (0, 1):
                os.environ[var] = str(p)
                t[p].append(_time(fn, iters))
        fl = 4 * B * H * S * S * D * (0.5 if causal else 1.0) * (1.0 if which == "fwd" else 2.5)
        med = {p: statistics.median(v) for p, v in t.items()}
        print(json.dumps({"shape": name, "switch": var, "pass": which, "ms_0": round(med[0], 4),
                          "ms_1": round(med[1], 4), "tflops_0": round(fl / med[0] / 1e9, 1),
                          "tflops_1": round(fl / med[1] / 1e9, 1)}), flush=True)
    os.environ.pop(var, None)


def pmc_run(n=5):
    """A few dispatches of each kernel for a counter pass (rocprofv3 --pmc):
    forward default, forward pipelined, backward, at both bench shapes."""
    for name, (B, S, H, D, causal) in SHAPES.items():
        g = torch.Generator(device="cuda").manual_seed(0)
        qkv = torch.randn(B, S, 3, H, D, device="cuda", dtype=torch.bfloat16, generator=g)
        q, k, v = qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]
        do = torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16, generator=g)
        dqkv = torch.empty_like(qkv)
        o, lse = K.attention_fwd(q, k, v, causal=causal)
        for p in ("0", "1"):
            os.environ["FFK_ATTN_FWD_PIPE"] = p
            for _ in range(n):
                K.attention_fwd(q, k, v, causal=causal, out=o)
        os.environ.pop("FFK_ATTN_FWD_PIPE", None)
        for _ in range(n):
            K.attention_bwd(q, k, v, o, lse, do, dqkv[:, :, 0], dqkv[:, :, 1], dqkv[:, :, 2], causal=causal)
        torch.cuda.synchronize()
        print(name, "done", flush=True)


def main():
    if "--pmc-run" in sys.argv:
        return pmc_run()
    if "--pipe-ab" in sys.argv:        # software-pipelined forward
        return env_ab("FFK_ATTN_FWD_PIPE", "fwd", 50)
    if "--delta-ab" in sys.argv:       # delta fused into the dQ kernel
        return env_ab("FFK_ATTN_BWD_FUSED_DELTA", "bwd", 30)
    if "--wide-ab" in sys.argv:        # 16-B output row stores (forward / backward epilogues)
        env_ab("FFK_ATTN_WIDE_STORE", "fwd", 50)
        return env_ab("FFK_ATTN_WIDE_STORE", "bwd", 30)
    if "--xcd-ab" in sys.argv:         # XCD-local head order (non-causal grids)
        env_ab("FFK_ATTN_XCD", "fwd", 50)
        return env_ab("FFK_ATTN_XCD", "bwd", 30)
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    for name, (B, S, H, D, causal) in SHAPES.items():
        g = torch.Generator(device="cuda").manual_seed(0)
        qkv = torch.randn(B, S, 3, H, D, device="cuda", dtype=torch.bfloat16, generator=g)
        q, k, v = qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]
        do = torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16, generator=g)
        dqkv = torch.empty_like(qkv)
        o, lse = K.attention_fwd(q, k, v, causal=causal)
        fwd = _time(lambda: K.attention_fwd(q, k, v, causal=causal, out=o), iters)
        bwd = _time(lambda: K.attention_bwd(q, k, v, o, lse, do, dqkv[:, :, 0], dqkv[:, :, 1], dqkv[:, :, 2],
                                            causal=causal), iters)
        fl = 4 * B * H * S * S * D * (0.5 if causal else 1.0)
        print(json.dumps({"shape": name, "pkg": os.environ.get("FF_PKG_ROOT", "tree"), "fwd_ms": round(fwd, 4),
                          "bwd_ms": round(bwd, 4), "fwd_tflops": round(fl / fwd / 1e9, 1),
                          "bwd_tflops": round(2.5 * fl / bwd / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    main()
