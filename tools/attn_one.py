#!/usr/bin/env python3
"""Run the flash-attention forward + backward N times on one shape (a
rocprofv3 --pmc / --kernel-trace target).

    python tools/attn_one.py [B S H D causal iters]     default: BERT-large 32 512 16 64 0 20
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from flexflow_train_amd import kernels as K  # noqa: E402


def main():
    a = [int(x) for x in sys.argv[1:]] + [32, 512, 16, 64, 0, 20][len(sys.argv) - 1:]
    B, S, H, D, causal, iters = a[:6]
    g = torch.Generator(device="cuda").manual_seed(0)
    qkv = torch.randn(B, S, 3, H, D, device="cuda", dtype=torch.bfloat16, generator=g)
    q, k, v = qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]
    do = torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16, generator=g)
    dqkv = torch.empty_like(qkv)
    o, lse = K.attention_fwd(q, k, v, causal=bool(causal))
    for _ in range(iters):
        K.attention_fwd(q, k, v, causal=bool(causal), out=o)
        K.attention_bwd(q, k, v, o, lse, do, dqkv[:, :, 0], dqkv[:, :, 1], dqkv[:, :, 2], causal=bool(causal))
    torch.cuda.synchronize()
    print("ok", B, S, H, D, causal, iters)


if __name__ == "__main__":
    main()
