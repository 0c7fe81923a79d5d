#!/usr/bin/env python3
"""Bandwidth of the NHWC BatchNorm / pooling kernels (bnpool.hip) at ResNet-50
layer-1 shapes (batch 256): achieved GB/s against the bytes each pass must move."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from flexflow_train_amd import kernels as K  # noqa: E402
from tools.bench_kernels import timeit  # noqa: E402


def main():
    for (N, C, H) in [(256, 256, 56), (256, 64, 56), (256, 2048, 7)]:
        x = torch.randn(N, C, H, H, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        dy = torch.randn_like(x)
        g = torch.ones(C, device="cuda", dtype=torch.bfloat16)
        b = torch.zeros(C, device="cuda", dtype=torch.bfloat16)
        nb = x.numel() * 2
        stats = torch.zeros(2 * C, device="cuda")
        t_stats = timeit(lambda: (stats.zero_(), K.bn_stats(x, stats)))
        scale, shift, mean, rstd = K.bn_finalize(stats, g, b, x.numel() // C, 1e-5)
        t_apply = timeit(lambda: K.bn_apply(x, scale, shift, True))
        y = K.bn_apply(x, scale, shift, True)
        t_apply_res = timeit(lambda: K.bn_apply(x, scale, shift, True, residual=dy))
        t_bwd = timeit(lambda: K.bn_bwd(dy, x, y, mean, rstd, g, True))
        ss = torch.stack([scale, shift]).reshape(-1)
        t_bwd_x = timeit(lambda: K.bn_bwd(dy, x, None, mean, rstd, g, True, scale_shift=ss))
        print(json.dumps({"bench": "batchnorm", "shape": [N, C, H, H], "MB": round(nb / 1e6, 1),
                          "stats_ms": round(t_stats, 4), "stats_GBps": round(nb / t_stats / 1e6, 1),
                          "apply_ms": round(t_apply, 4), "apply_GBps": round(2 * nb / t_apply / 1e6, 1),
                          "apply_res_GBps": round(3 * nb / t_apply_res / 1e6, 1),
                          "bwd_ms": round(t_bwd, 4), "bwd_GBps": round(7 * nb / t_bwd / 1e6, 1),
                          "bwd_mask_from_x_ms": round(t_bwd_x, 4),
                          "bwd_mask_from_x_GBps": round(5 * nb / t_bwd_x / 1e6, 1)}), flush=True)
    s = torch.empty(1 << 28, device="cuda", dtype=torch.bfloat16)
    d = torch.empty_like(s)
    t = timeit(lambda: d.copy_(s))
    print(json.dumps({"bench": "torch_copy_reference", "MB": 2 * s.numel() * 2 / 1e6,
                      "GBps": round(2 * s.numel() * 2 / t / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
