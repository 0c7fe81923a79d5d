#!/usr/bin/env python3
"""1x1-convolution forward paths on the ResNet-50 shapes (batch 256): the
implicit-GEMM conv with and without the BN-statistics epilogue, the
statistics pass alone, and hipBLASLt on the same GEMM -- where the 1x1
forward time goes.  One JSON line per shape."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from flexflow_train_amd import kernels as K  # noqa: E402
from bench_conv import timeit  # noqa: E402

SHAPES = [(56, 64, 64), (56, 64, 256), (56, 256, 64), (56, 256, 128), (28, 128, 512), (28, 512, 128),
          (14, 256, 1024), (14, 1024, 256), (7, 512, 2048), (7, 2048, 512)]


def main():
    N = 256
    for H, C, Ko in SHAPES:
        x = torch.randn(N, C, H, H, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        w = (torch.randn(Ko, 1, 1, C, device="cuda") * 0.05).to(torch.bfloat16).contiguous()
        stats = torch.zeros(2 * Ko, device="cuda")
        y = K.conv2d_fwd(x, w, None, (1, 1), (0, 0))
        r = {"H": H, "C": C, "K": Ko,
             "conv_stats": timeit(lambda: K.conv2d_fwd(x, w, None, (1, 1), (0, 0), stats=stats)),
             "conv": timeit(lambda: K.conv2d_fwd(x, w, None, (1, 1), (0, 0))),
             "bn_stats": timeit(lambda: K.bn_stats(y, stats, overwrite=True))}
        x2 = x.permute(0, 2, 3, 1).reshape(-1, C)
        w2 = w.reshape(Ko, C)
        r["blas"] = timeit(lambda: x2 @ w2.t())
        gb = (x.numel() + y.numel()) * 2 / 1e9
        r = {k: (round(v, 4) if isinstance(v, float) else v) for k, v in r.items()}
        r["io_gb"] = round(gb, 3)
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
