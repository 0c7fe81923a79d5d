#!/usr/bin/env python3
"""Per-layer micro-benchmark of the implicit-GEMM convolution kernels
(csrc/kernels/conv.hip) on the distinct ResNet-50 conv shapes at batch 256,
against MIOpen through PyTorch (channels_last bf16).  One JSON line per
shape with fwd / dgrad / wgrad times and TFLOP/s."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from flexflow_train_amd import kernels as K  # noqa: E402

# (H, C, K, R, stride, count in ResNet-50)
SHAPES = [
    (224, 8, 64, 7, 2, 1),  # stem (3 channels padded to 8)
    (56, 64, 64, 1, 1, 1), (56, 64, 64, 3, 1, 3), (56, 64, 256, 1, 1, 4), (56, 256, 64, 1, 1, 2),
    (56, 256, 128, 1, 1, 1), (56, 128, 128, 3, 2, 1), (28, 128, 512, 1, 1, 4), (56, 256, 512, 1, 2, 1),
    (28, 512, 128, 1, 1, 3), (28, 128, 128, 3, 1, 3), (28, 512, 256, 1, 1, 1), (28, 256, 256, 3, 2, 1),
    (14, 256, 1024, 1, 1, 6), (28, 512, 1024, 1, 2, 1), (14, 1024, 256, 1, 1, 5), (14, 256, 256, 3, 1, 5),
    (14, 1024, 512, 1, 1, 1), (14, 512, 512, 3, 2, 1), (7, 512, 2048, 1, 1, 3), (14, 1024, 2048, 1, 2, 1),
    (7, 2048, 512, 1, 1, 2), (7, 512, 512, 3, 1, 2),
]


def timeit(fn, iters=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = float("inf")
    for _ in range(3):
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        e.synchronize()
        best = min(best, s.elapsed_time(e) / iters)
    return best


def main():
    N = int(os.environ.get("BATCH", "256"))
    tot = {"ours": 0.0, "miopen": 0.0}
    for (H, C, Ko, R, st, cnt) in SHAPES:
        pad = R // 2
        x = torch.randn(N, C, H, H, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        w = (torch.randn(Ko, R, R, C, device="cuda") * 0.05).to(torch.bfloat16).contiguous()
        y = K.conv2d_fwd(x, w, None, (st, st), (pad, pad))
        dy = torch.randn_like(y).contiguous(memory_format=torch.channels_last)
        dw = torch.zeros(Ko * R * R * C, device="cuda")
        stats = torch.zeros(2 * Ko, device="cuda")
        t_f = timeit(lambda: K.conv2d_fwd(x, w, None, (st, st), (pad, pad), stats=stats))
        t_d = timeit(lambda: K.conv2d_dgrad(dy, w, tuple(x.shape), (st, st), (pad, pad)))
        t_w = timeit(lambda: K.conv2d_wgrad(x, dy, dw, R, R, (st, st), (pad, pad)))
        wt = w.permute(0, 3, 1, 2).contiguous(memory_format=torch.channels_last)
        xr = x.detach().requires_grad_(True)
        wr = wt.detach().requires_grad_(True)
        m_f = timeit(lambda: F.conv2d(x, wt, stride=st, padding=pad))
        out = F.conv2d(xr, wr, stride=st, padding=pad)
        m_b = timeit(lambda: torch.autograd.grad(out, (xr, wr), dy, retain_graph=True))
        P = y.shape[2]
        fl = 2.0 * N * P * P * Ko * R * R * C
        lib = {}
        if R == 1 and st == 1:  # a 1x1 stride-1 NHWC conv is a plain GEMM: time hipBLASLt on it
            x2 = x.permute(0, 2, 3, 1).reshape(-1, C)
            w2 = w.reshape(Ko, C)
            dy2 = dy.permute(0, 2, 3, 1).reshape(-1, Ko)
            dwf = torch.empty(Ko, C, device="cuda")
            lib = {"blas_fwd_ms": round(timeit(lambda: x2 @ w2.t()), 4),
                   "blas_dgrad_ms": round(timeit(lambda: dy2 @ w2), 4),
                   "blas_wgrad_ms": round(timeit(lambda: torch.mm(dy2.t(), x2, out_dtype=torch.float32, out=dwf)), 4)}
        ours = t_f + t_d + t_w
        tot["ours"] += cnt * ours
        tot["miopen"] += cnt * (m_f + m_b)
        print(json.dumps({"bench": "conv", "H": H, "C": C, "K": Ko, "R": R, "stride": st, "count": cnt,
                          "fwd_ms": round(t_f, 4), "dgrad_ms": round(t_d, 4), "wgrad_ms": round(t_w, 4),
                          "fwd_tflops": round(fl / t_f / 1e9, 1), "dgrad_tflops": round(fl / t_d / 1e9, 1),
                          "wgrad_tflops": round(fl / t_w / 1e9, 1),
                          "miopen_fwd_ms": round(m_f, 4), "miopen_bwd_ms": round(m_b, 4), **lib}), flush=True)
    print(json.dumps({"bench": "conv_total_resnet50", "batch": N, "ours_ms": round(tot["ours"], 3),
                      "miopen_ms": round(tot["miopen"], 3)}), flush=True)


if __name__ == "__main__":
    main()
