#!/usr/bin/env python3
"""Time the fused softmax + cross-entropy kernel at the BERT-large and
GPT-3-medium vocabulary shapes (HIP events); FF_PKG_ROOT selects the package
tree for a same-box A/B of two builds.

    python tools/ce_time.py [iters]
"""
import json
import os
import sys

sys.path.insert(0, os.environ.get("FF_PKG_ROOT") or os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from flexflow_train_amd import kernels as K  # noqa: E402

SHAPES = {"bert-large": (16384, 30528, 30522), "gpt3-medium": (16384, 50264, 50257)}


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    use_metrics = "--no-metrics" not in sys.argv
    for name, (M, V, Vv) in SHAPES.items():
        g = torch.Generator(device="cuda").manual_seed(0)
        x = (torch.randn(M, V, device="cuda", generator=g) * 3).to(torch.bfloat16)
        lab = torch.randint(0, Vv, (M,), device="cuda", generator=g)
        met = torch.zeros(4, device="cuda") if use_metrics else None
        for _ in range(3):
            K.softmax_ce(x, lab, 1.0 / M, metrics=met, valid_cols=Vv)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(iters):
            K.softmax_ce(x, lab, 1.0 / M, metrics=met, valid_cols=Vv)
        b.record()
        torch.cuda.synchronize()
        ms = a.elapsed_time(b) / iters
        print(json.dumps({"shape": name, "pkg": os.environ.get("FF_PKG_ROOT", "tree"), "metrics": use_metrics, "ms": round(ms, 4),
                          "TB_s": round(2 * M * V * 2 / ms / 1e9, 2)}), flush=True)
        del x


if __name__ == "__main__":
    main()
