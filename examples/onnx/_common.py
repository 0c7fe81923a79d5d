"""Shared helpers of the ONNX examples: the repo on sys.path, quick-run
overrides (FF_EXAMPLE_SAMPLES) and where .onnx files go (FF_EXAMPLE_DIR)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def num_samples(default: int) -> int:
    return int(os.environ.get("FF_EXAMPLE_SAMPLES", default))


def onnx_path(name: str) -> str:
    d = os.environ.get("FF_EXAMPLE_DIR", ".")
    os.makedirs(d, exist_ok=True)
    return os.path.join(d, name)


def upsample(x, size):
    import numpy as np
    idx = np.arange(size) * x.shape[-1] // size
    return x[:, :, idx][:, :, :, idx]


def test_type(default=1) -> int:
    """--test_type 1: the PyTorch-exported file, 0: the keras-exported one."""
    import argparse
    p = argparse.ArgumentParser(add_help=False)
    p.add_argument("--test_type", type=int, choices=[0, 1], default=default)
    return p.parse_known_args()[0].test_type


def report(ffconfig, ts_start, samples, epochs):
    run_time = 1e-6 * (ffconfig.get_current_time() - ts_start)
    print("epochs %d, ELAPSED TIME = %.4fs, THROUGHPUT = %.2f samples/s" %
          (epochs, run_time, samples * epochs / max(run_time, 1e-9)))
