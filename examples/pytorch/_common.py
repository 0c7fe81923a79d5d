"""Shared helpers of the PyTorch-frontend examples: the repo on sys.path,
quick-run sample override (FF_EXAMPLE_SAMPLES) and the directory the .ff
files are written to / read from (FF_EXAMPLE_DIR, default the current one)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def num_samples(default: int) -> int:
    return int(os.environ.get("FF_EXAMPLE_SAMPLES", default))


def ff_path(name: str) -> str:
    d = os.environ.get("FF_EXAMPLE_DIR", ".")
    os.makedirs(d, exist_ok=True)
    return os.path.join(d, name)


def upsample(x, size):
    """Nearest-neighbour resize of NCHW uint8 images (the reference uses PIL)."""
    import numpy as np
    idx = np.arange(size) * x.shape[-1] // size
    return x[:, :, idx][:, :, :, idx]


def report(ffconfig, ts_start, samples, epochs):
    run_time = 1e-6 * (ffconfig.get_current_time() - ts_start)
    print("epochs %d, ELAPSED TIME = %.4fs, THROUGHPUT = %.2f samples/s" %
          (epochs, run_time, samples * epochs / max(run_time, 1e-9)))
