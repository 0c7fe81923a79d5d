"""Shared helpers of the native examples: sample-count override for quick
runs (FF_EXAMPLE_SAMPLES) and the reference's THROUGHPUT line."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def num_samples(default: int) -> int:
    return int(os.environ.get("FF_EXAMPLE_SAMPLES", default))


def report(ffconfig, ts_start, samples, epochs):
    run_time = 1e-6 * (ffconfig.get_current_time() - ts_start)
    print("epochs %d, ELAPSED TIME = %.4fs, THROUGHPUT = %.2f samples/s" %
          (epochs, run_time, samples * epochs / max(run_time, 1e-9)))
