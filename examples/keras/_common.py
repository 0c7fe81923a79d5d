"""Shared helpers of the keras examples: the repo on sys.path, quick-run
overrides (FF_EXAMPLE_SAMPLES / FF_EXAMPLE_EPOCHS, used by
tests/test_examples.py) and the accuracy checks the reference's CI runs."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from accuracy import ModelAccuracy  # noqa: E402,F401


def quick() -> bool:
    return "FF_EXAMPLE_SAMPLES" in os.environ


def num_samples(default: int) -> int:
    return int(os.environ.get("FF_EXAMPLE_SAMPLES", default))


def epochs(default: int) -> int:
    return int(os.environ.get("FF_EXAMPLE_EPOCHS", 1 if quick() else default))


def verify(accuracy):
    """VerifyMetrics + EpochVerifyMetrics(accuracy) for full runs; a quick
    run (few samples, one epoch) only reports."""
    from flexflow.keras.callbacks import EpochVerifyMetrics, VerifyMetrics
    return [EpochVerifyMetrics(accuracy)] if quick() else [VerifyMetrics(accuracy), EpochVerifyMetrics(accuracy)]


def mnist_flat(n=60000):
    import numpy as np
    from flexflow.keras.datasets import mnist
    (x, y), _ = mnist.load_data(num_samples=num_samples(n))
    return x.reshape(len(x), 784).astype("float32") / 255, np.reshape(y.astype("int32"), (len(y), 1))


def mnist_images(n=60000):
    import numpy as np
    from flexflow.keras.datasets import mnist
    (x, y), _ = mnist.load_data(num_samples=num_samples(n))
    return x.reshape(len(x), 1, 28, 28).astype("float32") / 255, np.reshape(y.astype("int32"), (len(y), 1))


def cifar10(n=10000):
    from flexflow.keras.datasets import cifar10 as c
    (x, y), _ = c.load_data(num_samples(n))
    return x.astype("float32") / 255, y.astype("int32")
