"""MNIST (reference: python/flexflow/keras/datasets/mnist.py): x uint8
(N, 28, 28), y uint8 (N,)."""
from ._synthetic import images, local_npz


def load_data(path="mnist.npz", num_samples=None):
    got = local_npz(path)
    if got is not None:
        return got
    n = int(num_samples or 60000)
    return images((28, 28), 10, n, min(10000, max(1, n // 6)), seed=0)
