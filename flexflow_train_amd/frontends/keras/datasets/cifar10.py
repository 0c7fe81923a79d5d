"""CIFAR-10 (reference: python/flexflow/keras/datasets/cifar10.py): x uint8
channels-first (N, 3, 32, 32), y uint8 (N, 1)."""
from ._synthetic import images, local_npz


def load_data(num_samples=40000, path="cifar10.npz"):
    got = local_npz(path)
    if got is not None:
        return got
    n = int(num_samples)
    return images((3, 32, 32), 10, n, min(10000, max(1, n // 6)), seed=1, label_shape=(1,))
