"""Dataset loaders without network access: a local ``.npz`` (keys x_train,
y_train, x_test, y_test; read with allow_pickle=False) when one is given or
found under ~/.keras/datasets, else deterministic synthetic data with the
real dataset's shapes, dtypes and class count (class-conditional, so models
can learn it)."""
from __future__ import annotations

import os
from typing import Optional

import numpy as np


def local_npz(path: Optional[str]):
    if not path:
        return None
    for p in (path, os.path.join(os.path.expanduser("~"), ".keras", "datasets", path)):
        if os.path.isfile(p) and p.endswith(".npz"):
            with np.load(p, allow_pickle=False) as d:
                return (d["x_train"], d["y_train"]), (d["x_test"], d["y_test"])
    return None


def images(x_shape, n_classes, n_train, n_test, seed=0, label_shape=None):
    rng = np.random.default_rng(seed)
    centers = rng.integers(0, 255, (n_classes,) + tuple(x_shape))

    def mk(n):
        y = rng.integers(0, n_classes, n)
        x = np.clip(centers[y] + rng.normal(0, 30, (n,) + tuple(x_shape)), 0, 255).astype(np.uint8)
        y = y.astype(np.uint8)
        return x, (y.reshape((n,) + label_shape) if label_shape else y)
    return mk(n_train), mk(n_test)
