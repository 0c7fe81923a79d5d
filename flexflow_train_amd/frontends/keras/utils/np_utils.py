"""numpy helpers (reference: python/flexflow/keras/utils/np_utils.py)."""
from __future__ import annotations

import numpy as np


def to_categorical(y, num_classes=None, dtype="float32"):
    """Class ids (any shape, trailing 1 dropped) -> one-hot rows."""
    y = np.asarray(y, dtype="int64")
    shape = y.shape
    if shape and shape[-1] == 1 and len(shape) > 1:
        shape = shape[:-1]
    y = y.ravel()
    n = int(num_classes or (y.max() + 1 if y.size else 0))
    out = np.zeros((y.shape[0], n), dtype=dtype)
    out[np.arange(y.shape[0]), y] = 1
    return out.reshape(shape + (n,))


def normalize(x, axis=-1, order=2):
    """x / its L-``order`` norm along ``axis`` (zero norms left as they are)."""
    n = np.atleast_1d(np.linalg.norm(x, order, axis))
    n[n == 0] = 1
    return x / np.expand_dims(n, axis)
