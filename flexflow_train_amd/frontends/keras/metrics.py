"""Keras metric objects (reference: python/flexflow/keras/metrics.py)."""
from __future__ import annotations

from ...core import MetricsType


class Metric:
    type = None

    def __init__(self, name=None, dtype=None, **kw):
        self.name, self.dtype = name, dtype


class Accuracy(Metric):
    type = MetricsType.METRICS_ACCURACY

    def __init__(self, name="accuracy", dtype=None):
        super().__init__(name, dtype)


class CategoricalCrossentropy(Metric):
    type = MetricsType.METRICS_CATEGORICAL_CROSSENTROPY

    def __init__(self, name="categorical_crossentropy", dtype=None, from_logits=False, label_smoothing=0):
        super().__init__(name, dtype)


class SparseCategoricalCrossentropy(Metric):
    type = MetricsType.METRICS_SPARSE_CATEGORICAL_CROSSENTROPY

    def __init__(self, name="sparse_categorical_crossentropy", dtype=None, from_logits=False, axis=1):
        super().__init__(name, dtype)


class MeanSquaredError(Metric):
    type = MetricsType.METRICS_MEAN_SQUARED_ERROR

    def __init__(self, name="mean_squared_error", dtype=None):
        super().__init__(name, dtype)


class RootMeanSquaredError(Metric):
    type = MetricsType.METRICS_ROOT_MEAN_SQUARED_ERROR

    def __init__(self, name="root_mean_squared_error", dtype=None):
        super().__init__(name, dtype)


class MeanAbsoluteError(Metric):
    type = MetricsType.METRICS_MEAN_ABSOLUTE_ERROR

    def __init__(self, name="mean_absolute_error", dtype=None):
        super().__init__(name, dtype)


_BY_NAME = {"accuracy": Accuracy, "categorical_crossentropy": CategoricalCrossentropy,
            "sparse_categorical_crossentropy": SparseCategoricalCrossentropy,
            "mean_squared_error": MeanSquaredError, "mse": MeanSquaredError,
            "root_mean_squared_error": RootMeanSquaredError, "mean_absolute_error": MeanAbsoluteError,
            "mae": MeanAbsoluteError}


def get(m) -> Metric:
    if isinstance(m, Metric):
        return m
    if isinstance(m, MetricsType):
        o = Metric(m.name.lower())
        o.type = m
        return o
    if isinstance(m, str) and m in _BY_NAME:
        return _BY_NAME[m]()
    raise ValueError(f"unsupported metric {m!r}")
