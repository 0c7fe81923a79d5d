"""Keras loss objects (reference: python/flexflow/keras/losses.py)."""
from __future__ import annotations

from ...core import LossType


class Loss:
    type = None

    def __init__(self, name=None, reduction="auto"):
        self.name = name
        self.reduction = reduction


class CategoricalCrossentropy(Loss):
    type = LossType.LOSS_CATEGORICAL_CROSSENTROPY

    def __init__(self, from_logits=False, label_smoothing=0, reduction="auto", name="categorical_crossentropy"):
        super().__init__(name, reduction)


class SparseCategoricalCrossentropy(Loss):
    type = LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY

    def __init__(self, from_logits=False, reduction="auto", name="sparse_categorical_crossentropy"):
        super().__init__(name, reduction)


class MeanSquaredError(Loss):
    type = LossType.LOSS_MEAN_SQUARED_ERROR_AVG_REDUCE

    def __init__(self, reduction="auto", name="mean_squared_error"):
        super().__init__(name, reduction)
        if reduction == "sum":
            self.type = LossType.LOSS_MEAN_SQUARED_ERROR_SUM_REDUCE


class Identity(Loss):
    """The model output is the loss (its gradient is 1 / batch)."""
    type = LossType.LOSS_IDENTITY

    def __init__(self, reduction="auto", name="identity"):
        super().__init__(name, reduction)


_BY_NAME = {"categorical_crossentropy": CategoricalCrossentropy,
            "sparse_categorical_crossentropy": SparseCategoricalCrossentropy,
            "mean_squared_error": MeanSquaredError, "mse": MeanSquaredError, "identity": Identity}


def get(loss) -> Loss:
    if isinstance(loss, Loss):
        return loss
    if isinstance(loss, LossType):
        o = Loss(loss.name.lower())
        o.type = loss
        return o
    if isinstance(loss, str) and loss in _BY_NAME:
        return _BY_NAME[loss]()
    raise ValueError(f"unsupported loss {loss!r}")
