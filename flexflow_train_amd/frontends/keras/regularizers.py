"""Keras regularizers (reference: python/flexflow/keras/regularizers.py).
Dense(kernel_regularizer=L2(l)) adds l * W (L1: l * sign(W)) to the kernel
gradient in the Linear backward (runtime/executor.py _add_regularizer_grad)."""
from __future__ import annotations

from ...core import RegularizerMode


class Regularizer:
    def __init__(self):
        self.type = RegularizerMode.REG_MODE_NONE
        self._lambda = 0.0


class L1(Regularizer):
    def __init__(self, l1=0.01):
        super().__init__()
        self.type = RegularizerMode.REG_MODE_L1
        self._lambda = float(l1)


class L2(Regularizer):
    def __init__(self, l2=0.01):
        super().__init__()
        self.type = RegularizerMode.REG_MODE_L2
        self._lambda = float(l2)


l1 = L1
l2 = L2
