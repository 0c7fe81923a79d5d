"""Keras optimizers (reference: python/flexflow/keras/optimizers.py)."""
from __future__ import annotations

from ...core import AdamOptimizer, SGDOptimizer


class Optimizer:
    def __init__(self):
        self._ffhandle = None

    @property
    def ffhandle(self):
        return self._ffhandle

    def create_ffhandle(self, ffmodel):
        raise NotImplementedError

    # kept for the older frontend spelling
    def ff(self, ffmodel):
        return self.create_ffhandle(ffmodel)

    def set_learning_rate(self, learning_rate):
        self.lr = float(learning_rate)
        if self._ffhandle is not None:
            self._ffhandle.set_learning_rate(self.lr)


class SGD(Optimizer):
    def __init__(self, learning_rate=0.01, momentum=0.0, nesterov=False, decay=0.0, lr=None, **kw):
        super().__init__()
        self.lr = float(lr if lr is not None else learning_rate)
        self.momentum, self.nesterov, self.decay = momentum, nesterov, decay

    def create_ffhandle(self, ffmodel):
        self._ffhandle = SGDOptimizer(ffmodel, lr=self.lr, momentum=self.momentum, nesterov=self.nesterov,
                                      weight_decay=self.decay)
        return self._ffhandle


class Adam(Optimizer):
    def __init__(self, learning_rate=0.001, beta_1=0.9, beta_2=0.999, epsilon=1e-8, decay=0.0, lr=None, **kw):
        super().__init__()
        self.lr = float(lr if lr is not None else learning_rate)
        self.beta_1, self.beta_2, self.epsilon, self.decay = beta_1, beta_2, epsilon, decay

    def create_ffhandle(self, ffmodel):
        self._ffhandle = AdamOptimizer(ffmodel, alpha=self.lr, beta1=self.beta_1, beta2=self.beta_2,
                                       epsilon=self.epsilon, weight_decay=self.decay)
        return self._ffhandle


def get(opt) -> Optimizer:
    if isinstance(opt, Optimizer):
        return opt
    if isinstance(opt, str) and opt.lower() in ("sgd", "adam"):
        return SGD() if opt.lower() == "sgd" else Adam()
    raise ValueError(f"unsupported optimizer {opt!r}")
