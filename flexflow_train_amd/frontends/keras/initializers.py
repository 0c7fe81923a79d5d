"""Keras initializers (reference: python/flexflow/keras/initializers.py);
each wraps one of the core initializer objects (``ffhandle``)."""
from __future__ import annotations

import random

from ...core import initializers as _ci


class Initializer:
    def __init__(self):
        self._ffhandle = None

    @property
    def ffhandle(self):
        return self._ffhandle


class DefaultInitializer(Initializer):
    """The operator's own default (Glorot-uniform kernels, zero biases)."""


class Zeros(Initializer):
    def __init__(self):
        super().__init__()
        self._ffhandle = _ci.ZeroInitializer()


class Ones(Initializer):
    def __init__(self):
        super().__init__()
        self._ffhandle = _ci.ConstantInitializer(1.0)


class Constant(Initializer):
    def __init__(self, value=0.0):
        super().__init__()
        self.value = value
        self._ffhandle = _ci.ConstantInitializer(value)


class GlorotUniform(Initializer):
    def __init__(self, seed=None):
        super().__init__()
        self.seed = random.randint(0, 1024) if seed is None else seed
        self._ffhandle = _ci.GlorotUniformInitializer(self.seed)


class GlorotNormal(Initializer):
    def __init__(self, seed=None):
        super().__init__()
        self.seed = random.randint(0, 1024) if seed is None else seed
        self._ffhandle = _ci.GlorotNormalInitializer(self.seed)


class RandomUniform(Initializer):
    def __init__(self, minval=-0.05, maxval=0.05, seed=None):
        super().__init__()
        self.minval, self.maxval = minval, maxval
        self.seed = random.randint(0, 1024) if seed is None else seed
        self._ffhandle = _ci.UniformInitializer(self.seed, minval, maxval)


class RandomNormal(Initializer):
    """Normal(mean, stddev) (the reference builds a uniform initializer here,
    keras/initializers.py:54; this one samples the normal it is named for)."""

    def __init__(self, mean=0.0, stddev=0.05, seed=None):
        super().__init__()
        self.mean, self.stddev = mean, stddev
        self.seed = random.randint(0, 1024) if seed is None else seed
        self._ffhandle = _ci.NormInitializer(self.seed, mean, stddev)


class TruncatedNormal(Initializer):
    def __init__(self, mean=0.0, stddev=0.05, seed=None):
        super().__init__()
        self.seed = random.randint(0, 1024) if seed is None else seed
        self._ffhandle = _ci.TruncatedNormalInitializer(self.seed, mean, stddev)


_BY_NAME = {"glorot_uniform": GlorotUniform, "glorot_normal": GlorotNormal, "zeros": Zeros, "zero": Zeros,
            "ones": Ones, "uniform": RandomUniform, "random_uniform": RandomUniform, "normal": RandomNormal,
            "random_normal": RandomNormal, "truncated_normal": TruncatedNormal}


def get(init):
    """str | Initializer | core initializer | None -> Initializer."""
    if init is None:
        return DefaultInitializer()
    if isinstance(init, Initializer):
        return init
    if isinstance(init, _ci.Initializer):
        w = Initializer()
        w._ffhandle = init
        return w
    if isinstance(init, str):
        if init.lower() not in _BY_NAME:
            raise ValueError(f"unknown initializer {init!r}")
        return _BY_NAME[init.lower()]()
    raise TypeError(f"not an initializer: {init!r}")


def handle(init):
    return get(init).ffhandle
