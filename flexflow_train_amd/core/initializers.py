"""Initializer objects of the user API (flexflow_cffi.py:2330-2390); they
serialise to the JSON initializer attrs stored on WEIGHT layers
(lib/pcg/include/pcg/initializers/*)."""
import json


class Initializer:
    def to_json(self) -> str:
        return json.dumps(self.attrs())


class GlorotUniformInitializer(Initializer):
    def __init__(self, seed=0):
        self.seed = seed

    def attrs(self):
        return {"type": "glorot_uniform", "seed": self.seed}


class GlorotNormalInitializer(GlorotUniformInitializer):
    def attrs(self):
        return {"type": "glorot_normal", "seed": self.seed}


class ZeroInitializer(Initializer):
    def attrs(self):
        return {"type": "zero"}


class ConstantInitializer(Initializer):
    def __init__(self, value=0.0):
        self.value = value

    def attrs(self):
        return {"type": "constant", "value": float(self.value)}


class UniformInitializer(Initializer):
    def __init__(self, seed=0, minv=-0.05, maxv=0.05):
        self.seed, self.minv, self.maxv = seed, minv, maxv

    def attrs(self):
        return {"type": "uniform", "seed": self.seed, "min": float(self.minv), "max": float(self.maxv)}


class NormInitializer(Initializer):
    def __init__(self, seed=0, mean=0.0, stddev=1.0):
        self.seed, self.mean, self.stddev = seed, mean, stddev

    def attrs(self):
        return {"type": "normal", "seed": self.seed, "mean": float(self.mean), "stddev": float(self.stddev)}


class TruncatedNormalInitializer(Initializer):
    def __init__(self, seed=0, mean=0.0, stddev=1.0, min_cutoff=None, max_cutoff=None):
        self.seed, self.mean, self.stddev = seed, mean, stddev
        self.lo = mean - 2 * stddev if min_cutoff is None else min_cutoff
        self.hi = mean + 2 * stddev if max_cutoff is None else max_cutoff

    def attrs(self):
        return {"type": "truncated_normal", "seed": self.seed, "mean": float(self.mean),
                "stddev": float(self.stddev), "min_cutoff": float(self.lo), "max_cutoff": float(self.hi)}
