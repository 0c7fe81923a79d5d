"""flexflow.keras (reference: python/flexflow/keras/**): the keras frontend
of flexflow_train_amd under the reference's module paths
(flexflow.keras.layers, .models, .backend.internal, .datasets.mnist, ...)."""
import importlib
import sys

from flexflow_train_amd.frontends import keras as _k
from flexflow_train_amd.frontends.keras import *  # noqa: F401,F403

_SUB = ["backend", "backend.internal", "callbacks", "datasets", "datasets.mnist", "datasets.cifar10",
        "datasets.reuters", "initializers", "layers", "losses", "metrics", "models", "optimizers", "preprocessing",
        "preprocessing.sequence", "preprocessing.text", "regularizers", "utils", "utils.np_utils",
        "utils.data_utils"]
for _n in _SUB:
    _m = importlib.import_module(f"{_k.__name__}.{_n}")
    sys.modules[f"{__name__}.{_n}"] = _m
    if "." not in _n:
        globals()[_n] = _m
