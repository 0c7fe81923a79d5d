"""Keras-style frontend (reference: python/flexflow/keras/**): Sequential and
functional Models (nested models too), layers, backend functions, losses,
metrics, optimizers, initializers, regularizers, callbacks, datasets, utils
and preprocessing.  Models build an FFModel at compile time
(models.py)."""
from . import (backend, callbacks, datasets, initializers, layers, losses, metrics, models,  # noqa: F401
               optimizers, preprocessing, regularizers, utils)
from .callbacks import Callback, EpochVerifyMetrics, LearningRateScheduler, VerifyMetrics  # noqa: F401
from .layers import *  # noqa: F401,F403
from .models import BaseModel, Model, Sequential  # noqa: F401
from .optimizers import SGD, Adam  # noqa: F401
