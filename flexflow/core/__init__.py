"""flexflow.core (reference: python/flexflow/core/flexflow_cffi.py)."""
from flexflow_train_amd.core import *  # noqa: F401,F403
from flexflow_train_amd.core import (AdamOptimizer, FFConfig, FFModel, SGDOptimizer,  # noqa: F401
                                     SingleDataLoader)
from flexflow_train_amd.core.initializers import *  # noqa: F401,F403


def init_flexflow_runtime(configs=None):
    """No separate runtime to start: one process per GPU (torchrun)."""
    return None
