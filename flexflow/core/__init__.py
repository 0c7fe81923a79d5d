"""flexflow.core (reference: python/flexflow/core/flexflow_cffi.py)."""
from flexflow_train_amd.core import *  # noqa: F401,F403
from flexflow_train_amd.core import (AdamOptimizer, FFConfig, FFModel, SGDOptimizer,  # noqa: F401
                                     SingleDataLoader)
from flexflow_train_amd.core.initializers import *  # noqa: F401,F403


def init_flexflow_runtime(configs=None):
    """No separate runtime to start: one process per GPU (torchrun)."""
    return None


def DLRMConfig(argv=None):  # noqa: N802
    """DLRM settings from the command line (reference flexflow_cffi.py
    DLRMConfig, parsed by examples/cpp/DLRM/dlrm.cc)."""
    from flexflow_train_amd.models.recsys import DLRMConfig as _D
    return _D.from_args(argv)

