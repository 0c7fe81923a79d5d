"""flexflow.core-compatible API: FFConfig, FFModel, optimizers, initializers,
data loaders and enums."""
from .config import FFConfig, NetConfig, flexflow_python_binding, flexflow_python_interpreter  # noqa: F401
from .initializers import (ConstantInitializer, GlorotNormalInitializer, GlorotUniformInitializer,  # noqa: F401
                           NormInitializer, TruncatedNormalInitializer, UniformInitializer, ZeroInitializer)
from .model import (AdamOptimizer, FFModel, Layer, Parameter, SGDOptimizer, SingleDataLoader,  # noqa: F401
                    Tensor)
from .types import *  # noqa: F401,F403
from .recompile import RecompileState  # noqa: F401
