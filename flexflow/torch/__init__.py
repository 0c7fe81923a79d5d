"""flexflow.torch (reference: python/flexflow/torch)."""
from flexflow_train_amd.frontends.torch_fx import (PyTorchModel, copy_weights, string_to_ff)  # noqa: F401
from flexflow_train_amd.frontends.torch_compile import CompiledModel, backend, compile  # noqa: F401,E402
