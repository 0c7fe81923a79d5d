"""flexflow.config (reference: python/flexflow/config.py)."""
from flexflow_train_amd.core.config import flexflow_python_binding, flexflow_python_interpreter  # noqa: F401


def flexflow_init_import() -> bool:
    return True
