"""flexflow.type (reference: python/flexflow/type.py:5-143)."""
from flexflow_train_amd.core.types import *  # noqa: F401,F403
