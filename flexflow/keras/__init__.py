"""flexflow.keras (reference: python/flexflow/keras/**)."""
from flexflow_train_amd.frontends.keras import Input, Model, Sequential  # noqa: F401

from . import callbacks, datasets, layers, models, optimizers  # noqa: F401,E402
