"""Keras preprocessing (reference: python/flexflow/keras/preprocessing/)."""
from . import sequence, text  # noqa: F401
