"""Keras utilities (reference: python/flexflow/keras/utils/)."""
from . import data_utils, np_utils  # noqa: F401
from .data_utils import get_file  # noqa: F401
from .np_utils import normalize, to_categorical  # noqa: F401
