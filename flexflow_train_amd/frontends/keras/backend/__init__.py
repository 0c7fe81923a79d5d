"""Keras backend functions (reference: python/flexflow/keras/backend/)."""
from . import internal  # noqa: F401
from .internal import batch_dot, cos, exp, gather, pow, rsqrt, sin, sum  # noqa: F401,A004

_BACKEND = "flexflow"


def backend():
    """Name of the backend (always the framework's own)."""
    return _BACKEND


def image_data_format():
    return "channels_first"
