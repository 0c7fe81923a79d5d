"""Operator implementations (registered on import)."""
from . import attention, conv, dense, elementwise, embedding, moe, norm, shape  # noqa: F401
from .base import get_impl, registered_ops  # noqa: F401
