"""Keras datasets (reference: python/flexflow/keras/datasets/)."""
from . import cifar10, mnist, reuters  # noqa: F401
