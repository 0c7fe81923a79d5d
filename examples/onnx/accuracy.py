"""Accuracy targets (percent) of the keras examples' checks (reference:
examples/python/keras/accuracy.py)."""
from enum import Enum


class ModelAccuracy(Enum):
    MNIST_MLP = 90
    MNIST_CNN = 90
    REUTERS_MLP = 90
    CIFAR10_CNN = 90
    CIFAR10_ALEXNET = 90
