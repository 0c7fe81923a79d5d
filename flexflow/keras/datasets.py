from flexflow_train_amd.frontends.keras import datasets as _d

mnist = _d.mnist
cifar10 = _d.cifar10
reuters = _d.reuters
