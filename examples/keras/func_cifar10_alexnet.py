"""Keras functional AlexNet on CIFAR-10 upsampled to 229x229 (reference:
examples/python/keras/func_cifar10_alexnet.py; nearest-neighbour resize in
numpy instead of PIL)."""
import numpy as np
from _common import ModelAccuracy, cifar10, epochs, verify

import flexflow.keras.optimizers
from flexflow.keras.layers import Activation, Conv2D, Dense, Flatten, Input, MaxPooling2D
from flexflow.keras.models import Model


def resize_nearest(x, size=229):
    idx = (np.arange(size) * x.shape[-1] / size).astype(np.int64)
    return x[:, :, idx][:, :, :, idx]


def top_level_task():
    x_train, y_train = cifar10()
    x_train = resize_nearest(x_train)
    inp = Input(shape=(3, 229, 229), dtype="float32")
    t = Conv2D(filters=64, input_shape=(3, 229, 229), kernel_size=(11, 11), strides=(4, 4), padding=(2, 2),
               activation="relu")(inp)
    t = MaxPooling2D(pool_size=(3, 3), strides=(2, 2), padding="valid")(t)
    t = Conv2D(filters=192, kernel_size=(5, 5), strides=(1, 1), padding=(2, 2), activation="relu")(t)
    t = MaxPooling2D(pool_size=(3, 3), strides=(2, 2), padding="valid")(t)
    t = Conv2D(filters=384, kernel_size=(3, 3), strides=(1, 1), padding=(1, 1), activation="relu")(t)
    t = Conv2D(filters=256, kernel_size=(3, 3), strides=(1, 1), padding=(1, 1), activation="relu")(t)
    t = Conv2D(filters=256, kernel_size=(3, 3), strides=(1, 1), padding=(1, 1), activation="relu")(t)
    t = MaxPooling2D(pool_size=(3, 3), strides=(2, 2), padding="valid")(t)
    t = Flatten()(t)
    t = Dense(4096, activation="relu")(t)
    t = Dense(4096, activation="relu")(t)
    t = Dense(10)(t)
    out = Activation("softmax")(t)
    model = Model(inp, out)
    model.compile(optimizer=flexflow.keras.optimizers.SGD(learning_rate=0.01), loss="sparse_categorical_crossentropy",
                  metrics=["accuracy", "sparse_categorical_crossentropy"])
    print(model.summary())
    model.fit(x_train, y_train, epochs=epochs(40), callbacks=verify(ModelAccuracy.CIFAR10_ALEXNET))


if __name__ == "__main__":
    print("Functional API, cifar10 alexnet")
    top_level_task()
