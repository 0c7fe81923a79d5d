"""Keras functional CIFAR-10 CNN with two concatenated conv towers
(reference: examples/python/keras/func_cifar10_cnn_concat.py)."""
from _common import ModelAccuracy, cifar10, epochs, verify

import flexflow.keras.optimizers
from flexflow.keras.layers import Activation, Concatenate, Conv2D, Dense, Flatten, Input, MaxPooling2D
from flexflow.keras.models import Model


def tower(t):
    t = Conv2D(filters=32, kernel_size=(3, 3), strides=(1, 1), padding=(1, 1), activation="relu")(t)
    return Conv2D(filters=32, kernel_size=(3, 3), strides=(1, 1), padding=(1, 1), activation="relu")(t)


def top_level_task():
    x_train, y_train = cifar10()
    inp = Input(shape=(3, 32, 32), dtype="float32")
    t = Concatenate(axis=1)([tower(inp), tower(inp)])
    t = MaxPooling2D(pool_size=(2, 2), strides=(2, 2), padding="valid")(t)
    t = Conv2D(filters=64, kernel_size=(3, 3), strides=(1, 1), padding=(1, 1), activation="relu")(t)
    t = Conv2D(filters=64, kernel_size=(3, 3), strides=(1, 1), padding=(1, 1), activation="relu")(t)
    t = MaxPooling2D(pool_size=(2, 2), strides=(2, 2), padding="valid")(t)
    t = Flatten()(t)
    t = Dense(512, activation="relu")(t)
    t = Dense(10)(t)
    out = Activation("softmax")(t)
    model = Model(inp, out)
    model.compile(optimizer=flexflow.keras.optimizers.SGD(learning_rate=0.01), loss="sparse_categorical_crossentropy",
                  metrics=["accuracy", "sparse_categorical_crossentropy"])
    print(model.summary())
    model.fit(x_train, y_train, epochs=epochs(80), callbacks=verify(ModelAccuracy.CIFAR10_CNN))


if __name__ == "__main__":
    print("Functional API, cifar10 cnn concat")
    top_level_task()
