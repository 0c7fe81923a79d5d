"""Keras functional MLP with concatenated branches on MNIST (reference:
examples/python/keras/func_mnist_mlp_concat.py)."""
from _common import ModelAccuracy, epochs, mnist_flat, verify

import flexflow.keras.optimizers
from flexflow.keras.layers import Activation, Concatenate, Dense, Input
from flexflow.keras.models import Model


def top_level_task():
    x_train, y_train = mnist_flat()
    inp = Input(shape=(784,))
    branches = []
    for i in range(4):
        t = Dense(512, activation="relu", name=f"dense{i}")(inp)
        branches.append(Dense(512, activation="relu", name=f"dense{i}{i}")(t))
    t = Concatenate(axis=1)(branches)
    t = Dense(10)(t)
    out = Activation("softmax")(t)
    model = Model(inp, out)
    model.compile(optimizer=flexflow.keras.optimizers.SGD(learning_rate=0.01), loss="sparse_categorical_crossentropy",
                  metrics=["accuracy", "sparse_categorical_crossentropy"])
    print(model.summary())
    model.fit(x_train, y_train, epochs=epochs(10), callbacks=verify(ModelAccuracy.MNIST_MLP))


if __name__ == "__main__":
    print("Functional API, mnist mlp concat")
    top_level_task()
