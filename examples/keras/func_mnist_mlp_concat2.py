"""Keras functional MLP built from nested sub-models and extra inputs,
concatenated (reference: examples/python/keras/func_mnist_mlp_concat2.py)."""
from _common import ModelAccuracy, epochs, mnist_flat, verify

import flexflow.keras.optimizers
from flexflow.keras.layers import Activation, Concatenate, Dense, Input
from flexflow.keras.models import Model


def branch(idx):
    i = Input(shape=(784,))
    t = Dense(512, activation="relu", name=f"dense{idx}")(i)
    return Model(i, Dense(512, activation="relu", name=f"dense{idx}{idx}")(t))


def top_level_task():
    x_train, y_train = mnist_flat()
    # a sub-model that itself applies a nested model
    i11, i12 = Input(shape=(784,)), Input(shape=(784,))
    model11 = Model(i11, Dense(512, activation="relu", name="dense1")(i11))
    model1 = Model(i12, Dense(512, activation="relu", name="dense12")(model11(i12)))
    model2, model3 = branch(2), branch(3)
    inp = Input(shape=(784,))
    t00 = Input(shape=(784,), name="input_00")
    t01 = Input(shape=(784,), name="input_01")
    t = Concatenate(axis=1)([t00, t01, model1(inp), model2(inp), model3(inp)])
    t = Dense(10)(t)
    out = Activation("softmax")(t)
    model = Model([t00, t01, inp], out)
    model.compile(optimizer=flexflow.keras.optimizers.SGD(learning_rate=0.01), loss="sparse_categorical_crossentropy",
                  metrics=["accuracy", "sparse_categorical_crossentropy"])
    print(model.summary())
    model.fit([x_train, x_train, x_train], y_train, epochs=epochs(10), callbacks=verify(ModelAccuracy.MNIST_MLP))


if __name__ == "__main__":
    print("Functional API, mnist mlp concat with input")
    top_level_task()
