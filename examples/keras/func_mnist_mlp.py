"""Keras functional MLP on MNIST (reference: examples/python/keras/func_mnist_mlp.py)."""
from _common import ModelAccuracy, epochs, mnist_flat, verify

import flexflow.keras.optimizers
from flexflow.keras import metrics
from flexflow.keras.layers import Activation, Dense, Input
from flexflow.keras.models import Model


def top_level_task():
    x_train, y_train = mnist_flat()
    inp = Input(shape=(784,))
    t = Dense(512, input_shape=(784,), activation="relu")(inp)
    t = Dense(512, activation="relu")(t)
    t = Dense(10)(t)
    out = Activation("softmax")(t)
    model = Model(inp, out)
    model.compile(optimizer=flexflow.keras.optimizers.SGD(learning_rate=0.01), loss="sparse_categorical_crossentropy",
                  metrics=["accuracy", metrics.SparseCategoricalCrossentropy()])
    print(model.summary())
    model.fit(x_train, y_train, epochs=epochs(10), callbacks=verify(ModelAccuracy.MNIST_MLP))


if __name__ == "__main__":
    print("Functional API, mnist mlp")
    top_level_task()
