"""Reshape round trip in a functional MNIST MLP (reference: examples/python/keras/reshape.py)."""
from _common import ModelAccuracy, epochs, mnist_flat, verify

import flexflow.keras.optimizers
from flexflow.keras import metrics
from flexflow.keras.layers import Activation, Dense, Input, Reshape
from flexflow.keras.models import Model


def top_level_task():
    x_train, y_train = mnist_flat()
    inp = Input(shape=(784,))
    t = Reshape(target_shape=(28, 28))(inp)
    t = Reshape(target_shape=(784,))(t)
    t = Dense(512, input_shape=(784,), activation="relu")(t)
    t = Dense(512, activation="relu")(t)
    t = Dense(10)(t)
    model = Model(inp, Activation("softmax")(t))
    model.compile(optimizer=flexflow.keras.optimizers.SGD(learning_rate=0.01), loss="sparse_categorical_crossentropy",
                  metrics=["accuracy", metrics.SparseCategoricalCrossentropy()])
    print(model.summary())
    model.fit(x_train, y_train, epochs=epochs(10), callbacks=verify(ModelAccuracy.MNIST_MLP))


if __name__ == "__main__":
    print("Functional API, mnist mlp reshape")
    top_level_task()
