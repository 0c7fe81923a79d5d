"""Keras functional CNN with two concatenated conv branches on MNIST
(reference: examples/python/keras/func_mnist_cnn_concat.py)."""
from _common import ModelAccuracy, epochs, mnist_images, verify

import flexflow.keras.optimizers
from flexflow.keras.layers import Activation, Conv2D, Dense, Flatten, Input, MaxPooling2D, concatenate
from flexflow.keras.models import Model


def top_level_task():
    x_train, y_train = mnist_images()
    inp = Input(shape=(1, 28, 28), dtype="float32")
    a = Conv2D(filters=32, kernel_size=(3, 3), strides=(1, 1), padding=(1, 1), activation="relu")(inp)
    b = Conv2D(filters=32, kernel_size=(3, 3), strides=(1, 1), padding=(1, 1), activation="relu")(inp)
    t = concatenate([a, b])
    t = Conv2D(filters=64, kernel_size=(3, 3), strides=(1, 1), padding=(1, 1), activation="relu")(t)
    t = MaxPooling2D(pool_size=(2, 2), strides=(2, 2), padding="valid")(t)
    t = Flatten()(t)
    t = Dense(128, activation="relu")(t)
    t = Dense(10)(t)
    out = Activation("softmax")(t)
    model = Model(inp, out)
    model.compile(optimizer=flexflow.keras.optimizers.SGD(learning_rate=0.01), loss="sparse_categorical_crossentropy",
                  metrics=["accuracy", "sparse_categorical_crossentropy"])
    print(model.summary())
    model.fit(x_train, y_train, epochs=epochs(5), callbacks=verify(ModelAccuracy.MNIST_CNN))


if __name__ == "__main__":
    print("Functional API, mnist cnn concat")
    top_level_task()
