"""CIFAR-10 CNN built by applying two keras Models in sequence to a new
input (reference: examples/python/keras/func_cifar10_cnn_nested.py)."""
from _common import ModelAccuracy, cifar10, epochs, verify

import flexflow.keras.optimizers
from flexflow.keras.layers import Activation, Conv2D, Dense, Flatten, Input, MaxPooling2D
from flexflow.keras.models import Model


def top_level_task():
    x_train, y_train = cifar10()
    i1 = Input(shape=(3, 32, 32), dtype="float32")
    t = Conv2D(filters=32, kernel_size=(3, 3), strides=(1, 1), padding=(1, 1), activation="relu")(i1)
    t = Conv2D(filters=32, kernel_size=(3, 3), strides=(1, 1), padding=(1, 1), activation="relu")(t)
    model1 = Model(i1, MaxPooling2D(pool_size=(2, 2), strides=(2, 2), padding="valid")(t))
    i2 = Input(shape=(32, 16, 16), dtype="float32")
    t = Conv2D(filters=64, kernel_size=(3, 3), strides=(1, 1), padding=(1, 1), activation="relu")(i2)
    t = Conv2D(filters=64, kernel_size=(3, 3), strides=(1, 1), padding=(1, 1), activation="relu")(t)
    t = MaxPooling2D(pool_size=(2, 2), strides=(2, 2), padding="valid")(t)
    t = Flatten()(t)
    t = Dense(512, activation="relu")(t)
    t = Dense(10)(t)
    model2 = Model(i2, Activation("softmax")(t))
    i3 = Input(shape=(3, 32, 32), dtype="float32")
    model = Model(i3, model2(model1(i3)))
    model.compile(optimizer=flexflow.keras.optimizers.SGD(learning_rate=0.01), loss="sparse_categorical_crossentropy",
                  metrics=["accuracy", "sparse_categorical_crossentropy"])
    print(model.summary())
    model.fit(x_train, y_train, epochs=epochs(80), callbacks=verify(ModelAccuracy.CIFAR10_CNN))


if __name__ == "__main__":
    print("Functional API, cifar10 cnn nested")
    top_level_task()
