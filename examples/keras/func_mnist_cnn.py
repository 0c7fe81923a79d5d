"""Keras functional CNN on MNIST (reference: examples/python/keras/func_mnist_cnn.py)."""
from _common import ModelAccuracy, epochs, mnist_images, verify

import flexflow.keras.optimizers
from flexflow.keras import losses, metrics
from flexflow.keras.layers import Activation, Conv2D, Dense, Flatten, Input, MaxPooling2D
from flexflow.keras.models import Model


def top_level_task():
    x_train, y_train = mnist_images()
    inp = Input(shape=(1, 28, 28), dtype="float32")
    t = Conv2D(filters=32, input_shape=(1, 28, 28), kernel_size=(3, 3), strides=(1, 1), padding=(1, 1),
               activation="relu")(inp)
    t = Conv2D(filters=64, kernel_size=(3, 3), strides=(1, 1), padding=(1, 1), activation="relu")(t)
    t = MaxPooling2D(pool_size=(2, 2), strides=(2, 2), padding="valid")(t)
    t = Flatten()(t)
    t = Dense(128, activation="relu")(t)
    t = Dense(10)(t)
    out = Activation("softmax")(t)
    model = Model(inp, out)
    model.compile(optimizer=flexflow.keras.optimizers.SGD(learning_rate=0.01),
                  loss=losses.SparseCategoricalCrossentropy(),
                  metrics=[metrics.Accuracy(), metrics.SparseCategoricalCrossentropy()])
    print(model.summary())
    model.fit(x_train, y_train, epochs=epochs(5), callbacks=verify(ModelAccuracy.MNIST_CNN))


if __name__ == "__main__":
    print("Functional API, mnist cnn")
    top_level_task()
