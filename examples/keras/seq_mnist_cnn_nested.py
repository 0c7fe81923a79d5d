"""A Sequential model made of a nested Sequential (conv stack) and a
functional Model (classifier head) (reference:
examples/python/keras/seq_mnist_cnn_nested.py)."""
from _common import ModelAccuracy, epochs, mnist_images, verify

import flexflow.keras.optimizers
from flexflow.keras.layers import Activation, Conv2D, Dense, Flatten, Input, MaxPooling2D
from flexflow.keras.models import Model, Sequential


def top_level_task():
    x_train, y_train = mnist_images()
    model1 = Sequential([Conv2D(filters=32, input_shape=(1, 28, 28), kernel_size=(3, 3), strides=(1, 1),
                                padding=(1, 1), activation="relu"),
                         Conv2D(filters=64, kernel_size=(3, 3), strides=(1, 1), padding=(1, 1), activation="relu"),
                         MaxPooling2D(pool_size=(2, 2), strides=(2, 2), padding="valid"),
                         Flatten()])
    inp = Input(shape=(12544,), dtype="float32")
    t = Dense(512, input_shape=(12544,), activation="relu")(inp)
    t = Dense(10)(t)
    model2 = Model(inp, Activation("softmax")(t))
    model = Sequential()
    model.add(model1)
    model.add(model2)
    model.compile(optimizer=flexflow.keras.optimizers.SGD(learning_rate=0.01), loss="sparse_categorical_crossentropy",
                  metrics=["accuracy", "sparse_categorical_crossentropy"])
    print(model.summary())
    model.fit(x_train, y_train, epochs=epochs(5), callbacks=verify(ModelAccuracy.MNIST_CNN))


if __name__ == "__main__":
    print("Sequential model, mnist cnn nested model")
    top_level_task()
