"""Keras functional CNN on CIFAR-10 (reference: examples/python/keras/func_cifar10_cnn.py)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from flexflow.keras.datasets import cifar10  # noqa: E402
from flexflow.keras.layers import Conv2D, Dense, Flatten, Input, MaxPooling2D  # noqa: E402
from flexflow.keras.models import Model  # noqa: E402
from flexflow.keras.optimizers import SGD  # noqa: E402


def top_level_task():
    n = int(os.environ.get("FF_EXAMPLE_SAMPLES", 50000))
    (x_train, y_train), _ = cifar10.load_data(num_samples=n)
    x_train = x_train.astype("float32") / 255
    y_train = y_train.astype("int32").reshape(-1, 1)
    inp = Input(shape=(3, 32, 32), dtype="float32")
    t = Conv2D(filters=32, input_shape=(3, 32, 32), kernel_size=(3, 3), strides=(1, 1), padding=(1, 1),
               activation="relu")(inp)
    t = MaxPooling2D(pool_size=(2, 2), strides=(2, 2), padding="valid")(t)
    t = Conv2D(filters=64, kernel_size=(3, 3), strides=(1, 1), padding=(1, 1), activation="relu")(t)
    t = MaxPooling2D(pool_size=(2, 2), strides=(2, 2), padding="valid")(t)
    t = Flatten()(t)
    t = Dense(256, activation="relu")(t)
    out = Dense(10, activation="softmax")(t)
    model = Model(inp, out)
    model.compile(optimizer=SGD(learning_rate=0.01), loss="sparse_categorical_crossentropy", metrics=["accuracy"])
    model.fit(x_train, y_train, epochs=1, batch_size=64)


if __name__ == "__main__":
    top_level_task()
