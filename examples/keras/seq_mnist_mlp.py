"""Keras Sequential MLP on MNIST (reference: examples/python/keras/seq_mnist_mlp.py)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from flexflow.keras.datasets import mnist  # noqa: E402
from flexflow.keras.layers import Activation, Dense  # noqa: E402
from flexflow.keras.models import Sequential  # noqa: E402
from flexflow.keras.optimizers import SGD  # noqa: E402


def top_level_task():
    n = int(os.environ.get("FF_EXAMPLE_SAMPLES", 60000))
    (x_train, y_train), _ = mnist.load_data(num_samples=n)
    x_train = x_train.reshape(len(x_train), 784).astype("float32") / 255
    y_train = y_train.astype("int32").reshape(-1, 1)
    model = Sequential()
    model.add(Dense(512, input_shape=(784,), activation="relu"))
    model.add(Dense(512, activation="relu"))
    model.add(Dense(10))
    model.add(Activation("softmax"))
    model.compile(optimizer=SGD(learning_rate=0.01), loss="sparse_categorical_crossentropy",
                  metrics=["accuracy", "sparse_categorical_crossentropy"])
    model.fit(x_train, y_train, epochs=1, batch_size=64)


if __name__ == "__main__":
    top_level_task()
