"""LearningRateScheduler + accuracy callbacks on a CIFAR-10 CNN (reference:
examples/python/keras/callback.py)."""
from _common import ModelAccuracy, cifar10, epochs, verify

import flexflow.keras.optimizers
from flexflow.keras import backend as K
from flexflow.keras.callbacks import Callback, LearningRateScheduler
from flexflow.keras.layers import Activation, Conv2D, Dense, Flatten, Input, MaxPooling2D
from flexflow.keras.models import Model


def lr_scheduler(epoch):
    return 0.01 if epoch == 0 else 0.02


class BatchCounter(Callback):
    """Per-batch hooks (on_batch_begin / on_batch_end)."""

    def __init__(self):
        super().__init__()
        self.batches = 0

    def on_batch_end(self, batch, logs=None):
        self.batches += 1

    def on_train_end(self, logs=None):
        print(f"trained {self.batches} batches")


def top_level_task():
    print(K.backend())
    x_train, y_train = cifar10()
    inp = Input(shape=(3, 32, 32), dtype="float32")
    t = Conv2D(filters=32, input_shape=(3, 32, 32), kernel_size=(3, 3), strides=(1, 1), padding=(1, 1),
               activation="relu")(inp)
    t = Conv2D(filters=32, kernel_size=(3, 3), strides=(1, 1), padding=(1, 1), activation="relu")(t)
    t = MaxPooling2D(pool_size=(2, 2), strides=(2, 2), padding="valid")(t)
    t = Flatten()(t)
    t = Dense(512, activation="relu")(t)
    t = Dense(10)(t)
    model = Model(inp, Activation("softmax")(t))
    model.compile(optimizer=flexflow.keras.optimizers.SGD(learning_rate=0.02), loss="sparse_categorical_crossentropy",
                  metrics=["accuracy", "sparse_categorical_crossentropy"])
    print(model.summary())
    counter = BatchCounter()
    model.fit(x_train, y_train, epochs=epochs(80),
              callbacks=[LearningRateScheduler(lr_scheduler), counter] + verify(ModelAccuracy.CIFAR10_CNN))
    assert counter.batches > 0


if __name__ == "__main__":
    print("Functional API, cifar10 cnn callback")
    top_level_task()
