"""CIFAR-10 CNN whose two input towers are Sequential models joined by a
Concatenate on their outputs (reference:
examples/python/keras/func_cifar10_cnn_concat_seq_model.py)."""
from _common import ModelAccuracy, cifar10, epochs, verify

import flexflow.keras.optimizers
from flexflow.keras.layers import Activation, Concatenate, Conv2D, Dense, Flatten, MaxPooling2D
from flexflow.keras.models import Model, Sequential


def tower(i):
    m = Sequential()
    m.add(Conv2D(filters=32, input_shape=(3, 32, 32), kernel_size=(3, 3), strides=(1, 1), padding=(1, 1),
                 activation="relu", name=f"conv2d_0_{i}"))
    m.add(Conv2D(filters=32, kernel_size=(3, 3), strides=(1, 1), padding=(1, 1), activation="relu",
                 name=f"conv2d_1_{i}"))
    return m


def top_level_task():
    x_train, y_train = cifar10()
    model1, model2 = tower(0), tower(1)
    print(model1.summary())
    t = Concatenate(axis=1)([model1.output, model2.output])
    t = MaxPooling2D(pool_size=(2, 2), strides=(2, 2), padding="valid")(t)
    t = Conv2D(filters=64, kernel_size=(3, 3), strides=(1, 1), padding=(1, 1), activation="relu", name="conv2d_0_4")(t)
    t = Conv2D(filters=64, kernel_size=(3, 3), strides=(1, 1), padding=(1, 1), activation="relu")(t)
    t = MaxPooling2D(pool_size=(2, 2), strides=(2, 2), padding="valid")(t)
    t = Flatten()(t)
    t = Dense(512, activation="relu")(t)
    t = Dense(10)(t)
    out = Activation("softmax")(t)
    model = Model([model1.input[0], model2.input[0]], out)
    model.compile(optimizer=flexflow.keras.optimizers.SGD(learning_rate=0.01), loss="sparse_categorical_crossentropy",
                  metrics=["accuracy", "sparse_categorical_crossentropy"])
    print(model.summary())
    model.fit([x_train, x_train], y_train, epochs=epochs(80), callbacks=verify(ModelAccuracy.CIFAR10_CNN))


if __name__ == "__main__":
    print("Functional API, cifar10 cnn concat sequential model")
    top_level_task()
