"""Teacher -> student weight transfer on a functional CIFAR-10 CNN
(reference: examples/python/keras/func_cifar10_cnn_net2net.py)."""
from _common import ModelAccuracy, cifar10, epochs, verify

import flexflow.keras.optimizers
from flexflow.keras.layers import Activation, Conv2D, Dense, Flatten, Input, MaxPooling2D
from flexflow.keras.models import Model


def build():
    inp = Input(shape=(3, 32, 32), dtype="float32")
    t = Conv2D(filters=32, kernel_size=(3, 3), strides=(1, 1), padding=(1, 1), activation="relu")(inp)
    t = Conv2D(filters=32, kernel_size=(3, 3), strides=(1, 1), padding=(1, 1), activation="relu")(t)
    t = MaxPooling2D(pool_size=(2, 2), strides=(2, 2), padding="valid")(t)
    t = Conv2D(filters=64, kernel_size=(3, 3), strides=(1, 1), padding=(1, 1), activation="relu")(t)
    t = Conv2D(filters=64, kernel_size=(3, 3), strides=(1, 1), padding=(1, 1), activation="relu")(t)
    t = MaxPooling2D(pool_size=(2, 2), strides=(2, 2), padding="valid")(t)
    t = Flatten()(t)
    t = Dense(512, activation="relu")(t)
    t = Dense(10)(t)
    model = Model(inp, Activation("softmax")(t))
    model.compile(optimizer=flexflow.keras.optimizers.SGD(learning_rate=0.01), loss="sparse_categorical_crossentropy",
                  metrics=["accuracy", "sparse_categorical_crossentropy"])
    return model


def top_level_task():
    x_train, y_train = cifar10()
    teacher = build()
    teacher.fit(x_train, y_train, epochs=epochs(40))
    student = build()
    for i in (0, 1, 3, 4, 7, 8):   # the conv and dense layers
        student.get_layer(index=i).set_weights(student.ffmodel, *teacher.get_layer(index=i).get_weights(teacher.ffmodel))
    student.fit(x_train, y_train, epochs=epochs(40), callbacks=verify(ModelAccuracy.CIFAR10_CNN))


if __name__ == "__main__":
    print("Functional API, cifar10 cnn teacher student")
    top_level_task()
