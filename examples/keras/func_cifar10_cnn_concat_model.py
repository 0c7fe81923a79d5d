"""CIFAR-10 CNN whose two input towers are separate keras Models joined by
a Concatenate (reference: examples/python/keras/func_cifar10_cnn_concat_model.py)."""
from _common import ModelAccuracy, cifar10, epochs, verify

import flexflow.keras.optimizers
from flexflow.keras.layers import Activation, Concatenate, Conv2D, Dense, Flatten, Input, MaxPooling2D
from flexflow.keras.models import Model


def cifar_cnn_sub(input_tensor, postfix):
    t = Conv2D(filters=32, input_shape=(3, 32, 32), kernel_size=(3, 3), strides=(1, 1), padding=(1, 1),
               activation="relu", name=f"conv2d_0_{postfix}")(input_tensor)
    return Conv2D(filters=32, kernel_size=(3, 3), strides=(1, 1), padding=(1, 1), activation="relu",
                  name=f"conv2d_1_{postfix}")(t)


def top_level_task():
    x_train, y_train = cifar10()
    in1 = Input(shape=(3, 32, 32), dtype="float32", name="input1")
    in2 = Input(shape=(3, 32, 32), dtype="float32", name="input2")
    model1 = Model(in1, cifar_cnn_sub(in1, 1))
    model2 = Model(in2, cifar_cnn_sub(in2, 2))
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
    model = Model([in1, in2], out)
    model.compile(optimizer=flexflow.keras.optimizers.SGD(learning_rate=0.01), loss="sparse_categorical_crossentropy",
                  metrics=["accuracy", "sparse_categorical_crossentropy"])
    print(model.summary())
    model.fit([x_train, x_train], y_train, epochs=epochs(80), callbacks=verify(ModelAccuracy.CIFAR10_CNN))


if __name__ == "__main__":
    print("Functional API, cifar10 cnn concat model")
    top_level_task()
