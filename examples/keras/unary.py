"""Add / subtract merges plus the unary backend functions (reference:
examples/python/keras/unary.py)."""
import numpy as np
import _common  # noqa: F401

import flexflow.keras.optimizers
from flexflow.keras import backend as K
from flexflow.keras.layers import Add, Dense, Input, subtract
from flexflow.keras.models import Model


def merge_test(merge):
    in1 = Input(shape=(16,), dtype="float32")
    in2 = Input(shape=(32,), dtype="float32")
    x1 = Dense(8, activation="relu")(in1)
    x2 = Dense(8, activation="relu")(in2)
    out = Dense(4)(merge([x1, x2]))
    model = Model([in1, in2], out)
    model.compile(optimizer=flexflow.keras.optimizers.SGD(learning_rate=0.01), loss="sparse_categorical_crossentropy",
                  metrics=["accuracy", "sparse_categorical_crossentropy"])
    print(model.summary())
    model.ffmodel.init_layers()


def unary_test():
    inp = Input(shape=(16,), dtype="float32")
    x = Dense(8, activation="relu")(inp)
    y = K.exp(K.sin(x)) + K.cos(x) + K.pow(x, 2)
    model = Model(inp, Dense(1)(y))
    model.compile(optimizer=flexflow.keras.optimizers.Adam(learning_rate=0.001), loss="mean_squared_error",
                  metrics=["mean_squared_error"])
    model.fit(np.random.randn(300, 16).astype(np.float32), np.random.randn(300, 1).astype(np.float32), epochs=1)


if __name__ == "__main__":
    merge_test(lambda xs: Add()(xs))
    merge_test(subtract)
    unary_test()
