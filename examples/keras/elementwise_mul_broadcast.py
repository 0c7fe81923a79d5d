"""Multiply with numpy-style broadcasting (reference:
examples/python/keras/elementwise_mul_broadcast.py)."""
import numpy as np
import _common  # noqa: F401

import flexflow.keras.models
import flexflow.keras.optimizers
from flexflow.keras.layers import Dense, Input, Multiply, Reshape


def run(d0, s0, s1, swap=False):
    in0 = Input(shape=(32,), dtype="float32")
    in1 = Input(shape=(10,), dtype="float32")
    x0 = Reshape(s0)(Dense(d0, activation="relu")(in0))
    x1 = Reshape(s1)(Dense(10, activation="relu")(in1))
    m = Multiply()([x1, x0] if swap else [x0, x1])    # broadcast to (B, 10, 2)
    out = Dense(1)(Reshape((20,))(m))
    model = flexflow.keras.models.Model([in0, in1], out)
    model.compile(optimizer=flexflow.keras.optimizers.Adam(learning_rate=0.001), loss="mean_squared_error",
                  metrics=["mean_squared_error"])
    print(model.summary())
    model.fit(x=[np.random.randn(300, 32).astype(np.float32), np.random.randn(300, 10).astype(np.float32)],
              y=np.random.randn(300, 1).astype(np.float32), epochs=2)


if __name__ == "__main__":
    run(20, (10, 2), (10, 1), swap=True)   # broadcast1
    run(20, (10, 2), (10, 1))              # broadcast2
    run(2, (1, 2), (10, 1))                # broadcast both operands
