"""keras backend sum over one / several axes, with and without keepdims
(reference: examples/python/keras/reduce_sum.py)."""
import numpy as np
import _common  # noqa: F401

import flexflow.keras.backend
import flexflow.keras.models
import flexflow.keras.optimizers
from flexflow.keras.layers import Dense, Input, Reshape


def run(axis, keepdims, y_shape):
    in0 = Input(shape=(32,), dtype="float32")
    nx0 = Reshape((10, 2))(Dense(20, activation="relu")(in0))
    out = flexflow.keras.backend.sum(nx0, axis=axis, keepdims=keepdims)
    model = flexflow.keras.models.Model(in0, out)
    model.compile(optimizer=flexflow.keras.optimizers.Adam(learning_rate=0.001), loss="mean_squared_error",
                  metrics=["mean_squared_error"])
    print(model.summary())
    model.fit(x=np.random.randn(300, 32).astype(np.float32), y=np.random.randn(300, *y_shape).astype(np.float32),
              epochs=2)


if __name__ == "__main__":
    run(1, False, (2,))          # (B, 2)
    run([1, 2], False, ())       # (B,)
    run([1, 2], True, (1, 1))    # (B, 1, 1)
