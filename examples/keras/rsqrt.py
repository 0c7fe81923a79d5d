"""rsqrt through keras backend.internal on a tensor sum (reference: examples/python/keras/rsqrt.py)."""
import numpy as np
import _common  # noqa: F401

import flexflow.keras.models
import flexflow.keras.optimizers
from flexflow.keras.backend.internal import rsqrt
from flexflow.keras.layers import Dense, Input


def test_rsqrt():
    in1 = Input(shape=(32,), dtype="float32")
    in2 = Input(shape=(20,), dtype="float32")
    x = Dense(20, activation="relu")(in1)
    out = rsqrt(x + in2)
    model = flexflow.keras.models.Model([in1, in2], out)
    model.compile(optimizer=flexflow.keras.optimizers.Adam(learning_rate=0.001), loss="mean_squared_error",
                  metrics=["mean_squared_error"])
    print(model.summary())
    model.fit(x=[np.random.randn(300, 32).astype(np.float32), np.ones((300, 20)).astype(np.float32)],
              y=np.random.randn(300, 20).astype(np.float32), epochs=2)


if __name__ == "__main__":
    test_rsqrt()
