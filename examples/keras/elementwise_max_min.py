"""Maximum / Minimum merge layers (reference: examples/python/keras/elementwise_max_min.py)."""
import numpy as np
import _common  # noqa: F401

import flexflow.keras.models
import flexflow.keras.optimizers
from flexflow.keras.layers import Dense, Input, Maximum, Minimum


def run(merge):
    in0 = Input(shape=(32,), dtype="float32")
    in1 = Input(shape=(10,), dtype="float32")
    x0 = Dense(20, activation="relu")(in0)
    x1 = Dense(20, activation="relu")(in1)
    out = Dense(1)(merge()([x0, x1]))
    model = flexflow.keras.models.Model([in0, in1], out)
    model.compile(optimizer=flexflow.keras.optimizers.Adam(learning_rate=0.001), loss="mean_squared_error",
                  metrics=["mean_squared_error"])
    print(model.summary())
    model.fit(x=[np.random.randn(300, 32).astype(np.float32), np.random.randn(300, 10).astype(np.float32)],
              y=np.random.randn(300, 1).astype(np.float32), epochs=2)


if __name__ == "__main__":
    run(Maximum)
    run(Minimum)
