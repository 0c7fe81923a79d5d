"""torch.gather-style Gather through keras backend.internal.gather
(reference: examples/python/keras/gather.py)."""
import numpy as np
import _common  # noqa: F401

import flexflow.keras.models
import flexflow.keras.optimizers
from flexflow.keras.backend.internal import gather
from flexflow.keras.layers import Dense, Input, Reshape


def gather_example():
    h = 3
    idx = np.array([[5, 7, 10], [8, 4, 0]]).reshape(-1, 1).repeat(h, 1).astype(np.int32)   # (6, 3)
    in0 = Input(shape=(10,), dtype="float32")
    in1 = Input(shape=idx.shape, dtype="int32")
    x0 = Reshape((20, h))(Dense(60, activation="relu")(in0))          # (B, 20, 3)
    f0 = Reshape((18,))(gather(x0, in1, axis=1))                     # (B, 6, 3) -> (B, 18)
    out = Dense(1)(f0)
    model = flexflow.keras.models.Model([in0, in1], out)
    model.compile(optimizer=flexflow.keras.optimizers.Adam(learning_rate=0.001), loss="mean_squared_error",
                  metrics=["mean_squared_error"])
    print(model.summary())
    model.fit(x=[np.random.randn(300, 10).astype(np.float32), idx[None, ...].repeat(300, 0).astype(np.int32)],
              y=np.random.randn(300, 1).astype(np.float32), epochs=2)


if __name__ == "__main__":
    gather_example()
