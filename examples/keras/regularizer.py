"""L2 kernel regularizer on a Dense layer (reference: examples/python/keras/regularizer.py)."""
import numpy as np
import _common  # noqa: F401

import flexflow.keras as keras
import flexflow.keras.models
import flexflow.keras.optimizers
from flexflow.keras.layers import Dense, Input


def regularizer_example():
    in0 = Input(shape=(10,), dtype="float32")
    x0 = Dense(16, activation="relu", kernel_regularizer=keras.regularizers.L2(0.001))(in0)
    out = Dense(1)(x0)
    model = flexflow.keras.models.Model(in0, out)
    model.compile(optimizer=flexflow.keras.optimizers.Adam(learning_rate=0.001), loss="mean_squared_error",
                  metrics=["mean_squared_error"])
    model.fit(x=np.random.randn(300, 10).astype(np.float32), y=np.random.randn(300, 1).astype(np.float32), epochs=2)


if __name__ == "__main__":
    regularizer_example()
