"""The 'identity' loss: the model output (a per-sample sum) is minimised
directly (reference: examples/python/keras/identity_loss.py)."""
import numpy as np
import _common  # noqa: F401

import flexflow.keras.backend
import flexflow.keras.models
import flexflow.keras.optimizers
from flexflow.keras.layers import Dense, Input


def test_identity_loss():
    in0 = Input(shape=(32,), dtype="float32")
    x0 = Dense(20, activation="relu")(in0)
    out = flexflow.keras.backend.sum(x0, axis=1)     # (B,)
    model = flexflow.keras.models.Model(in0, out)
    model.compile(optimizer=flexflow.keras.optimizers.Adam(learning_rate=0.01), loss="identity",
                  metrics=["mean_absolute_error"])
    print(model.summary())
    model.fit(x=np.random.randn(300, 32).astype(np.float32), y=np.zeros((300,)).astype(np.float32), epochs=2)


if __name__ == "__main__":
    test_identity_loss()
