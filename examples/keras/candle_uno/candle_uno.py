"""CANDLE-Uno drug-response regression with the keras API (reference:
examples/python/keras/candle_uno/candle_uno.py): one dense feature tower per
cell / drug input (a nested keras Model each), concatenation with the dose
inputs, a dense trunk, one regression output, MSE.

The reference downloads and preprocesses the CANDLE Uno data; there is no
network here, so the inputs are synthetic arrays of its feature shapes
(flexflow_train_amd/models/recsys.py CandleUnoConfig, the reference's
uno_default_model.txt sizes) with a target that depends on them."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))))

import numpy as np  # noqa: E402

import flexflow.keras.optimizers  # noqa: E402
from flexflow.keras.layers import Add, Concatenate, Dense, Dropout, Input  # noqa: E402
from flexflow.keras.models import Model  # noqa: E402
from flexflow_train_amd.models.recsys import CandleUnoConfig  # noqa: E402


def build_feature_model(input_shape, name="", dense_layers=(1000, 1000), activation="relu", residual=False,
                        dropout_rate=0.0):
    x_input = Input(shape=input_shape)
    h = x_input
    for layer in dense_layers:
        x = h
        h = Dense(layer, activation=activation)(h)
        if dropout_rate > 0:
            h = Dropout(dropout_rate)(h)
        if residual and x.shape == h.shape:
            h = Add()([h, x])
    return Model(x_input, h, name=name)


def build_model(cfg: CandleUnoConfig):
    towers = {k for k in cfg.feature_shapes if k.split(".")[0] in ("cell", "drug")}
    inputs, encoded = [], []
    for fea_name, fea_type in cfg.input_features.items():
        shape = (cfg.feature_shapes[fea_type],)
        fea_input = Input(shape, name="input." + fea_name)
        inputs.append(fea_input)
        if fea_type in towers:
            sub = build_feature_model(shape, fea_type, cfg.dense_feature_layers, dropout_rate=cfg.dropout,
                                      residual=cfg.residual)
            encoded.append(sub(fea_input))
        else:
            encoded.append(fea_input)
    h = Concatenate(axis=1)(encoded)
    for layer in cfg.dense_layers:
        x = h
        h = Dense(layer, activation="relu")(h)
        if cfg.dropout > 0:
            h = Dropout(cfg.dropout)(h)
        if cfg.residual and x.shape == h.shape:
            h = Add()([h, x])
    return inputs, Model(inputs, Dense(1)(h))


def synthetic(cfg: CandleUnoConfig, n: int, seed=0):
    rng = np.random.default_rng(seed)
    xs = [rng.standard_normal((n, cfg.feature_shapes[t])).astype(np.float32) for t in cfg.input_features.values()]
    w = [rng.standard_normal(x.shape[1]).astype(np.float32) / np.sqrt(x.shape[1]) for x in xs]
    y = np.tanh(sum(x @ v for x, v in zip(xs, w)) / len(xs)).astype(np.float32).reshape(-1, 1)
    return xs, y


def top_level_task():
    quick = "FF_EXAMPLE_SAMPLES" in os.environ
    cfg = CandleUnoConfig()
    if quick:
        cfg = CandleUnoConfig(dense_layers=[64] * 2, dense_feature_layers=[64] * 2,
                              feature_shapes={"dose": 1, "cell.rnaseq": 94, "drug.descriptors": 527,
                                              "drug.fingerprints": 204})
    n = int(os.environ.get("FF_EXAMPLE_SAMPLES", 10000))
    xs, y = synthetic(cfg, n)
    _, model = build_model(cfg)
    model.compile(optimizer=flexflow.keras.optimizers.SGD(learning_rate=0.001), loss="mean_squared_error",
                  metrics=["mean_squared_error", "mean_absolute_error"])
    print(model.summary())
    model.fit(xs, y, epochs=int(os.environ.get("FF_EXAMPLE_EPOCHS", 1)))


if __name__ == "__main__":
    top_level_task()
