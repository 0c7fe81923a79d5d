"""Keras frontend API (reference: python/flexflow/keras/**): layers, nested
models, weights, callbacks, backend functions, utils and preprocessing."""
import numpy as np
import pytest

import flexflow.keras as keras
from flexflow.keras import backend as K
from flexflow.keras.callbacks import Callback, LearningRateScheduler
from flexflow.keras.layers import (Activation, Add, Concatenate, Conv2D, Dense, Flatten, Input, Maximum, Minimum,
                                   Permute, Reshape)
from flexflow.keras.models import Model, Sequential
from flexflow.keras.optimizers import SGD, Adam


def _mlp(seed=0, reg=None):
    inp = Input(shape=(8,))
    t = Dense(16, activation="relu", kernel_regularizer=reg, name="d1")(inp)
    out = Dense(3, name="d2")(t)
    m = Model(inp, Activation("softmax")(out))
    m.compile(optimizer=SGD(learning_rate=0.1), loss="sparse_categorical_crossentropy", metrics=["accuracy"],
              batch_size=8)
    return m


def _data(n=64, seed=0):
    rng = np.random.default_rng(seed)
    x = rng.standard_normal((n, 8)).astype(np.float32)
    y = (x[:, 0] > 0).astype(np.int32) + (x[:, 1] > 0).astype(np.int32)
    return x, y.reshape(-1, 1)


def test_weights_roundtrip_and_transfer():
    a, b = _mlp(), _mlp()
    ka, ba = a.get_layer(name="d1").get_weights(a.ffmodel)
    b.get_layer(index=0).set_weights(b.ffmodel, ka, ba)
    kb, bb = b.get_layer(index=0).get_weights(b.ffmodel)
    np.testing.assert_array_equal(ka, kb)
    np.testing.assert_array_equal(ba, bb)
    # whole-model get/set
    b.set_weights(a.get_weights())
    for wa, wb in zip(a.get_weights(), b.get_weights()):
        np.testing.assert_array_equal(wa, wb)
    x, _ = _data(16)
    np.testing.assert_allclose(a.predict(x), b.predict(x), rtol=1e-6, atol=1e-6)


def test_fit_with_other_batch_keeps_weights():
    m = _mlp()
    k0 = m.get_layer(index=0).get_weights(m.ffmodel)[0]
    x, y = _data(64)
    m.fit(x, y, batch_size=16, epochs=0)      # rebuild only
    np.testing.assert_array_equal(m.get_layer(index=0).get_weights(m.ffmodel)[0], k0)
    h = m.fit(x, y, batch_size=16, epochs=3)
    assert len(h.history["loss"]) == 3


def test_nested_model_matches_flat_model():
    inner_in = Input(shape=(8,))
    inner = Model(inner_in, Dense(6, activation="relu", name="inner_d")(inner_in))
    x_in = Input(shape=(8,))
    outer = Model(x_in, Activation("softmax")(Dense(3, name="head")(inner(x_in))))
    outer.compile(optimizer="sgd", loss="sparse_categorical_crossentropy", metrics=["accuracy"], batch_size=8)
    assert [l.name for l in outer.layers] == ["inner_d", "head", outer.layers[2].name]
    x, _ = _data(8)
    k, b = outer.get_layer(name="inner_d").get_weights(outer.ffmodel)
    hk, hb = outer.get_layer(name="head").get_weights(outer.ffmodel)
    # weights are stored (in, out) for the Linear kernel of this framework
    kk = k if k.shape == (8, 6) else k.T
    hkk = hk if hk.shape == (6, 3) else hk.T
    logits = np.maximum(x @ kk + b, 0) @ hkk + hb
    ref = np.exp(logits - logits.max(1, keepdims=True))
    ref /= ref.sum(1, keepdims=True)
    np.testing.assert_allclose(outer.predict(x), ref, rtol=1e-4, atol=1e-5)


def test_sequential_add_pop_and_nested_sequential():
    s = Sequential()
    s.add(Input(shape=(4, 4)))
    s.add(Flatten())
    s.add(Dense(5))
    s.add(Dense(7))
    assert s.output.shape == (None, 7)
    s.pop()
    assert s.output.shape == (None, 5)
    outer = Sequential([s, Dense(2)])
    assert outer.output.shape == (None, 2)
    outer.compile(optimizer=Adam(), loss="mean_squared_error", metrics=["mean_squared_error"], batch_size=4)
    rng = np.random.default_rng(0)
    outer.fit(rng.standard_normal((16, 4, 4)).astype(np.float32), rng.standard_normal((16, 2)).astype(np.float32))


def test_merge_and_tensor_ops_shapes():
    a, b = Input(shape=(10, 2)), Input(shape=(10, 1))
    assert Add()([a, b]).shape == (None, 10, 2)
    assert (a * b).shape == (None, 10, 2)
    assert (a - a).shape == (None, 10, 2)
    assert Maximum()([a, a]).shape == Minimum()([a, a]).shape == (None, 10, 2)
    assert Concatenate(axis=1)([a, a]).shape == (None, 20, 2)
    assert Permute((2, 1))(a).shape == (None, 2, 10)
    assert Permute((0, 2, 1))(a).shape == (None, 2, 10)       # the reference's full-permutation form
    assert Reshape((-1,))(a).shape == (None, 20)
    assert K.sum(a, axis=1).shape == (None, 2)
    assert K.sum(a, axis=[1, 2], keepdims=True).shape == (None, 1, 1)
    c = Input(shape=(2, 3))
    assert K.batch_dot(a, c).shape == (None, 10, 3)
    assert (a @ c).shape == (None, 10, 3)
    assert Conv2D(4, 3, padding="same")(Input(shape=(3, 8, 8))).shape == (None, 4, 8, 8)


def test_elementwise_max_min_values():
    a, b = Input(shape=(6,)), Input(shape=(6,))
    for layer, fn in ((Maximum, np.maximum), (Minimum, np.minimum)):
        m = Model([a, b], layer()([a, b]))
        m.compile(optimizer="sgd", loss="mean_squared_error", metrics=["mean_squared_error"], batch_size=4)
        rng = np.random.default_rng(1)
        x0, x1 = rng.standard_normal((4, 6)).astype(np.float32), rng.standard_normal((4, 6)).astype(np.float32)
        np.testing.assert_allclose(m.predict([x0, x1]), fn(x0, x1), rtol=1e-6)


def test_callbacks_schedule_and_batch_hooks():
    m = _mlp()
    seen, lrs = [], []

    class Rec(Callback):
        def on_batch_begin(self, batch, logs=None):
            seen.append(("b", batch))

        def on_batch_end(self, batch, logs=None):
            seen.append(("e", batch))

        def on_epoch_begin(self, epoch, logs=None):
            lrs.append(self.model.optimizer.ffhandle.cfg.lr)

    x, y = _data(32)
    m.fit(x, y, epochs=2, callbacks=[LearningRateScheduler(lambda e: 0.05 * (e + 1)), Rec()])
    assert lrs == [0.05, 0.1]
    assert seen[:4] == [("b", 0), ("e", 0), ("b", 1), ("e", 1)] and len(seen) == 2 * 2 * 4


def test_keras_regularizer_reaches_linear():
    m = _mlp(reg=keras.regularizers.L2(0.01))
    ex = m.ffmodel.executor
    regs = [p.regularizer for p in ex.params if p.regularizer]
    assert regs == [("l2", 0.01)]


def test_losses_metrics_initializers_objects():
    from flexflow.keras import initializers, losses, metrics
    inp = Input(shape=(8,))
    out = Dense(3, kernel_initializer=initializers.Zeros(), bias_initializer=initializers.Constant(0.5))(inp)
    m = Model(inp, out)
    m.compile(optimizer="adam", loss=losses.MeanSquaredError(),
              metrics=[metrics.MeanSquaredError(), metrics.MeanAbsoluteError()], batch_size=4)
    k, b = m.layers[0].get_weights(m.ffmodel)
    assert not k.any() and np.allclose(b, 0.5)
    with pytest.raises(ValueError):
        m.compile(optimizer="sgd", loss="hinge")


def test_utils_and_preprocessing():
    from flexflow.keras.preprocessing.sequence import pad_sequences
    from flexflow.keras.preprocessing.text import Tokenizer, text_to_word_sequence, tokenizer_from_json
    from flexflow.keras.utils import normalize, to_categorical
    np.testing.assert_array_equal(to_categorical([[1], [0], [2]], 3), np.eye(3)[[1, 0, 2]])
    np.testing.assert_allclose(np.linalg.norm(normalize(np.array([[3.0, 4.0]])), axis=-1), 1.0)
    np.testing.assert_array_equal(pad_sequences([[1, 2, 3], [4]], maxlen=2), [[2, 3], [0, 4]])
    np.testing.assert_array_equal(pad_sequences([[1, 2, 3], [4]], maxlen=2, padding="post", truncating="post"),
                                  [[1, 2], [4, 0]])
    assert text_to_word_sequence("Hello, World! hello") == ["hello", "world", "hello"]
    t = Tokenizer(num_words=10)
    t.fit_on_texts(["the cat sat", "the dog"])
    assert t.word_index["the"] == 1
    seqs = t.texts_to_sequences(["the cat", "a dog"])
    assert seqs[0] == [1, t.word_index["cat"]] and seqs[1] == [t.word_index["dog"]]
    mat = t.sequences_to_matrix(seqs, mode="count")
    assert mat.shape == (2, 10) and mat[0, 1] == 1
    assert tokenizer_from_json(t.to_json()).word_index == t.word_index


def test_datasets_shapes():
    from flexflow.keras.datasets import cifar10, mnist, reuters
    (x, y), _ = mnist.load_data(num_samples=100)
    assert x.shape == (100, 28, 28) and x.dtype == np.uint8 and y.shape == (100,)
    (x, y), _ = cifar10.load_data(100)
    assert x.shape == (100, 3, 32, 32) and y.shape == (100, 1)
    (x, y), (xt, yt) = reuters.load_data(num_words=500, test_split=0.2)
    assert len(x) + len(xt) == reuters.N_SAMPLES and max(max(s) for s in x) < 500 and y.max() < 46
    assert K.backend() == "flexflow"
