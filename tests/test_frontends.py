"""Frontends: torch.fx importer (+ .ff round trip, numerics vs torch),
Keras-style API, ONNX importer (wire-format reader/writer)."""
import numpy as np
import pytest
import torch
import torch.nn as nn

from flexflow.core import DataType, FFConfig, FFModel, LossType, MetricsType, SGDOptimizer
from flexflow.torch.model import PyTorchModel, copy_weights, file_to_ff


class SmallCNN(nn.Module):
    def __init__(self):
        super().__init__()
        self.conv = nn.Conv2d(3, 8, 3, 1, 1)
        self.pool = nn.MaxPool2d(2, 2)
        self.fc1 = nn.Linear(8 * 4 * 4, 32)
        self.fc2 = nn.Linear(32, 10)

    def forward(self, x):
        x = self.pool(torch.relu(self.conv(x)))
        x = torch.flatten(x, 1)
        x = torch.relu(self.fc1(x)) * 0.5 + 1.0
        return torch.softmax(self.fc2(x), dim=-1)


class TinyAttn(nn.Module):
    def __init__(self):
        super().__init__()
        self.attn = nn.MultiheadAttention(16, 4, batch_first=True)
        self.ln = nn.LayerNorm(16)
        self.out = nn.Linear(16, 5)

    def forward(self, x):
        a = self.attn(x, x, x)[0]
        return torch.softmax(self.out(self.ln(a + x)), dim=-1)


def _compile(m):
    m.compile(optimizer=SGDOptimizer(m, lr=0.0), loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY,
              metrics=[MetricsType.METRICS_ACCURACY])
    return m


@pytest.mark.parametrize("mode", ["memory", "file"])
def test_torch_import_matches_torch(tmp_path, mode):
    torch.manual_seed(0)
    net = SmallCNN().eval()
    pm = PyTorchModel(net)
    ff = FFModel(FFConfig())
    x = ff.create_tensor([4, 3, 8, 8], DataType.DT_FLOAT, name="x")
    if mode == "memory":
        pm.torch_to_ff(ff, [x])
    else:
        path = str(tmp_path / "m.ff")
        pm.torch_to_file(path)
        text = open(path).read()
        assert "; LINEAR; 32; 10; 1" in text and "; CONV2D; 8; 3; 3; 1; 1; 1; 1; 10; 1; 1" in text
        file_to_ff(path, ff, [x])
    _compile(ff)
    copy_weights(ff, pm.weights())
    inp = torch.randn(4, 3, 8, 8)
    out = ff.executor.forward({"x": inp}, training=False)
    torch.testing.assert_close(out.float(), net(inp), rtol=1e-4, atol=1e-5)


def test_torch_import_attention_matches_torch():
    torch.manual_seed(1)
    net = TinyAttn().eval()
    ff = FFModel(FFConfig())
    x = ff.create_tensor([2, 6, 16], DataType.DT_FLOAT, name="x")
    pm = PyTorchModel(net)
    pm.torch_to_ff(ff, [x])
    _compile(ff)
    copy_weights(ff)
    inp = torch.randn(2, 6, 16)
    out = ff.executor.forward({"x": inp}, training=False)
    torch.testing.assert_close(out.float(), net(inp), rtol=1e-4, atol=1e-5)


class TinyCross(nn.Module):
    def __init__(self):
        super().__init__()
        self.attn = nn.MultiheadAttention(16, 2, batch_first=True)

    def forward(self, q, kv):
        return torch.softmax(self.attn(q, kv, kv)[0], dim=-1)


def test_torch_import_cross_attention_matches_torch():
    torch.manual_seed(2)
    net = TinyCross().eval()
    ff = FFModel(FFConfig())
    q = ff.create_tensor([2, 5, 16], DataType.DT_FLOAT, name="q")
    kv = ff.create_tensor([2, 7, 16], DataType.DT_FLOAT, name="kv")
    PyTorchModel(net).torch_to_ff(ff, [q, kv])
    _compile(ff)
    copy_weights(ff)
    a, b = torch.randn(2, 5, 16), torch.randn(2, 7, 16)
    out = ff.executor.forward({"q": a, "kv": b}, training=False)
    torch.testing.assert_close(out.float(), net(a, b), rtol=1e-4, atol=1e-5)


def test_keras_sequential_learns_synthetic_mnist():
    from flexflow.keras import Sequential, datasets
    from flexflow.keras.layers import Dense, Flatten
    from flexflow.keras.optimizers import SGD

    (xt, yt), _ = datasets.mnist.load_data(num_samples=1024)
    xt = (xt.astype(np.float32) / 255.0)
    model = Sequential([Flatten(input_shape=(28, 28)), Dense(64, activation="relu"), Dense(10, activation="softmax")])
    model.compile(optimizer=SGD(learning_rate=0.1), loss="sparse_categorical_crossentropy", metrics=["accuracy"])
    hist = model.fit(xt, yt.astype(np.int32), batch_size=64, epochs=3)
    assert hist["history"][-1]["accuracy"] > 0.9


def test_keras_functional_concat_cnn():
    from flexflow.keras import Input, Model
    from flexflow.keras.layers import Concatenate, Conv2D, Dense, Flatten, MaxPooling2D

    inp = Input((3, 8, 8))
    a = MaxPooling2D()(Conv2D(4, 3, padding="same", activation="relu")(inp))
    b = MaxPooling2D()(Conv2D(4, 1, activation="relu")(inp))
    t = Dense(5, activation="softmax")(Flatten()(Concatenate(axis=1)([a, b])))
    model = Model(inp, t)
    model.compile(optimizer="sgd", loss="sparse_categorical_crossentropy", metrics=["accuracy"])
    x = np.random.default_rng(0).standard_normal((32, 3, 8, 8)).astype(np.float32)
    y = np.random.default_rng(1).integers(0, 5, 32).astype(np.int32)
    model.fit(x, y, batch_size=16, epochs=1)
    assert "Conv2D" in model.summary()


def test_onnx_import_roundtrip():
    from flexflow.onnx.model import Node, ONNXModel, encode_model

    rng = np.random.default_rng(0)
    W1 = rng.standard_normal((16, 32)).astype(np.float32)
    b1 = rng.standard_normal(32).astype(np.float32)
    W2 = rng.standard_normal((10, 32)).astype(np.float32)   # transB
    b2 = rng.standard_normal(10).astype(np.float32)
    nodes = [Node("Gemm", ["x", "W1", "b1"], ["h"], "fc1"), Node("Relu", ["h"], ["r"], "relu"),
             Node("Gemm", ["r", "W2", "b2"], ["z"], "fc2", {"transB": 1}),
             Node("Softmax", ["z"], ["y"], "sm", {"axis": -1})]
    blob = encode_model(nodes, {"W1": W1, "b1": b1, "W2": W2, "b2": b2}, [("x", [8, 16])], [("y", [8, 10])])
    om = ONNXModel(blob)
    ff = FFModel(FFConfig())
    x = ff.create_tensor([8, 16], DataType.DT_FLOAT, name="x")
    om.apply(ff, [x])
    _compile(ff)
    om.copy_weights(ff)
    xin = rng.standard_normal((8, 16)).astype(np.float32)
    out = ff.executor.forward({"x": torch.as_tensor(xin)}, training=False).numpy()
    z = np.maximum(xin @ W1 + b1, 0) @ W2.T + b2
    ref = np.exp(z - z.max(-1, keepdims=True))
    ref /= ref.sum(-1, keepdims=True)
    np.testing.assert_allclose(out, ref, rtol=1e-4, atol=1e-5)


def test_reference_tensor_access_api():
    """Legion-era Tensor/FFModel calls (inline_map, attach_numpy_array,
    get_array, add_layer, prefetch, PerfMetrics.get_accuracy) keep working."""
    import numpy as np
    from flexflow_train_amd.core import DataType, FFConfig, FFModel, LossType, MetricsType, SGDOptimizer

    cfg = FFConfig()
    cfg.batch_size = 8
    m = FFModel(cfg)
    x = m.create_tensor([8, 16], DataType.DT_FLOAT, name="x")
    t = m.add_layer("LINEAR", name="lin", inputs=[x], out_channels=4, activation="none", use_bias=True)
    m.softmax(t)
    m.compile(optimizer=SGDOptimizer(m, lr=0.05), loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY,
              metrics=[MetricsType.METRICS_ACCURACY])
    data = np.arange(128, dtype=np.float32).reshape(8, 16) / 128
    x.attach_numpy_array(m, cfg, data)
    x.inline_map(m, cfg)
    assert x.is_mapped()
    np.testing.assert_allclose(x.get_array(m, cfg), data)
    assert x.get_flat_array(m, cfg).shape == (128,)
    x.inline_unmap(m, cfg)
    assert not x.is_mapped()
    assert m.prefetch() is None
    assert m.get_perf_metrics().get_accuracy() == 0.0
    x.detach_numpy_array(m, cfg)


def test_activation_value_and_gradient_access():
    import numpy as np
    import torch
    from flexflow_train_amd.core import ActiMode, DataType, FFConfig, FFModel, LossType, MetricsType, SGDOptimizer

    cfg = FFConfig()
    cfg.batch_size = 4
    m = FFModel(cfg)
    x = m.create_tensor([4, 8], DataType.DT_FLOAT, name="x")
    h = m.dense(x, 6, ActiMode.AC_MODE_RELU, name="h")
    m.softmax(m.dense(h, 3, name="o"))
    m.compile(optimizer=SGDOptimizer(m, lr=0.0), loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY,
              metrics=[MetricsType.METRICS_ACCURACY])
    assert h.get_tensor(m) is None          # registers retention
    assert h.get_gradients(m) is None
    rng = np.random.default_rng(0)
    X = rng.standard_normal((4, 8)).astype(np.float32)
    Y = np.array([[0], [1], [2], [1]], np.int32)
    m.fit(x=X, y=Y, epochs=1)
    hv = h.get_tensor(m)
    W = m.get_layer_by_name("h").get_weight_tensor().get_weights(m)
    b = m.get_layer_by_name("h").get_bias_tensor().get_weights(m)
    np.testing.assert_allclose(hv, np.maximum(X @ W + b, 0), rtol=1e-4, atol=1e-5)
    g = h.get_gradients(m)
    assert g.shape == (4, 6) and np.isfinite(g).all() and np.abs(g).sum() > 0


@pytest.mark.parametrize("kind", ["l2", "l1"])
def test_dense_kernel_regularizer(kind):
    """dense(kernel_regularizer=...) adds lambda*W (L2) / lambda*sign(W) (L1)
    to the kernel gradient (reference linear_kernels.cu:258); the bias and the
    other layer are untouched."""
    import numpy as np
    from flexflow_train_amd.core import ActiMode, DataType, FFConfig, FFModel, LossType, SGDOptimizer

    rng = np.random.default_rng(0)
    X = rng.standard_normal((4, 8)).astype(np.float32)
    Y = np.array([[0], [1], [2], [1]], np.int32)
    lr, lam = 0.5, 0.1

    def run(reg):
        cfg = FFConfig()
        cfg.batch_size = 4
        m = FFModel(cfg)
        x = m.create_tensor([4, 8], DataType.DT_FLOAT, name="x")
        h = m.dense(x, 6, ActiMode.AC_MODE_RELU, kernel_regularizer=reg, name="h")
        m.softmax(m.dense(h, 3, name="o"))
        m.compile(optimizer=SGDOptimizer(m, lr=lr), loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY)
        layer = m.get_layer_by_name("h")
        w0 = layer.get_weight_tensor().get_weights(m).copy()
        m.fit(x=X, y=Y, epochs=1)
        return (w0, layer.get_weight_tensor().get_weights(m), layer.get_bias_tensor().get_weights(m),
                m.get_layer_by_name("o").get_weight_tensor().get_weights(m))

    w0a, wa, ba, oa = run(None)
    w0b, wb, bb, ob = run((kind, lam))
    np.testing.assert_array_equal(w0a, w0b)
    step = lam * (w0a if kind == "l2" else np.sign(w0a))
    np.testing.assert_allclose(wb, wa - lr * step, rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(bb, ba, rtol=1e-6, atol=1e-7)
    np.testing.assert_allclose(ob, oa, rtol=1e-6, atol=1e-7)


def test_onnx_export_torch_roundtrip_matches_torch():
    """export_torch (fx -> ONNX wire format) -> ONNXModel import -> same
    forward as the torch module (weights carried as initializers)."""
    import torch
    import torch.nn as nn
    from flexflow.core import DataType, FFConfig, FFModel, LossType, SGDOptimizer
    from flexflow.onnx.model import ONNXModel, export_torch

    class Net(nn.Module):
        def __init__(self):
            super().__init__()
            self.conv = nn.Conv2d(3, 4, 3, padding=1)
            self.pool = nn.MaxPool2d(2, 2)
            self.fc = nn.Linear(4 * 4 * 4, 5)

        def forward(self, x):
            y = self.pool(torch.relu(self.conv(x)))
            return torch.softmax(self.fc(torch.flatten(y, 1)), dim=-1)

    torch.manual_seed(0)
    net = Net().eval()
    x = torch.randn(4, 3, 8, 8)
    data = export_torch(net, x)
    cfg = FFConfig()
    cfg.batch_size = 4
    ff = FFModel(cfg)
    t = ff.create_tensor([4, 3, 8, 8], DataType.DT_FLOAT)
    om = ONNXModel(data)
    om.apply(ff, {"input.1": t})
    ff.compile(optimizer=SGDOptimizer(ff, 0.0), loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY)
    om.copy_weights(ff)
    out = ff.executor.forward({t.name: x}, training=False)
    torch.testing.assert_close(out.float(), net(x), rtol=1e-4, atol=1e-5)


def test_onnx_export_keras_roundtrip_matches_keras():
    import numpy as np
    from flexflow.core import DataType, FFConfig, FFModel, LossType, SGDOptimizer
    from flexflow.keras.layers import Activation, Conv2D, Dense, Flatten, Input, MaxPooling2D
    from flexflow.keras.models import Model
    from flexflow.onnx.model import ONNXModelKeras, export_keras

    inp = Input(shape=(3, 8, 8))
    t = MaxPooling2D()(Conv2D(4, 3, padding="same", activation="relu")(inp))
    out = Activation("softmax")(Dense(5)(Dense(6, activation="relu")(Flatten()(t))))
    km = Model(inp, out)
    km.compile(optimizer="sgd", loss="sparse_categorical_crossentropy", metrics=["accuracy"], batch_size=4)
    data = export_keras(km)
    cfg = FFConfig()
    cfg.batch_size = 4
    ff = FFModel(cfg)
    x = ff.create_tensor([4, 3, 8, 8], DataType.DT_FLOAT)
    om = ONNXModelKeras(data, cfg, ff)
    om.apply(ff, {"input_1": x})
    assert [n.op_type for n in om.graph.nodes].count("MatMul") == 2      # keras2onnx form, fused on import
    ff.compile(optimizer=SGDOptimizer(ff, 0.0), loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY)
    om.copy_weights(ff)
    xv = np.random.default_rng(0).standard_normal((4, 3, 8, 8)).astype(np.float32)
    import torch
    got = ff.executor.forward({x.name: torch.as_tensor(xv)}, training=False).float().numpy()
    np.testing.assert_allclose(got, km.predict(xv), rtol=1e-4, atol=1e-5)


def test_hf_mt5_import_matches_torch():
    """PyTorchModel(is_hf_model=True): a Hugging Face MT5 (encoder-decoder,
    relative position buckets, RMS norms, gated GELU, padding mask) through
    torch.export + the ATen lowering gives the module's logits."""
    import torch
    transformers = pytest.importorskip("transformers")
    from flexflow.core import DataType, FFConfig, FFModel, LossType, SGDOptimizer
    from flexflow.torch.model import PyTorchModel, copy_weights

    cfg = transformers.MT5Config(vocab_size=256, d_model=32, d_kv=8, d_ff=64, num_layers=2, num_decoder_layers=2,
                                 num_heads=4, relative_attention_num_buckets=8, dropout_rate=0.0)
    torch.manual_seed(0)
    m = transformers.MT5ForConditionalGeneration(cfg).eval()
    B, S = 2, 10
    ids, dids = torch.randint(0, 256, (B, S)), torch.randint(0, 256, (B, S))
    mask = torch.ones(B, S, dtype=torch.long)
    mask[1, 7:] = 0
    with torch.no_grad():
        ref = m(input_ids=ids, attention_mask=mask, decoder_input_ids=dids, use_cache=False).logits
    fc = FFConfig()
    fc.batch_size = B
    ff = FFModel(fc)
    names = ["input_ids", "attention_mask", "decoder_input_ids"]
    ts = [ff.create_tensor([B, S], DataType.DT_INT64, create_grad=False, name=n) for n in names]
    outs = PyTorchModel(m, is_hf_model=True, input_names=names).torch_to_ff(ff, ts)
    assert isinstance(outs, list) and tuple(outs[0].dims) == (B, S, 256)
    ff.compile(optimizer=SGDOptimizer(ff, 0.0), loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY)
    copy_weights(ff)
    got = ff.executor.forward(dict(zip(names, (ids, mask, dids))), training=False)
    torch.testing.assert_close(got.float(), ref, rtol=1e-4, atol=1e-4)
