"""Keras-style frontend (python/flexflow/keras/**: Sequential / functional
Model, layers, string losses/metrics, callbacks, datasets).

Layers are symbolic until ``compile``; ``fit`` builds the FFModel for the
batch size it is called with (the reference builds at compile time with
FFConfig's batch size; both are supported: ``compile(batch_size=...)``).
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional, Sequence

import numpy as np

from ..core import (ActiMode, AdamOptimizer, AggrMode, DataType, FFConfig, FFModel, LossType, MetricsType,
                    PoolType, SGDOptimizer)

_ACT = {None: ActiMode.AC_MODE_NONE, "linear": ActiMode.AC_MODE_NONE, "relu": ActiMode.AC_MODE_RELU,
        "sigmoid": ActiMode.AC_MODE_SIGMOID, "tanh": ActiMode.AC_MODE_TANH, "gelu": ActiMode.AC_MODE_GELU,
        "softmax": ActiMode.AC_MODE_NONE}
_LOSS = {"sparse_categorical_crossentropy": LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY,
         "categorical_crossentropy": LossType.LOSS_CATEGORICAL_CROSSENTROPY,
         "mean_squared_error": LossType.LOSS_MEAN_SQUARED_ERROR_AVG_REDUCE,
         "mse": LossType.LOSS_MEAN_SQUARED_ERROR_AVG_REDUCE}
_METRIC = {"accuracy": MetricsType.METRICS_ACCURACY,
           "categorical_crossentropy": MetricsType.METRICS_CATEGORICAL_CROSSENTROPY,
           "sparse_categorical_crossentropy": MetricsType.METRICS_SPARSE_CATEGORICAL_CROSSENTROPY,
           "mean_squared_error": MetricsType.METRICS_MEAN_SQUARED_ERROR,
           "root_mean_squared_error": MetricsType.METRICS_ROOT_MEAN_SQUARED_ERROR,
           "mean_absolute_error": MetricsType.METRICS_MEAN_ABSOLUTE_ERROR}


# ------------------------------------------------------------------- tensors
class KTensor:
    def __init__(self, layer: "Layer", inputs: List["KTensor"], shape, dtype="float32"):
        self.layer, self.inputs, self.shape, self.dtype = layer, inputs, tuple(shape), dtype


class Layer:
    _count: Dict[str, int] = {}

    def __init__(self, name: Optional[str] = None, input_shape=None, **kw):
        base = type(self).__name__.lower()
        n = Layer._count.get(base, 0)
        Layer._count[base] = n + 1
        self.name = name or f"{base}_{n}"
        self.input_shape = input_shape

    def __call__(self, x):
        xs = x if isinstance(x, (list, tuple)) else [x]
        return KTensor(self, list(xs), self.out_shape([t.shape for t in xs]))

    def out_shape(self, shapes):
        return shapes[0]

    def build_ff(self, ff: FFModel, ins):
        raise NotImplementedError


class InputLayer(Layer):
    def __init__(self, shape, dtype="float32", name=None):
        super().__init__(name)
        self.shape, self.dtype = tuple(shape), dtype


def Input(shape, dtype="float32", name=None, batch_size=None):  # noqa: N802
    layer = InputLayer(shape, dtype, name)
    t = KTensor(layer, [], (batch_size,) + tuple(shape), dtype)
    return t


class Dense(Layer):
    def __init__(self, units, activation=None, use_bias=True, input_shape=None, name=None, **kw):
        super().__init__(name)
        self.units, self.activation, self.use_bias, self.input_shape = units, activation, use_bias, input_shape

    def out_shape(self, s):
        return s[0][:-1] + (self.units,)

    def build_ff(self, ff, ins):
        t = ff.dense(ins[0], self.units, _ACT[self.activation], self.use_bias, name=self.name)
        return ff.softmax(t, name=self.name + "_softmax") if self.activation == "softmax" else t


class Conv2D(Layer):
    def __init__(self, filters, kernel_size, strides=(1, 1), padding="valid", activation=None, use_bias=True,
                 groups=1, input_shape=None, name=None, **kw):
        super().__init__(name)
        k = kernel_size if isinstance(kernel_size, (tuple, list)) else (kernel_size, kernel_size)
        s = strides if isinstance(strides, (tuple, list)) else (strides, strides)
        self.filters, self.k, self.s, self.padding = filters, tuple(k), tuple(s), padding
        self.activation, self.use_bias, self.groups, self.input_shape = activation, use_bias, groups, input_shape

    def _pad(self):
        if self.padding == "same":
            return (self.k[0] - 1) // 2, (self.k[1] - 1) // 2
        if isinstance(self.padding, (tuple, list)):
            return tuple(self.padding)
        return 0, 0

    def out_shape(self, s):
        b, c, h, w = s[0]
        ph, pw = self._pad()
        return (b, self.filters, (h + 2 * ph - self.k[0]) // self.s[0] + 1, (w + 2 * pw - self.k[1]) // self.s[1] + 1)

    def build_ff(self, ff, ins):
        ph, pw = self._pad()
        return ff.conv2d(ins[0], self.filters, self.k[0], self.k[1], self.s[0], self.s[1], ph, pw,
                         _ACT[self.activation], self.groups, self.use_bias, name=self.name)


class _Pool(Layer):
    kind = PoolType.POOL_MAX

    def __init__(self, pool_size=(2, 2), strides=None, padding="valid", name=None, **kw):
        super().__init__(name)
        p = pool_size if isinstance(pool_size, (tuple, list)) else (pool_size, pool_size)
        s = strides or p
        s = s if isinstance(s, (tuple, list)) else (s, s)
        self.p, self.s, self.pad = tuple(p), tuple(s), (0, 0) if padding == "valid" else ((p[0] - 1) // 2,
                                                                                          (p[1] - 1) // 2)

    def out_shape(self, s):
        b, c, h, w = s[0]
        return (b, c, (h + 2 * self.pad[0] - self.p[0]) // self.s[0] + 1,
                (w + 2 * self.pad[1] - self.p[1]) // self.s[1] + 1)

    def build_ff(self, ff, ins):
        return ff.pool2d(ins[0], self.p[0], self.p[1], self.s[0], self.s[1], self.pad[0], self.pad[1], self.kind,
                         name=self.name)


class MaxPooling2D(_Pool):
    kind = PoolType.POOL_MAX


class AveragePooling2D(_Pool):
    kind = PoolType.POOL_AVG


class Flatten(Layer):
    def out_shape(self, s):
        return (s[0][0], int(np.prod(s[0][1:])))

    def build_ff(self, ff, ins):
        return ff.flat(ins[0], name=self.name)


class Embedding(Layer):
    def __init__(self, input_dim, output_dim, input_length=None, name=None, **kw):
        super().__init__(name)
        self.input_dim, self.output_dim = input_dim, output_dim

    def out_shape(self, s):
        return s[0] + (self.output_dim,)

    def build_ff(self, ff, ins):
        return ff.embedding(ins[0], self.input_dim, self.output_dim, AggrMode.AGGR_MODE_NONE, name=self.name)


class Activation(Layer):
    def __init__(self, activation, name=None):
        super().__init__(name)
        self.activation = activation

    def build_ff(self, ff, ins):
        a = self.activation
        fn = {"relu": ff.relu, "sigmoid": ff.sigmoid, "tanh": ff.tanh, "gelu": ff.gelu, "elu": ff.elu,
              "softmax": ff.softmax}[a]
        return fn(ins[0], name=self.name)


class Dropout(Layer):
    def __init__(self, rate, seed=0, name=None):
        super().__init__(name)
        self.rate, self.seed = rate, seed

    def build_ff(self, ff, ins):
        return ff.dropout(ins[0], self.rate, self.seed, name=self.name)


class BatchNormalization(Layer):
    def build_ff(self, ff, ins):
        return ff.batch_norm(ins[0], False, name=self.name)


class LayerNormalization(Layer):
    def __init__(self, epsilon=1e-5, name=None, **kw):
        super().__init__(name)
        self.eps = epsilon

    def build_ff(self, ff, ins):
        return ff.layer_norm(ins[0], [-1], True, self.eps, name=self.name)


class Reshape(Layer):
    def __init__(self, target_shape, name=None):
        super().__init__(name)
        self.target = tuple(target_shape)

    def out_shape(self, s):
        return (s[0][0],) + self.target

    def build_ff(self, ff, ins):
        return ff.reshape(ins[0], [ins[0].dims[0]] + list(self.target), name=self.name)


class Permute(Layer):
    def __init__(self, dims, name=None):
        super().__init__(name)
        self.dims = tuple(dims)  # 1-based, excluding batch (Keras convention)

    def out_shape(self, s):
        return (s[0][0],) + tuple(s[0][d] for d in self.dims)

    def build_ff(self, ff, ins):
        return ff.transpose(ins[0], [0] + list(self.dims), name=self.name)


class _Merge(Layer):
    op = "add"

    def build_ff(self, ff, ins):
        t = ins[0]
        for i, x in enumerate(ins[1:]):
            t = getattr(ff, self.op)(t, x, name=f"{self.name}_{i}" if len(ins) > 2 else self.name)
        return t


class Add(_Merge):
    op = "add"


class Subtract(_Merge):
    op = "subtract"


class Multiply(_Merge):
    op = "multiply"


class Concatenate(Layer):
    def __init__(self, axis=-1, name=None):
        super().__init__(name)
        self.axis = axis

    def out_shape(self, s):
        ax = self.axis % len(s[0])
        out = list(s[0])
        out[ax] = sum(x[ax] for x in s)
        return tuple(out)

    def build_ff(self, ff, ins):
        return ff.concat(list(ins), self.axis, name=self.name)


def concatenate(xs, axis=-1):
    return Concatenate(axis)(xs)


def add(xs):
    return Add()(xs)


# ---------------------------------------------------------------- optimizers
class SGD:
    def __init__(self, learning_rate=0.01, momentum=0.0, nesterov=False, decay=0.0, lr=None):
        self.lr = lr if lr is not None else learning_rate
        self.momentum, self.nesterov, self.decay = momentum, nesterov, decay

    def ff(self, model):
        return SGDOptimizer(model, lr=self.lr, momentum=self.momentum, nesterov=self.nesterov,
                            weight_decay=self.decay)


class Adam:
    def __init__(self, learning_rate=0.001, beta_1=0.9, beta_2=0.999, epsilon=1e-8, lr=None):
        self.lr = lr if lr is not None else learning_rate
        self.b1, self.b2, self.eps = beta_1, beta_2, epsilon

    def ff(self, model):
        return AdamOptimizer(model, alpha=self.lr, beta1=self.b1, beta2=self.b2, epsilon=self.eps)


# ---------------------------------------------------------------- callbacks
class Callback:
    def on_train_begin(self, logs=None): ...

    def on_epoch_begin(self, epoch, logs=None): ...

    def on_epoch_end(self, epoch, logs=None): ...

    def on_train_end(self, logs=None): ...


class LearningRateScheduler(Callback):
    def __init__(self, schedule):
        self.schedule = schedule
        self.model = None

    def on_epoch_begin(self, epoch, logs=None):
        if self.model is not None:
            lr = self.schedule(epoch)
            self.model._ff._optimizer.set_learning_rate(lr)


class VerifyMetrics(Callback):
    """Stops with an error when accuracy ends below a target (reference:
    keras/callbacks.py VerifyMetrics used by the CI examples)."""

    def __init__(self, accuracy_target):
        self.target = accuracy_target
        self.model = None

    def on_train_end(self, logs=None):
        acc = self.model._ff.get_perf_metrics().accuracy * 100
        assert acc >= self.target, f"accuracy {acc:.2f}% < target {self.target}%"


class EpochVerifyMetrics(VerifyMetrics):
    def on_epoch_end(self, epoch, logs=None):
        acc = self.model._ff.get_perf_metrics().accuracy * 100
        if acc >= self.target:
            self.model._stop = True


# -------------------------------------------------------------------- models
class Model:
    def __init__(self, inputs=None, outputs=None, name=None):
        self.inputs = [] if inputs is None else (inputs if isinstance(inputs, (list, tuple)) else [inputs])
        self.outputs = [] if outputs is None else (outputs if isinstance(outputs, (list, tuple)) else [outputs])
        self.name = name or "model"
        self._compiled = None
        self._ff = None
        self._stop = False

    def compile(self, optimizer="sgd", loss=None, metrics=None, batch_size=None, ffconfig=None):
        opt = {"sgd": SGD(), "adam": Adam()}.get(optimizer, optimizer) if isinstance(optimizer, str) else optimizer
        self._compiled = dict(optimizer=opt, loss=loss, metrics=list(metrics or []), ffconfig=ffconfig)
        if batch_size:
            self._build(batch_size)
        return self

    def _graph_tensors(self):
        order, seen = [], set()

        def visit(t):
            if id(t) in seen:
                return
            seen.add(id(t))
            for i in t.inputs:
                visit(i)
            order.append(t)
        for o in self.outputs:
            visit(o)
        return order

    def _build(self, batch_size: int):
        c = self._compiled
        cfg = c["ffconfig"] or FFConfig()
        cfg.batch_size = batch_size
        ff = FFModel(cfg)
        env = {}
        for t in self._graph_tensors():
            if isinstance(t.layer, InputLayer):
                dt = DataType.DT_INT32 if "int" in t.dtype else DataType.DT_FLOAT
                env[id(t)] = ff.create_tensor([batch_size] + list(t.layer.shape), dt,
                                              create_grad=dt == DataType.DT_FLOAT, name=t.layer.name)
            else:
                env[id(t)] = t.layer.build_ff(ff, [env[id(i)] for i in t.inputs])
        loss = c["loss"]
        ff.compile(optimizer=c["optimizer"].ff(ff), loss_type=_LOSS[loss] if isinstance(loss, str) else loss,
                   metrics=[_METRIC[m] if isinstance(m, str) else m for m in c["metrics"]])
        self._ff = ff
        self._batch = batch_size
        return ff

    def fit(self, x=None, y=None, batch_size=None, epochs=1, callbacks=None, verbose=1):
        xs = x if isinstance(x, (list, tuple)) else [x]
        bs = batch_size or self._batch if self._ff is not None else (batch_size or 64)
        if self._ff is None or self._batch != bs:
            self._build(bs)
        callbacks = list(callbacks or [])
        for cb in callbacks:
            cb.model = self
            cb.on_train_begin()
        y = np.asarray(y)
        if y.ndim == 1:
            y = y.reshape(-1, 1)
        hist = []
        for e in range(epochs):
            for cb in callbacks:
                cb.on_epoch_begin(e)
            self._ff.fit(x=[np.asarray(a) for a in xs], y=y, batch_size=bs, epochs=1)
            pm = self._ff.get_perf_metrics()
            hist.append({"loss": pm.loss, "accuracy": pm.accuracy})
            for cb in callbacks:
                cb.on_epoch_end(e, hist[-1])
            if self._stop:
                break
        for cb in callbacks:
            cb.on_train_end()
        return {"history": hist}

    def evaluate(self, x=None, y=None, batch_size=None):
        xs = x if isinstance(x, (list, tuple)) else [x]
        y = np.asarray(y)
        if y.ndim == 1:
            y = y.reshape(-1, 1)
        return self._ff.eval(x=[np.asarray(a) for a in xs], y=y, batch_size=batch_size or self._batch)

    def summary(self):
        lines = [f'Model: "{self.name}"']
        for t in self._graph_tensors():
            lines.append(f"  {t.layer.name:<24} {type(t.layer).__name__:<20} {t.shape}")
        s = "\n".join(lines)
        print(s)
        return s

    @property
    def ffmodel(self):
        return self._ff


class Sequential(Model):
    def __init__(self, layers: Optional[Sequence[Layer]] = None, name=None):
        super().__init__(name=name or "sequential")
        self._layers: List[Layer] = []
        self._input = None
        for l in layers or []:
            self.add(l)

    def add(self, layer):
        if isinstance(layer, KTensor):  # keras.Input
            self._input = layer
            return
        if self._input is None:
            shp = getattr(layer, "input_shape", None)
            if shp is None:
                raise ValueError("the first layer needs input_shape= (or add a keras Input first)")
            self._input = Input(shp)
        self._layers.append(layer)
        t = self._input
        for l in self._layers:
            t = l(t)
        self.inputs, self.outputs = [self._input], [t]


# -------------------------------------------------------------------- datasets
class _Synthetic:
    """Keras dataset loaders.  There is no network access: ``load_data``
    reads a local ``.npz`` (``path=``, keys x_train/y_train/x_test/y_test,
    loaded with allow_pickle=False) or returns deterministic synthetic data
    of the real dataset's shapes."""

    def __init__(self, x_shape, n_classes, n_train, n_test, dtype=np.uint8, seq=False):
        self.x_shape, self.n_classes, self.n_train, self.n_test, self.dtype, self.seq = \
            x_shape, n_classes, n_train, n_test, dtype, seq

    def load_data(self, path: Optional[str] = None, num_samples: Optional[int] = None, **kw):
        if path:
            with np.load(path, allow_pickle=False) as d:
                return (d["x_train"], d["y_train"]), (d["x_test"], d["y_test"])
        rng = np.random.default_rng(0)
        ntr = num_samples or self.n_train
        nte = min(self.n_test, max(1, ntr // 6))

        def mk(n):
            y = rng.integers(0, self.n_classes, n)
            if self.seq:
                x = rng.integers(1, 1000, (n,) + self.x_shape)
            else:
                centers = rng.integers(0, 255, (self.n_classes,) + self.x_shape)
                x = np.clip(centers[y] + rng.normal(0, 30, (n,) + self.x_shape), 0, 255).astype(self.dtype)
            return x, y.astype(np.int64)
        return mk(ntr), mk(nte)


class datasets:  # noqa: N801
    mnist = _Synthetic((28, 28), 10, 60000, 10000)
    cifar10 = _Synthetic((3, 32, 32), 10, 50000, 10000)
    reuters = _Synthetic((100,), 46, 8982, 2246, np.int64, seq=True)
