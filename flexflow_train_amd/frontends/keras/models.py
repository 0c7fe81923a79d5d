"""Keras models (reference: python/flexflow/keras/models/{base_model,model,
sequential,tensor}.py).

``compile`` builds the FFModel right away for the configured batch size
(``FFConfig.batch_size``, or ``compile(batch_size=...)``), so layer weights
can be read and written before training (``get_layer(...).set_weights``, the
net2net examples).  ``fit(batch_size=B)`` with another B rebuilds the FFModel
for B and carries the weights over.  A Model is itself callable on tensors
(nested models): its graph is re-applied to the new inputs.
"""
from __future__ import annotations

import os
import sys
import time
from typing import Dict, List, Optional, Sequence

import numpy as np

from ...core import DataType, FFConfig, FFModel, LossType
from . import losses as _losses
from . import metrics as _metrics
from . import optimizers as _opt
from .callbacks import Callback
from .layers import Input, InputLayer, KTensor, Layer, Tensor  # noqa: F401


def _graph_order(outputs: Sequence[KTensor]) -> List[KTensor]:
    order, seen = [], set()

    def visit(t):
        if id(t) in seen:
            return
        seen.add(id(t))
        for i in t.inputs:
            visit(i)
        order.append(t)
    for o in outputs:
        visit(o)
    return order


def _default_config() -> FFConfig:
    """FFConfig with the command line applied (-b, -e, --lr, ... as the
    reference's keras models read it), except under a test runner whose own
    flags are not ours."""
    cfg = FFConfig()
    if "pytest" not in os.path.basename(sys.argv[0] if sys.argv else "") and "pytest" not in sys.modules:
        try:
            cfg.parse_args()
        except SystemExit:
            pass
    return cfg


class BaseModel:
    def __init__(self, name=None):
        self.name = name or "model"
        self.inputs: List[KTensor] = []
        self.outputs: List[KTensor] = []
        self._ff: Optional[FFModel] = None
        self._ffconfig: Optional[FFConfig] = None
        self._optimizer: Optional[_opt.Optimizer] = None
        self._loss: Optional[_losses.Loss] = None
        self._metrics: List[_metrics.Metric] = []
        self._batch: Optional[int] = None
        self._stop = False

    # ---------------------------------------------------------- properties
    @property
    def input(self):
        """The list of input tensors (as the reference returns it)."""
        return list(self.inputs)

    @property
    def output(self):
        return self.outputs[0] if len(self.outputs) == 1 else self.outputs

    @property
    def layers(self) -> List[Layer]:
        """Non-input layers in topological order, each once."""
        out, seen = [], set()
        for t in _graph_order(self.outputs):
            if isinstance(t.layer, InputLayer) or id(t.layer) in seen:
                continue
            seen.add(id(t.layer))
            out.append(t.layer)
        return out

    @property
    def optimizer(self):
        return self._optimizer

    @property
    def ffmodel(self) -> Optional[FFModel]:
        return self._ff

    @property
    def ffconfig(self) -> Optional[FFConfig]:
        return self._ffconfig

    def get_layer(self, name=None, index=None) -> Layer:
        layers = self.layers
        if index is not None:
            if not 0 <= index < len(layers):
                raise ValueError(f"get_layer: index {index} out of range ({len(layers)} layers)")
            return layers[index]
        for l in layers:
            if l.name == name:
                return l
        raise ValueError(f"get_layer: no layer named {name!r}")

    def count_params(self) -> int:
        return sum(l.count_params() for l in self.layers)

    def summary(self, line_length=None, positions=None, print_fn=None) -> str:
        """The model table as a string (the reference returns it; pass
        ``print_fn`` to have it printed as well)."""
        lines = [f'Model: "{self.name}"', f"{'Layer (name)':<24} {'Type':<20} {'Output Shape':<24} Connected to",
                 "=" * 90]
        for t in _graph_order(self.outputs):
            if isinstance(t.layer, InputLayer):
                lines.append(f"{t.layer.name:<24} {'InputLayer':<20} {str(t.shape):<24}")
            else:
                ins = ", ".join(i.layer.name for i in t.inputs)
                lines.append(f"{t.layer.name:<24} {type(t.layer).__name__:<20} {str(t.shape):<24} {ins}")
        lines += ["=" * 90, f"Total params: {self.count_params()}"]
        s = "\n".join(lines)
        if print_fn is not None:
            print_fn(s)
        return s

    # ------------------------------------------------------- nested models
    def __call__(self, x):
        """Apply this model's graph to new input tensors."""
        xs = list(x) if isinstance(x, (list, tuple)) else [x]
        if len(xs) != len(self.inputs):
            raise ValueError(f"{self.name}: expects {len(self.inputs)} inputs, got {len(xs)}")
        env: Dict[int, KTensor] = {id(i): t for i, t in zip(self.inputs, xs)}
        for t in _graph_order(self.outputs):
            if id(t) in env:
                continue
            if isinstance(t.layer, InputLayer):
                raise ValueError(f"{self.name}: output depends on an input that is not a model input")
            env[id(t)] = t.layer([env[id(i)] for i in t.inputs] if len(t.inputs) > 1 else env[id(t.inputs[0])])
        outs = [env[id(o)] for o in self.outputs]
        return outs[0] if len(outs) == 1 else outs

    # ---------------------------------------------------------- compile/fit
    def compile(self, optimizer="sgd", loss=None, metrics=None, loss_weights=None, weighted_metrics=None,
                run_eagerly=None, comp_mode=None, batch_size=None, ffconfig=None, **kw):
        for arg, v in (("loss_weights", loss_weights), ("weighted_metrics", weighted_metrics),
                       ("run_eagerly", run_eagerly)):
            if v is not None:
                raise NotImplementedError(f"compile: {arg} is not supported (as in the reference)")
        if loss is None:
            raise ValueError("compile: loss is required")
        self._optimizer = _opt.get(optimizer)
        self._loss = _losses.get(loss)
        self._metrics = [_metrics.get(m) for m in (metrics or [])]
        self._ffconfig = ffconfig or self._ffconfig or _default_config()
        self._comp_mode = comp_mode
        self._build(int(batch_size or self._ffconfig.batch_size))
        return self

    def _build(self, batch_size: int) -> FFModel:
        if not self.outputs:
            raise ValueError(f"{self.name}: the model has no layers")
        old, old_batch = self._ff, self._batch
        cfg = self._ffconfig
        cfg.batch_size = batch_size
        ff = FFModel(cfg)
        env: Dict[int, object] = {}
        uses: Dict[str, int] = {}
        for layer in self.layers:
            layer._ff_names = []
        # FF inputs in the model's input order (fit() feeds arrays by position)
        for t in self.inputs:
            dt = DataType.DT_INT32 if "int" in t.dtype else DataType.DT_FLOAT
            env[id(t)] = ff.create_tensor([batch_size] + list(t.shape[1:]), dt,
                                          create_grad=dt == DataType.DT_FLOAT, name=t.layer.name)
        for t in _graph_order(self.outputs):
            if id(t) in env:
                continue
            if isinstance(t.layer, InputLayer):
                raise ValueError(f"{self.name}: the output depends on input {t.layer.name}, which is not "
                                 f"among the model's inputs")
            layer = t.layer
            k = uses.get(layer.name, 0)
            uses[layer.name] = k + 1
            saved = layer.name
            if k:   # the same layer object applied again: its own FF op and weights
                layer.name = f"{saved}_{k}"
            try:
                env[id(t)] = layer.build_ff(ff, [env[id(i)] for i in t.inputs])
            finally:
                layer.name = saved
        self._optimizer.create_ffhandle(ff)
        ff.compile(optimizer=self._optimizer.ffhandle, loss_type=self._loss.type,
                   metrics=[m.type for m in self._metrics], comp_mode=self._comp_mode)
        self._ff, self._batch = ff, batch_size
        if old is not None and old_batch != batch_size:
            self._copy_weights(old, ff)
        return ff

    @staticmethod
    def _copy_weights(src: FFModel, dst: FFModel):
        names = set(dst.executor.parameter_names())
        for n in src.executor.parameter_names():
            if n in names:
                dst.executor.set_parameter(n, src.executor.get_parameter(n))

    def _arrays(self, x, y):
        xs = list(x) if isinstance(x, (list, tuple)) else [x]
        if len(xs) != len(self.inputs):
            raise ValueError(f"{self.name}: {len(self.inputs)} inputs, got {len(xs)} arrays")
        xs = [np.asarray(a) for a in xs]
        for a, t in zip(xs, self.inputs):
            if tuple(a.shape[1:]) != tuple(t.shape[1:]):
                raise ValueError(f"input {t.layer.name}: array shape {a.shape[1:]} != model input {t.shape[1:]}")
        y = np.asarray(y)
        if y.ndim == 1:
            y = y.reshape(-1, 1)
        if self._loss.type == LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY:
            y = y.astype(np.int32)
        return xs, y

    def fit(self, x=None, y=None, batch_size=None, epochs=1, verbose=1, callbacks=None, validation_split=0.0,
            validation_data=None, shuffle=True, class_weight=None, sample_weight=None, initial_epoch=0,
            steps_per_epoch=None, **kw):
        if self._ff is None:
            raise RuntimeError("fit: compile the model first")
        for arg, v, dflt in (("validation_split", validation_split, 0.0), ("validation_data", validation_data, None),
                             ("class_weight", class_weight, None), ("sample_weight", sample_weight, None),
                             ("steps_per_epoch", steps_per_epoch, None)):
            if v != dflt:
                raise NotImplementedError(f"fit: {arg} is not supported (as in the reference)")
        if batch_size and batch_size != self._batch:
            self._build(int(batch_size))
        xs, y = self._arrays(x, y)
        callbacks = list(callbacks or [])
        params = {"epochs": epochs, "batch_size": self._batch, "samples": len(y)}
        for cb in callbacks:
            cb.set_params(params)
            cb.set_model(self)
        for cb in callbacks:
            cb.on_train_begin()
        hooks = None
        if any(type(cb).on_batch_begin is not Callback.on_batch_begin or
               type(cb).on_batch_end is not Callback.on_batch_end for cb in callbacks):
            hooks = (lambda it: [cb.on_batch_begin(it) for cb in callbacks],
                     lambda it: [cb.on_batch_end(it) for cb in callbacks])
        hist: List[dict] = []
        self._stop = False
        t0 = time.time()
        for e in range(initial_epoch, epochs):
            for cb in callbacks:
                cb.on_epoch_begin(e)
            self._ff.fit(x=xs, y=y, batch_size=self._batch, epochs=1, batch_hooks=hooks)
            pm = self._ff.get_perf_metrics()
            logs = {"loss": pm.loss, "accuracy": pm.accuracy}
            hist.append(logs)
            for cb in callbacks:
                if cb.on_epoch_end(e, logs) is True:
                    self._stop = True
            if self._stop:
                print(f"Accuracy reaches, now early stop, epoch: {e}")
                break
        el = time.time() - t0
        n = len(y) * len(hist)
        print(f"epochs {len(hist)}, ELAPSED TIME = {el:.4f}s, samples {len(y)}, "
              f"THROUGHPUT = {n / max(el, 1e-9):.2f} samples/s")
        for cb in callbacks:
            cb.on_train_end()
        return History(hist)

    def evaluate(self, x=None, y=None, batch_size=None, verbose=1, callbacks=None, **kw):
        if self._ff is None:
            raise RuntimeError("evaluate: compile the model first")
        if batch_size and batch_size != self._batch:
            self._build(int(batch_size))
        xs, y = self._arrays(x, y)
        return self._ff.eval(x=xs, y=y, batch_size=self._batch)

    def predict(self, x, batch_size=None):
        """Forward pass over ``x`` in batches -> numpy outputs (the last
        partial batch is zero-padded and trimmed)."""
        import torch
        if self._ff is None:
            raise RuntimeError("predict: compile the model first")
        if batch_size and batch_size != self._batch:
            self._build(int(batch_size))
        xs = [np.asarray(a) for a in (x if isinstance(x, (list, tuple)) else [x])]
        n, b = len(xs[0]), self._batch
        ex, outs = self._ff.executor, []
        for s in range(0, n, b):
            feeds = {}
            for t, a in zip(self._ff._inputs, xs):
                chunk = a[s:s + b]
                if len(chunk) < b:
                    chunk = np.concatenate([chunk, np.zeros((b - len(chunk),) + chunk.shape[1:], chunk.dtype)])
                feeds[t.name] = torch.as_tensor(chunk)
            out = ex.forward(feeds, training=False)
            outs.append(out.float().cpu().numpy()[:min(b, n - s)])
        return np.concatenate(outs)

    def get_weights(self):
        ex = self._ff.executor
        return [ex.get_parameter(n).cpu().numpy() for n in ex.parameter_names()]

    def set_weights(self, weights):
        ex = self._ff.executor
        import torch
        for n, w in zip(ex.parameter_names(), weights):
            ex.set_parameter(n, torch.as_tensor(np.asarray(w, np.float32)))


class History(dict):
    """fit() result: ``history["history"]`` is the per-epoch list (the
    existing spelling), ``.history`` maps metric -> per-epoch values (Keras)."""

    def __init__(self, epochs: List[dict]):
        super().__init__(history=epochs)
        self.epochs = epochs

    @property
    def history(self):
        keys = list(self.epochs[0]) if self.epochs else []
        return {k: [e[k] for e in self.epochs] for k in keys}


class Model(BaseModel):
    def __init__(self, inputs=None, outputs=None, name=None):
        super().__init__(name or "model")
        self.inputs = [] if inputs is None else (list(inputs) if isinstance(inputs, (list, tuple)) else [inputs])
        self.outputs = [] if outputs is None else (list(outputs) if isinstance(outputs, (list, tuple)) else [outputs])
        if len(self.outputs) > 1:
            raise NotImplementedError("Model: one output tensor (as in the reference)")


class Sequential(BaseModel):
    def __init__(self, layers: Optional[Sequence] = None, name=None):
        super().__init__(name or "sequential")
        self._items: List = []
        self._input: Optional[KTensor] = None
        for l in layers or []:
            self.add(l)

    def add(self, item):
        """A Layer, a nested Model / Sequential, or a keras ``Input``."""
        if isinstance(item, KTensor):
            if self._items:
                raise ValueError("Sequential: an Input must come first")
            self._input = item
            return
        if self._input is None:
            shp = getattr(item, "input_shape", None)
            if isinstance(item, BaseModel):
                shp = item.inputs[0].shape[1:]
            if shp is None:
                raise ValueError("the first layer needs input_shape= (or add a keras Input first)")
            self._input = Input(tuple(shp))
        self._items.append(item)
        self._rewire()

    def pop(self):
        if not self._items:
            raise TypeError("Sequential.pop: no layers")
        self._items.pop()
        self._rewire()

    def _rewire(self):
        t = self._input
        for l in self._items:
            if isinstance(l, Layer):
                l.inbound, l.outbound = [], []
        for l in self._items:
            t = l(t)
        self.inputs, self.outputs = [self._input], ([t] if self._items else [])
