"""Keras layers (reference: python/flexflow/keras/layers/{base_layer,input_layer,
core,convolutional,pool,normalization,merge}.py).

A layer is a symbolic node until its model is compiled: calling it on
``KTensor``s records the connection and the output shape; ``build_ff`` emits
the FFModel operator(s) when the model is built.  A layer object used in
several places (a nested model applied twice) is built once per use.
"""
from __future__ import annotations

from typing import Dict, List, Optional

import numpy as np

from ...core import ActiMode, AggrMode, DataType, PoolType
from . import initializers as _init

_ACT = {None: ActiMode.AC_MODE_NONE, "linear": ActiMode.AC_MODE_NONE, "relu": ActiMode.AC_MODE_RELU,
        "sigmoid": ActiMode.AC_MODE_SIGMOID, "tanh": ActiMode.AC_MODE_TANH, "gelu": ActiMode.AC_MODE_GELU,
        "softmax": ActiMode.AC_MODE_NONE}


def _pair(v):
    return tuple(v) if isinstance(v, (tuple, list)) else (v, v)


# ------------------------------------------------------------------- tensors
class KTensor:
    """Symbolic tensor (reference keras/models/tensor.py): ``shape`` is the
    batch shape with ``None`` for the batch dimension until the model is
    built."""

    def __init__(self, layer: "Layer", inputs: List["KTensor"], shape, dtype="float32"):
        self.layer, self.inputs, self.shape, self.dtype = layer, list(inputs), tuple(shape), dtype

    @property
    def batch_shape(self):
        return self.shape

    @property
    def num_dims(self):
        return len(self.shape)

    def __repr__(self):
        return f"KTensor({self.layer.name}, shape={self.shape}, dtype={self.dtype})"

    # elementwise arithmetic builds merge layers (reference keras/models/tensor.py)
    def __add__(self, other):
        return Add()([self, other])

    def __sub__(self, other):
        return Subtract()([self, other])

    def __mul__(self, other):
        return Multiply()([self, other])

    def __matmul__(self, other):
        from .backend.internal import batch_dot
        return batch_dot(self, other)

    def __pow__(self, a):
        from .backend.internal import pow as _pow
        return _pow(self, a)


Tensor = KTensor


class Layer:
    _count: Dict[str, int] = {}

    def __init__(self, name: Optional[str] = None, input_shape=None, **kw):
        base = type(self).__name__.lower()
        n = Layer._count.get(base, 0)
        Layer._count[base] = n + 1
        self.name = name or f"{base}_{n}"
        self.input_shape = tuple(input_shape) if input_shape is not None else None
        self.ffhandle = None           # the FFModel layer of the last build
        self._ff_names: List[str] = []  # FF layer names of the weight-bearing op, one per use
        self.inbound: List[List[KTensor]] = []
        self.outbound: List[KTensor] = []

    # --- symbolic connection
    def __call__(self, x):
        xs = list(x) if isinstance(x, (list, tuple)) else [x]
        out = KTensor(self, xs, self.out_shape([t.shape for t in xs]), self.out_dtype([t.dtype for t in xs]))
        self.inbound.append(xs)
        self.outbound.append(out)
        return out

    @property
    def input(self):
        ins = self.inbound[0] if self.inbound else []
        return ins[0] if len(ins) == 1 else ins

    @property
    def output(self):
        return self.outbound[0] if self.outbound else None

    @property
    def output_shape(self):
        return self.output.shape if self.output is not None else None

    def out_shape(self, shapes):
        return shapes[0]

    def out_dtype(self, dtypes):
        return dtypes[0] if dtypes else "float32"

    # --- FFModel emission
    def build_ff(self, ff, ins):
        raise NotImplementedError(type(self).__name__)

    def _emit(self, ff, t):
        """Record the weight-bearing FF layer just added."""
        self.ffhandle = ff.get_last_layer()
        self._ff_names.append(self.ffhandle.name)
        return t

    # --- weights (reference Layer._get_weights / _set_weights)
    def _ff_layer(self, ffmodel):
        if not self._ff_names:
            raise RuntimeError(f"{self.name}: the model holding this layer is not compiled")
        return ffmodel.get_layer_by_name(self._ff_names[-1])

    def get_weights(self, ffmodel):
        """-> [kernel, bias] (or [kernel]) as numpy arrays, in the
        framework's parameter layout."""
        lay = self._ff_layer(ffmodel)
        return [lay.get_parameter_by_id(i).get_weights(ffmodel) for i in range(lay.get_number_parameters())]

    def set_weights(self, ffmodel, kernel, bias=None):
        lay = self._ff_layer(ffmodel)
        lay.get_weight_tensor().set_weights(ffmodel, kernel)
        if bias is not None and lay.get_bias_tensor() is not None:
            lay.get_bias_tensor().set_weights(ffmodel, bias)

    def count_params(self):
        return 0

    def get_summary(self):
        ins = ", ".join(t.layer.name for t in (self.inbound[0] if self.inbound else []))
        return f"{self.name:<24} {type(self).__name__:<20} {str(self.output_shape):<24} {ins}"


class InputLayer(Layer):
    def __init__(self, shape=None, batch_size=None, dtype="float32", name=None):
        super().__init__(name)
        self.shape, self.dtype, self.batch_size = tuple(shape or ()), dtype or "float32", batch_size


def Input(shape=None, batch_size=None, name=None, dtype="float32", sparse=False, tensor=None,  # noqa: N802
          ragged=False, **kw):
    """Symbolic model input; ``shape`` excludes the batch dimension
    (reference keras/layers/input_layer.py)."""
    layer = InputLayer(shape, batch_size, dtype, name)
    t = KTensor(layer, [], (batch_size,) + tuple(shape), layer.dtype)
    layer.outbound.append(t)
    return t


# ---------------------------------------------------------------------- core
class Dense(Layer):
    def __init__(self, units, input_shape=None, activation=None, use_bias=True, kernel_initializer="glorot_uniform",
                 bias_initializer="zeros", kernel_regularizer=None, bias_regularizer=None, activity_regularizer=None,
                 kernel_constraint=None, bias_constraint=None, name=None, **kw):
        if isinstance(input_shape, str):   # Keras order: Dense(units, activation)
            input_shape, activation = None, input_shape
        super().__init__(name, input_shape)
        if activation not in _ACT:
            raise ValueError(f"Dense: unsupported activation {activation!r}")
        self.units, self.activation, self.use_bias = int(units), activation, use_bias
        self.kernel_initializer = _init.get(kernel_initializer)
        self.bias_initializer = _init.get(bias_initializer)
        self.kernel_regularizer = kernel_regularizer

    def out_shape(self, s):
        return s[0][:-1] + (self.units,)

    def count_params(self):
        i = self.inbound[0][0].shape[-1] if self.inbound else 0
        return i * self.units + (self.units if self.use_bias else 0)

    def build_ff(self, ff, ins):
        t = self._emit(ff, ff.dense(ins[0], self.units, _ACT[self.activation], self.use_bias,
                                    kernel_initializer=_init.handle(self.kernel_initializer),
                                    bias_initializer=_init.handle(self.bias_initializer),
                                    kernel_regularizer=self.kernel_regularizer, name=self.name))
        return ff.softmax(t, name=self.name + "_softmax") if self.activation == "softmax" else t


class Conv2D(Layer):
    """NCHW convolution; ``padding`` is "valid", "same" or an explicit
    (pad_h, pad_w) pair as in the reference (keras/layers/convolutional.py)."""

    def __init__(self, filters, input_shape=None, kernel_size=0, strides=(1, 1), padding="valid", data_format=None,
                 dilation_rate=(1, 1), groups=1, activation=None, use_bias=True, kernel_initializer="glorot_uniform",
                 bias_initializer="zeros", kernel_regularizer=None, name=None, **kw):
        # the reference's order is (filters, input_shape, kernel_size); Keras'
        # is (filters, kernel_size): a positional int / pair is a kernel size
        if kernel_size == 0 and (isinstance(input_shape, int) or
                                 (isinstance(input_shape, (tuple, list)) and len(input_shape) == 2)):
            input_shape, kernel_size = None, input_shape
        super().__init__(name, input_shape)
        self.filters, self.k, self.s = int(filters), _pair(kernel_size), _pair(strides)
        if tuple(_pair(dilation_rate)) != (1, 1):
            raise ValueError("Conv2D: dilation_rate != 1 is not supported (as in the reference)")
        self.padding, self.activation, self.use_bias, self.groups = padding, activation, use_bias, groups
        self.kernel_initializer = _init.get(kernel_initializer)
        self.bias_initializer = _init.get(bias_initializer)

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

    def count_params(self):
        c = self.inbound[0][0].shape[1] if self.inbound else 0
        return self.filters * (c // self.groups) * self.k[0] * self.k[1] + (self.filters if self.use_bias else 0)

    def build_ff(self, ff, ins):
        ph, pw = self._pad()
        t = self._emit(ff, ff.conv2d(ins[0], self.filters, self.k[0], self.k[1], self.s[0], self.s[1], ph, pw,
                                     _ACT[self.activation], self.groups, self.use_bias,
                                     kernel_initializer=_init.handle(self.kernel_initializer),
                                     bias_initializer=_init.handle(self.bias_initializer), name=self.name))
        return ff.softmax(t, axis=1, name=self.name + "_softmax") if self.activation == "softmax" else t


class Pooling2D(Layer):
    kind = PoolType.POOL_MAX

    def __init__(self, pool_size=(2, 2), strides=None, padding="valid", data_format=None, pool_type=None, name=None,
                 **kw):
        super().__init__(name)
        self.p = _pair(pool_size)
        self.s = _pair(strides) if strides is not None else self.p
        if pool_type is not None:
            self.kind = pool_type
        if isinstance(padding, (tuple, list)):
            self.pad = tuple(padding)
        else:
            self.pad = (0, 0) if padding == "valid" else ((self.p[0] - 1) // 2, (self.p[1] - 1) // 2)

    def out_shape(self, s):
        b, c, h, w = s[0]
        return (b, c, (h + 2 * self.pad[0] - self.p[0]) // self.s[0] + 1,
                (w + 2 * self.pad[1] - self.p[1]) // self.s[1] + 1)

    def build_ff(self, ff, ins):
        return ff.pool2d(ins[0], self.p[0], self.p[1], self.s[0], self.s[1], self.pad[0], self.pad[1], self.kind,
                         name=self.name)


class MaxPooling2D(Pooling2D):
    kind = PoolType.POOL_MAX


class AveragePooling2D(Pooling2D):
    kind = PoolType.POOL_AVG


class Flatten(Layer):
    def __init__(self, input_shape=None, name=None, **kw):
        super().__init__(name, input_shape)

    def out_shape(self, s):
        return (s[0][0], int(np.prod(s[0][1:])))

    def build_ff(self, ff, ins):
        return ff.flat(ins[0], name=self.name)


class Embedding(Layer):
    """Token embedding.  Keras semantics by default: (B, L) ids -> (B, L, D).
    ``aggr="sum"`` gives the reference keras layer's behaviour (it always
    sum-pools the L embeddings into (B, D), keras/layers/core.py Embedding)."""

    def __init__(self, input_dim, output_dim, embeddings_initializer="uniform", input_length=None, aggr=None,
                 name=None, **kw):
        super().__init__(name)
        self.input_dim, self.output_dim, self.input_length = int(input_dim), int(output_dim), input_length
        self.embeddings_initializer = _init.get(embeddings_initializer)
        self.aggr = {None: AggrMode.AGGR_MODE_NONE, "sum": AggrMode.AGGR_MODE_SUM,
                     "avg": AggrMode.AGGR_MODE_AVG}.get(aggr, aggr)

    def out_shape(self, s):
        if self.aggr != AggrMode.AGGR_MODE_NONE:
            return (s[0][0], self.output_dim)
        return s[0] + (self.output_dim,)

    def out_dtype(self, dtypes):
        return "float32"

    def count_params(self):
        return self.input_dim * self.output_dim

    def build_ff(self, ff, ins):
        return self._emit(ff, ff.embedding(ins[0], self.input_dim, self.output_dim, self.aggr,
                                           kernel_initializer=_init.handle(self.embeddings_initializer),
                                           name=self.name))


class Activation(Layer):
    def __init__(self, activation, name=None, **kw):
        super().__init__(name)
        if activation not in ("relu", "sigmoid", "tanh", "gelu", "elu", "softmax", "linear", None):
            raise ValueError(f"Activation: unsupported {activation!r}")
        self.activation = activation

    def build_ff(self, ff, ins):
        a = self.activation
        if a in (None, "linear"):
            return ff.identity(ins[0], name=self.name)
        fn = {"relu": ff.relu, "sigmoid": ff.sigmoid, "tanh": ff.tanh, "gelu": ff.gelu, "elu": ff.elu,
              "softmax": ff.softmax}[a]
        return fn(ins[0], name=self.name)


class Dropout(Layer):
    def __init__(self, rate, noise_shape=None, seed=0, name=None, **kw):
        super().__init__(name)
        self.rate, self.seed = float(rate), seed or 0

    def build_ff(self, ff, ins):
        return ff.dropout(ins[0], self.rate, self.seed, name=self.name)


class Reshape(Layer):
    """``target_shape`` excludes the batch dimension."""

    def __init__(self, target_shape, input_shape=None, name=None, **kw):
        super().__init__(name, input_shape)
        self.target = tuple(target_shape)

    def out_shape(self, s):
        tgt = list(self.target)
        if -1 in tgt:
            known = int(np.prod([d for d in tgt if d != -1]))
            tgt[tgt.index(-1)] = int(np.prod(s[0][1:])) // known
        return (s[0][0],) + tuple(tgt)

    def build_ff(self, ff, ins):
        return ff.reshape(ins[0], [ins[0].dims[0]] + list(self.out_shape([tuple(ins[0].dims)])[1:]), name=self.name)


class Permute(Layer):
    """Keras form: 1-based ``dims`` over the non-batch axes, e.g. (2, 1);
    the reference's form, a full permutation that keeps axis 0 first, e.g.
    (0, 2, 1), is accepted too (keras/layers/core.py Permute)."""

    def __init__(self, dims, input_shape=None, name=None, **kw):
        super().__init__(name, input_shape)
        dims = tuple(int(d) for d in dims)
        self.perm = dims if 0 in dims else (0,) + dims

    def out_shape(self, s):
        return tuple(s[0][d] for d in self.perm)

    def build_ff(self, ff, ins):
        return ff.transpose(ins[0], list(self.perm), name=self.name)


# ------------------------------------------------------------- normalization
class BatchNormalization(Layer):
    """Batch norm over the channel axis of NCHW input (no fused ReLU: the
    reference keras layer calls FFModel.batch_norm with its relu=True default,
    which is not what Keras' layer computes; docs/PARITY.md)."""

    def __init__(self, axis=1, momentum=0.99, epsilon=1e-3, center=True, scale=True, name=None, **kw):
        super().__init__(name)
        self.axis, self.momentum, self.epsilon = axis, momentum, epsilon

    def build_ff(self, ff, ins):
        return self._emit(ff, ff.batch_norm(ins[0], False, name=self.name))


class LayerNormalization(Layer):
    def __init__(self, axis=-1, epsilon=1e-5, center=True, scale=True, name=None, **kw):
        super().__init__(name)
        self.axes = list(axis) if isinstance(axis, (tuple, list)) else [axis]
        self.eps, self.center, self.scale = epsilon, center, scale

    def build_ff(self, ff, ins):
        return self._emit(ff, ff.layer_norm(ins[0], self.axes, self.scale, self.eps, use_bias=self.center,
                                            name=self.name))


# --------------------------------------------------------------------- merge
class _Merge(Layer):
    op = "add"

    def __init__(self, name=None, **kw):
        super().__init__(name)

    def out_shape(self, s):
        out = list(s[0])
        for x in s[1:]:   # numpy-style broadcast of the non-batch dims
            if len(x) != len(out):
                raise ValueError(f"{type(self).__name__}: inputs of different ranks {s}")
            out = [a if b == 1 else b if a == 1 else a for a, b in zip(out, x)]
        return tuple(out)

    def build_ff(self, ff, ins):
        t = ins[0]
        for i, x in enumerate(ins[1:]):
            t = getattr(ff, self.op)(t, x, name=f"{self.name}_{i}" if len(ins) > 2 else self.name)
        return t


class Add(_Merge):
    op = "add"


class Subtract(_Merge):
    op = "subtract"

    def __call__(self, x):
        if len(x) != 2:
            raise ValueError("Subtract takes exactly two inputs")
        return super().__call__(x)


class Multiply(_Merge):
    op = "multiply"


class Maximum(_Merge):
    op = "max"


class Minimum(_Merge):
    op = "min"


class Concatenate(Layer):
    """Concatenation along ``axis`` (default 1, the reference's default)."""

    def __init__(self, axis=1, name=None, **kw):
        super().__init__(name)
        self.axis = axis

    def out_shape(self, s):
        ax = self.axis % len(s[0])
        out = list(s[0])
        out[ax] = sum(x[ax] for x in s)
        return tuple(out)

    def build_ff(self, ff, ins):
        return ff.concat(list(ins), self.axis, name=self.name)


def concatenate(input_tensors, _axis=1, axis=None):
    return Concatenate(axis if axis is not None else _axis)(input_tensors)


def add(input_tensors):
    return Add()(input_tensors)


def subtract(input_tensors):
    return Subtract()(input_tensors)


def multiply(input_tensors):
    return Multiply()(input_tensors)


def maximum(input_tensors):
    return Maximum()(input_tensors)


def minimum(input_tensors):
    return Minimum()(input_tensors)


__all__ = ["KTensor", "Tensor", "Layer", "InputLayer", "Input", "Dense", "Conv2D", "Pooling2D", "MaxPooling2D",
           "AveragePooling2D", "Flatten", "Embedding", "Activation", "Dropout", "Reshape", "Permute",
           "BatchNormalization", "LayerNormalization", "Add", "Subtract", "Multiply", "Maximum", "Minimum",
           "Concatenate", "concatenate", "add", "subtract", "multiply", "maximum", "minimum"]
