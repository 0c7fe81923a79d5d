"""FFModel: the user-facing model-building / training API.

Parity: python/flexflow/core/flexflow_cffi.py (FFModel :883-2300, Tensor
:574-846, Parameter :849-881, SGDOptimizer/AdamOptimizer :2303-2330,
SingleDataLoader :2449-2490) and the C++ FFModel (lib/runtime/src/
model.h:41-127).  Layers are recorded into the native ComputationGraph
(flexflow_train_amd._ffcore, shape inference in C++); ``compile`` runs the
strategy search (Unity / MCMC / data-parallel, or --import-strategy) to get a
ParallelComputationGraph + machine views and lowers it onto this rank's
Executor; ``fit`` / ``eval`` drive the training loop and report the
reference's "THROUGHPUT = ... samples/s" metric.
"""
from __future__ import annotations

import json
import math
import os
import time
from typing import Dict, List, Optional, Sequence, Union

import numpy as np
import torch

from .. import _ffcore as C
from ..ops.loss import normalize_loss_type, normalize_metric
from ..parallel.comm import DistContext
from ..runtime.executor import ExecConfig, Executor
from ..runtime.optimizer import AdamConfig, SGDConfig
from . import initializers as I
from .config import FFConfig
from .types import (ACTI_TO_STR, AGGR_TO_STR, DT_TO_STR, POOL_TO_STR, ActiMode, AggrMode, CompMode, DataType,
                    LossType, MetricsType, PoolType, STR_TO_DT)

_NP_DT = {"float": np.float32, "double": np.float64, "int32": np.int32, "int64": np.int64, "half": np.float16,
          "bool": np.bool_, "bfloat16": np.float32}


def _dt_str(dt) -> str:
    if dt is None:
        return "float"
    if isinstance(dt, DataType):
        return DT_TO_STR[dt]
    return str(dt)


def _act(a) -> str:
    if a is None:
        return "none"
    if isinstance(a, ActiMode):
        return ACTI_TO_STR[a]
    return str(a)


def _regularizer(r):
    """-> ("none" | "l1" | "l2", lambda) from a regularizer object
    (``.type`` RegularizerMode, ``._lambda``) or a (kind, lambda) pair."""
    if r is None:
        return "none", 0.0
    if isinstance(r, (tuple, list)):
        kind, lam = r
        return str(kind).lower(), float(lam)
    kind = getattr(r, "type", None)
    name = getattr(kind, "name", str(kind)).upper()
    lam = float(getattr(r, "_lambda", getattr(r, "lambda_", 0.0)))
    if name.endswith("L1"):
        return "l1", lam
    if name.endswith("L2"):
        return "l2", lam
    return "none", 0.0


class Tensor:
    def __init__(self, model: "FFModel", vref, name: Optional[str] = None):
        self.model = model
        self.vref = vref
        self.name = name

    @property
    def dims(self):
        if self.vref is None:   # the label tensor: no graph value
            return tuple(getattr(self, "_dims", ()))
        return tuple(self.model.cg.shape(self.vref).dims)

    @property
    def num_dims(self):
        return len(self.dims)

    @property
    def data_type(self):
        return STR_TO_DT.get(C.datatype_to_string(self.model.cg.shape(self.vref).dtype), DataType.DT_FLOAT)

    @property
    def owner_layer(self):
        return self.model._layer_of_node.get(self.vref.node)

    def set_tensor(self, ffmodel, np_array):
        """Attach a value: for inputs it is the next fed batch; for weights it
        overwrites the parameter (see Parameter.set_weights)."""
        ffmodel._pending_feeds[self.name or f"input_{self.vref.node}"] = np.asarray(np_array)

    def get_tensor(self, ffmodel):
        return ffmodel._get_value(self)

    def get_gradients(self, ffmodel, comm_type=None):
        return ffmodel._get_gradient(self)

    def get_model_output_tensor(self, ffmodel):
        return ffmodel._get_value(self)

    def get_model_output_gradients(self, ffmodel, comm_type=None):
        return ffmodel._get_gradient(self)

    # ---- Legion region access (flexflow_cffi.py Tensor.inline_map /
    # attach_numpy_array / get_array ...).  There are no regions here: a
    # "mapped" tensor is a host numpy view of the current value (inputs and
    # the label: the pending feed, others: the last computed value), and
    # attaching an array makes it the next fed batch.  The reference's
    # spellings (ffconfig), (ffmodel, ffconfig) and (ffconfig, data_type) are
    # all accepted.
    def _args(self, args):
        m, rest = self.model, list(args)
        if rest and isinstance(rest[0], FFModel):
            m = rest.pop(0)
        if rest and isinstance(rest[0], FFConfig):
            rest.pop(0)
        return m, rest

    def _feed_key(self):
        return self.name or f"input_{self.vref.node}"

    def _host_value(self, m):
        """Current value; an input / label with nothing fed yet gets a zero
        array that becomes its pending feed (writes into it are seen)."""
        v = m._get_value(self)
        if v is not None:
            return v
        is_input = any(t is self or t.name == self.name for t in m._inputs) or self.name == "label"
        if not is_input:
            return None
        dims = m._label_dims() if self.vref is None else list(self.dims)
        dt = DataType.DT_INT32 if self.name == "label" and m._sparse_labels() else self.data_type
        arr = np.zeros(dims, dtype=_NP_DT[_dt_str(dt)])
        m._pending_feeds[self._feed_key()] = arr
        return arr

    def inline_map(self, *args):
        m, _ = self._args(args)
        self._mapped = self._host_value(m)
        return self._mapped

    def inline_unmap(self, *args):
        self._mapped = None

    def is_mapped(self):
        return getattr(self, "_mapped", None) is not None

    def get_array(self, *args):
        m, _ = self._args(args)
        a = self._mapped if self.is_mapped() else self._host_value(m)
        return None if a is None else np.asarray(a)

    def get_flat_array(self, *args):
        a = self.get_array(*args)
        return None if a is None else a.reshape(-1)

    def attach_numpy_array(self, *args):
        m, rest = self._args(args)
        self.set_tensor(m, rest[-1])

    def detach_numpy_array(self, *args):
        m, _ = self._args(args)
        m._pending_feeds.pop(self._feed_key(), None)

    def __repr__(self):
        return f"Tensor({self.name}, dims={self.dims})"


class Parameter(Tensor):
    def set_weights(self, ffmodel, np_array):
        ffmodel.executor.set_parameter(self.name, torch.as_tensor(np.asarray(np_array, dtype=np.float32)))
        return True

    def get_weights(self, ffmodel):
        return ffmodel.executor.get_parameter(self.name).cpu().numpy()


class Layer:
    def __init__(self, model: "FFModel", node: int, name: str, op_type: str):
        self.model = model
        self.node = node
        self.name = name
        self.op_type = op_type

    def _weights(self):
        return [Parameter(self.model, v, self.model.cg.layer_name(v.node)) for v in self.model.cg.layer_weights(self.node)]

    def get_number_parameters(self):
        return len(self._weights())

    def get_parameter_by_id(self, i):
        return self._weights()[i]

    def get_weight_tensor(self):
        return self._weights()[0]

    def get_bias_tensor(self):
        w = self._weights()
        return w[1] if len(w) > 1 else None

    def get_number_inputs(self):
        return len(self.model.cg.layer_data_inputs(self.node))

    def get_input_by_id(self, i):
        v = self.model.cg.layer_data_inputs(self.node)[i]
        for t in self.model._inputs:   # a model input: the same tensor object (its feed name)
            if t.vref.node == v.node and t.vref.idx == v.idx:
                return t
        return Tensor(self.model, v)

    def get_input_tensor_by_id(self, i):
        return self.get_input_by_id(i)

    def get_input_tensor(self):
        return self.get_input_by_id(0)

    def get_number_outputs(self):
        return self.model.cg.num_outputs(self.node)

    def get_output_by_id(self, i):
        return Tensor(self.model, C.ValueRef(self.node, i))

    def get_output_tensor(self):
        return self.get_output_by_id(0)

    def __repr__(self):
        return f"Layer({self.name}, {self.op_type})"


class SGDOptimizer:
    def __init__(self, ffmodel=None, lr=0.01, momentum=0.0, nesterov=False, weight_decay=0.0):
        self.cfg = SGDConfig(lr, momentum, nesterov, weight_decay)

    def set_learning_rate(self, learning_rate):
        self.cfg.lr = learning_rate


class AdamOptimizer:
    def __init__(self, ffmodel=None, alpha=0.001, beta1=0.9, beta2=0.999, weight_decay=0.0, epsilon=1e-8,
                 decoupled=False):
        self.cfg = AdamConfig(alpha, beta1, beta2, weight_decay, epsilon, decoupled)

    def set_learning_rate(self, learning_rate):
        self.cfg.lr = learning_rate


def _param_sync_str(v) -> str:
    """FFConfig.parameter_sync: "nccl" / "ps" or a ParameterSyncType."""
    name = getattr(v, "name", str(v)).lower()
    return "ps" if name in ("ps", "parameter_server") else "nccl"


class SingleDataLoader:
    """Holds the full dataset on the host and yields global batches (the
    executor keeps only this rank's piece).  Parity: flexflow_cffi.py:2449."""

    def __init__(self, ffmodel, input, full_input, num_samples=None, data_type=None):
        self.model = ffmodel
        self.tensor = input
        self.full = np.asarray(full_input)
        self._num_samples = int(num_samples if num_samples is not None else self.full.shape[0])
        self.batch_size = ffmodel.ffconfig.batch_size
        self.idx = 0

    @property
    def num_samples(self):
        return self._num_samples

    @num_samples.setter
    def num_samples(self, v):
        self._num_samples = int(v)

    def reset(self):
        self.idx = 0

    def next_batch(self, ffmodel=None):
        """Next global batch; also attached to the loader's tensor so a
        following ``ffmodel.forward()`` consumes it (reference semantics)."""
        b = self.batch_size
        if self.idx + b > self._num_samples:
            self.idx = 0
        out = self.full[self.idx:self.idx + b]
        self.idx += b
        if self.tensor is not None:
            (ffmodel or self.model)._pending_feeds[self.tensor.name or f"input_{self.tensor.vref.node}"] = out
        return out


class FFModel:
    def __init__(self, ffconfig: Optional[FFConfig] = None):
        self.ffconfig = ffconfig or FFConfig()
        self.cg = C.ComputationGraph()
        self._layers: List[Layer] = []
        self._layer_of_node: Dict[int, Layer] = {}
        self._inputs: List[Tensor] = []
        self._optimizer = None
        self.executor: Optional[Executor] = None
        self.loss_type = None
        self.metrics: List[str] = []
        self._pending_feeds: Dict[str, np.ndarray] = {}
        self._constants: Dict[str, np.ndarray] = {}
        self._traces: Dict[int, dict] = {}
        self._active_trace: Optional[dict] = None
        self.ffconfig._models.append(self)
        self._label_tensor: Optional[Tensor] = None
        self._last_labels = None
        self._name_counter = 0
        self.dist: Optional[DistContext] = None
        self.pcg = None
        self.views = {}
        self.search_report: Dict = {}
        self.valid_classes = None

    # ------------------------------------------------------------------ utils
    def _uname(self, name, prefix):
        if name:
            return name
        self._name_counter += 1
        return f"{prefix}_{self._name_counter}"

    def _add(self, op_type: str, inputs: Sequence[Tensor], name=None, inits=(), **attrs):
        op = C.OpAttrs(op_type, **attrs)
        nm = self._uname(name, op_type.lower())
        outs = self.cg.add_layer(op, [t.vref for t in inputs], nm, [i.to_json() if hasattr(i, "to_json") else (i or "")
                                                                    for i in inits])
        node = outs[0].node
        layer = Layer(self, node, nm, op_type)
        self._layers.append(layer)
        self._layer_of_node[node] = layer
        res = [Tensor(self, v, nm) for v in outs]
        return res[0] if len(res) == 1 else res

    def get_layers(self):
        return list(self._layers)

    def get_layer_by_id(self, layer_id):
        return self._layers[layer_id]

    def get_last_layer(self):
        return self._layers[-1]

    def get_layer_by_name(self, layer_name):
        for l in self._layers:
            if l.name == layer_name:
                return l
        return None

    def get_tensor_by_id(self, id):
        return self._layers[id].get_output_tensor()

    def print_layers(self, id=-1):
        for i, l in enumerate(self._layers):
            if id in (-1, i):
                outs = [tuple(self.cg.shape(C.ValueRef(l.node, k)).dims) for k in range(self.cg.num_outputs(l.node))]
                print(f"layer[{i}] {l.name} {l.op_type} outputs={outs}")

    # --------------------------------------------------------------- inputs
    def create_tensor(self, dims, data_type=DataType.DT_FLOAT, create_grad=True, name=None):
        dt = _dt_str(data_type)
        nm = self._uname(name, "input")
        v = self.cg.create_input(C.TensorShape(list(dims), C.datatype_from_string(dt)), bool(create_grad), nm)
        t = Tensor(self, v, nm)
        self._inputs.append(t)
        return t

    def create_constant(self, dims, value, data_type=DataType.DT_FLOAT, name=None):
        """A constant tensor filled with ``value`` (not trainable, never fed)."""
        return self.create_constant_array(np.full(dims, value, dtype=_NP_DT[_dt_str(data_type)]), name=name)

    def create_constant_array(self, array, name=None):
        """A constant tensor holding ``array`` (e.g. position buckets or masks
        folded by a frontend): an executor input that is placed on the device
        once and never fed by data loaders."""
        arr = np.ascontiguousarray(array)
        dt = {np.dtype(np.float32): DataType.DT_FLOAT, np.dtype(np.float64): DataType.DT_FLOAT,
              np.dtype(np.int32): DataType.DT_INT32, np.dtype(np.int64): DataType.DT_INT64,
              np.dtype(np.float16): DataType.DT_HALF, np.dtype(np.bool_): DataType.DT_BOOLEAN}[arr.dtype]
        if arr.dtype == np.float64:
            arr = arr.astype(np.float32)
        t = self.create_tensor(list(arr.shape), dt, create_grad=False, name=self._uname(name, "constant"))
        self._inputs.remove(t)       # not a fed input
        self.cg.set_input_replicated(t.vref.node)   # no sample dimension: replicated under data parallelism
        self._constants[t.name] = arr
        t._constant = True
        return t

    # --------------------------------------------------------------- layers
    def exp(self, x, name=None):
        return self._add("EXP", [x], name)

    def sin(self, x, name=None):
        return self._add("SIN", [x], name)

    def cos(self, x, name=None):
        return self._add("COS", [x], name)

    def add(self, x, y, inplace_a=False, name=None):
        return self._add("EW_ADD", [x, y], name)

    def subtract(self, x, y, inplace_a=False, name=None):
        return self._add("EW_SUB", [x, y], name)

    def multiply(self, x, y, inplace_a=False, name=None):
        return self._add("EW_MUL", [x, y], name)

    def divide(self, x, y, inplace_a=False, name=None):
        return self._add("EW_DIV", [x, y], name)

    def max(self, x, y, inplace_a=False, name=None):
        return self._add("EW_MAX", [x, y], name)

    def min(self, x, y, inplace_a=False, name=None):
        return self._add("EW_MIN", [x, y], name)

    def reduce_sum(self, input, axes, keepdims=False, name=None):
        return self._add("REDUCE_SUM", [input], name, axes=list(axes), keepdims=keepdims)

    def rsqrt(self, input, name=None):
        return self._add("RSQRT", [input], name)

    def pow(self, input, exponent, name=None):
        return self._add("POW", [input], name, exponent=float(exponent))

    def mean(self, input, dims, keepdims=False, name=None):
        return self._add("REDUCE_MEAN", [input], name, axes=list(dims), keepdims=keepdims)

    def conv2d(self, input, out_channels, kernel_h, kernel_w, stride_h, stride_w, padding_h, padding_w,
               activation=ActiMode.AC_MODE_NONE, groups=1, use_bias=True, shared_op=None, kernel_initializer=None,
               bias_initializer=None, name=None):
        return self._add("CONV2D", [input], name, (kernel_initializer, bias_initializer), out_channels=out_channels,
                         kernel_h=kernel_h, kernel_w=kernel_w, stride_h=stride_h, stride_w=stride_w,
                         padding_h=padding_h, padding_w=padding_w, activation=_act(activation), groups=groups,
                         use_bias=use_bias)

    def embedding(self, input, num_embeddings, embedding_dim, aggr=AggrMode.AGGR_MODE_NONE,
                  dtype=DataType.DT_FLOAT, shared_op=None, kernel_initializer=None, name=None):
        aggr_s = AGGR_TO_STR[aggr] if isinstance(aggr, AggrMode) else str(aggr)
        return self._add("EMBEDDING", [input], name, (kernel_initializer,), num_entries=num_embeddings,
                         out_channels=embedding_dim, aggr=aggr_s, data_type=_dt_str(dtype))

    def pool2d(self, input, kernel_h, kernel_w, stride_h, stride_w, padding_h, padding_w, pool_type=PoolType.POOL_MAX,
               activation=ActiMode.AC_MODE_NONE, name=None):
        return self._add("POOL2D", [input], name, kernel_h=kernel_h, kernel_w=kernel_w, stride_h=stride_h,
                         stride_w=stride_w, padding_h=padding_h, padding_w=padding_w,
                         pool_type=POOL_TO_STR[pool_type] if isinstance(pool_type, PoolType) else str(pool_type),
                         activation=_act(activation))

    def batch_norm(self, input, relu=True, name=None):
        return self._add("BATCHNORM", [input], name, relu=relu)

    def layer_norm(self, input, axes, elementwise_affine=True, eps=1e-5, use_bias=True, name=None):
        return self._add("LAYERNORM", [input], name, axes=list(axes), elementwise_affine=elementwise_affine,
                         eps=float(eps), use_bias=use_bias)

    def batch_matmul(self, A, B, a_seq_length_dim=None, b_seq_length_dim=None, name=None):
        return self._add("BATCHMATMUL", [A, B], name,
                         a_seq_length_dim=-1 if a_seq_length_dim is None else a_seq_length_dim,
                         b_seq_length_dim=-1 if b_seq_length_dim is None else b_seq_length_dim)

    def dense(self, input, out_dim, activation=ActiMode.AC_MODE_NONE, use_bias=True, datatype=None, shared_op=None,
              kernel_initializer=None, bias_initializer=None, kernel_regularizer=None, name=None):
        """Linear layer.  ``kernel_regularizer`` (an object with ``type`` =
        RegularizerMode and ``_lambda``, e.g. flexflow.keras.regularizers.L2,
        or a ("l1" | "l2", lambda) pair) adds lambda * W (L2) or
        lambda * sign(W) (L1) to the kernel gradient, as the reference's
        Linear backward does (linear_kernels.cu:258, cublasSgeam dW += lambda W)."""
        reg, lam = _regularizer(kernel_regularizer)
        return self._add("LINEAR", [input], name, (kernel_initializer, bias_initializer), out_channels=out_dim,
                         activation=_act(activation), use_bias=use_bias, regularizer=reg, regularizer_lambda=lam)

    def concat(self, tensors, axis, name=None):
        return self._add("CONCAT", list(tensors), name, axis=axis)

    def split(self, input, sizes, axis, name=None):
        if isinstance(sizes, int):
            n = input.dims[axis]
            sizes = [n // sizes] * sizes
        out = self._add("SPLIT", [input], name, axis=axis, splits=list(sizes))
        return out if isinstance(out, list) else [out]

    def flat(self, input, name=None):
        return self._add("FLAT", [input], name)

    def softmax(self, input, axis=-1, name=None):
        return self._add("SOFTMAX", [input], name, dim=axis)

    def reshape(self, input, shape, name=None):
        return self._add("RESHAPE", [input], name, shape=list(shape))

    def gather(self, input, index, dim, name=None):
        return self._add("GATHER", [input, index], name, dim=dim)

    def transpose(self, input, perm, name=None):
        return self._add("TRANSPOSE", [input], name, perm=list(perm))

    def reverse(self, input, axis, name=None):
        return self._add("REVERSE", [input], name, axis=axis)

    def scalar_multiply(self, input, scalar, inplace=True, name=None):
        return self._add("SCALAR_MULTIPLY", [input], name, scalar=float(scalar))

    def scalar_add(self, input, scalar, inplace=True, name=None):
        return self._add("SCALAR_ADD", [input], name, scalar=float(scalar))

    def scalar_sub(self, input, scalar, inplace=True, name=None):
        return self._add("SCALAR_SUB", [input], name, scalar=float(scalar))

    def scalar_true_divide(self, input, scalar, inplace=True, name=None):
        return self._add("SCALAR_TRUE_DIV", [input], name, scalar=float(scalar))

    def gelu(self, input, inplace=True, name=None):
        return self._add("GELU", [input], name)

    def relu(self, input, inplace=True, name=None):
        return self._add("RELU", [input], name)

    def identity(self, input, name=None):
        return self._add("IDENTITY", [input], name)

    def sigmoid(self, input, name=None):
        return self._add("SIGMOID", [input], name)

    def tanh(self, input, name=None):
        return self._add("TANH", [input], name)

    def elu(self, input, inplace=True, name=None):
        return self._add("ELU", [input], name)

    def dropout(self, input, rate, seed, name=None):
        return self._add("DROPOUT", [input], name, rate=float(rate), seed=int(seed))

    def multihead_attention(self, query, key, value, embed_dim, num_heads, kdim=0, vdim=0, dropout=0.0, bias=True,
                            add_bias_kv=False, add_zero_attn=False, kernel_initializer=None, causal=False, name=None,
                            seq_parallel_mode="auto"):
        """``seq_parallel_mode`` selects the lowering when a strategy shards
        the sequence dim: "ulysses" (all-to-all), "ring" or "auto"."""
        return self._add("MULTIHEAD_ATTENTION", [query, key, value], name, (kernel_initializer,),
                         embed_dim=embed_dim, num_heads=num_heads, kdim=kdim, vdim=vdim, dropout=float(dropout),
                         bias=bias, add_bias_kv=add_bias_kv, add_zero_attn=add_zero_attn, causal=causal,
                         seq_parallel_mode=seq_parallel_mode)

    def experts(self, input, expert_ids, gate_weights, num_experts, hidden_size, out_dim=None,
                activation=ActiMode.AC_MODE_RELU, use_bias=True, expert_parallel_mode="replicated", name=None):
        """Routed expert FFN block: ``input`` [B, D], ``expert_ids`` /
        ``gate_weights`` [B, k] (e.g. the indices / values of ``top_k``)."""
        out_dim = out_dim or input.dims[-1]
        return self._add("EXPERTS", [input, expert_ids, gate_weights], name, num_experts=num_experts,
                         hidden_size=hidden_size, out_dim=out_dim, activation=_act(activation), use_bias=use_bias,
                         expert_parallel_mode=expert_parallel_mode)

    def moe(self, input, num_exp, num_select, expert_hidden_size, alpha=2.0, lambda_bal=0.04, out_dim=None,
            expert_parallel_mode="replicated", name=None):
        """Mixture of experts (reference: examples/cpp/mixture_of_experts/
        moe.cc:159-164): softmax gate -> top-k -> routed experts.  ``alpha``
        (capacity factor) and ``lambda_bal`` (balance loss) are accepted for
        API parity; routing here is dropless."""
        nm = name or self._uname(None, "moe")
        gate = self.softmax(self.dense(input, num_exp, name=f"{nm}.gate"), name=f"{nm}.gate_softmax")
        vals, idx = self.top_k(gate, num_select, True, name=f"{nm}.topk")
        return self.experts(input, idx, vals, num_exp, expert_hidden_size, out_dim=out_dim,
                            expert_parallel_mode=expert_parallel_mode, name=f"{nm}.experts")

    def cast(self, input, dtype, name=None):
        return self._add("CAST", [input], name, dtype=_dt_str(dtype))

    def top_k(self, input, k, sorted=True, name=None):
        return self._add("TOPK", [input], name, k=k, sorted=sorted)

    # ------------------------------------------------------------- training
    @property
    def optimizer(self):
        return self._optimizer

    @optimizer.setter
    def optimizer(self, opt):
        self._optimizer = opt

    def set_optimizer(self, optimizer):
        self._optimizer = optimizer

    @property
    def label_tensor(self):
        return self._label_tensor

    def compile(self, optimizer=None, loss_type=None, metrics=None, comp_mode=None, output=None):
        from ..search import strategy as strat

        if optimizer is not None:
            self._optimizer = optimizer
        if self._optimizer is None:
            self._optimizer = SGDOptimizer(self, lr=self.ffconfig.learning_rate)
        self.loss_type = loss_type
        self.metrics = [normalize_metric(m) for m in (metrics or [])]
        cuda = torch.cuda.is_available() and not self.ffconfig.cpu_only and not self.ffconfig.local_execution
        local_rank = int(os.environ.get("LOCAL_RANK", "0"))
        if cuda and local_rank >= torch.cuda.device_count():
            # more ranks than GPUs (gloo rehearsal of a multi-GPU run on one
            # card).  RCCL cannot put two ranks on one GPU: refuse before any
            # process-group init instead of hanging inside it.
            if os.environ.get("FF_DIST_BACKEND", "").lower() != "gloo":
                raise RuntimeError(
                    f"LOCAL_RANK {local_rank} >= {torch.cuda.device_count()} visible GPUs: launch at most one rank "
                    "per GPU, or set FF_DIST_BACKEND=gloo to rehearse several ranks on a shared GPU")
            local_rank %= torch.cuda.device_count()
        device = torch.device(f"cuda:{local_rank}") if cuda else torch.device("cpu")
        if cuda:
            torch.cuda.set_device(device)
        self.dist = DistContext.from_env(device=device)
        world = self.dist.world
        self.pcg, self.views, self.search_report = strat.build_pcg(self.cg, self.ffconfig, world)
        if self.ffconfig.export_strategy_file:
            strat.export_strategy(self.ffconfig.export_strategy_file, self.pcg, self.views, self.search_report)
        # "bfloat16" is the GPU default and means fp32 on the CPU; a CPU run
        # computes in bf16 only when asked by name ("bfloat16-cpu")
        dt = self.ffconfig.compute_dtype
        if dt == "bfloat16-cpu":
            dt = "bfloat16"
        elif not cuda and dt == "bfloat16":
            dt = "float"
        cdt = {"bfloat16": torch.bfloat16, "float": torch.float32, "float32": torch.float32,
               "half": torch.float16}[dt]
        cfg = ExecConfig(compute_dtype=cdt, device=device, seed=self.ffconfig.seed,
                         profiling=self.ffconfig.profiling, fuse_add_layernorm=self.ffconfig.perform_fusion,
                         shard_optimizer=bool(self.ffconfig.shard_optimizer),
                         param_sync=_param_sync_str(self.ffconfig.parameter_sync),
                         bucket_bytes=int(self.ffconfig.bucket_mb) << 20,
                         inplace=bool(self.ffconfig.enable_inplace_optimizations))
        if self.ffconfig.softmax_identity_backward:
            cfg.softmax_identity_backward = True
        out_v = None
        if output is not None:
            out_v = self._pcg_value_of(output)
        self.executor = Executor(self.pcg, self.dist, cfg, views=self.views,
                                 loss_type=normalize_loss_type(loss_type) if loss_type is not None else None,
                                 metrics=self.metrics, optimizer=self._optimizer.cfg, output=out_v,
                                 valid_classes=self.valid_classes)
        self.executor.init_parameters()
        self.executor.constants = dict(self._constants)
        if (getattr(self.ffconfig, "device_arena", False) and self.executor.cfg.device.type == "cuda"
                and self.dist.world == 1):
            # the step's activations / gradients / workspaces out of one
            # plan-sized device region (runtime/arena.py, csrc/runtime/arena.cpp)
            from ..runtime import arena as _arena
            self.executor.enable_arena(_arena.plan_bytes(
                self.pcg, self.views, 1, 0, _arena.bytes_per_param(self._optimizer.cfg),
                self.executor.cfg.compute_dtype == torch.bfloat16))
        self.local_backing = None
        if self.ffconfig.local_execution:
            self._init_local_backing(loss_type)
        # label tensor (reference: created in compile, [batch, 1] int32 for sparse CE)
        out_lay = self.executor.value_layout[self.executor.loss_value]
        if loss_type is not None:
            sparse = normalize_loss_type(loss_type) == "sparse_categorical_crossentropy"
            ldims = list(out_lay.sizes[:-1]) + [1] if sparse else list(out_lay.sizes)
            self._label_tensor = Tensor(self, None, "label")
            self._label_tensor._dims = tuple(ldims)
        return self

    def _pcg_value_of(self, t: Tensor):
        mapping = self.search_report.get("cg_to_pcg", {})
        if t.vref.node in mapping:
            return (mapping[t.vref.node], t.vref.idx)
        return None

    def prefetch(self):
        """Reference: Legion prefetch of the next batch's regions.  The native
        loader (runtime/dataloader.py) already stages batches ahead; no-op."""
        return None

    def add_layer(self, op_type, name=None, inputs=(), **attrs):
        """Generic layer constructor (reference: FFModel.add_layer / _add_to_model):
        any operator of the IR by type name with attributes."""
        t = op_type if isinstance(op_type, str) else getattr(op_type, "name", str(op_type))
        if t.startswith("OP_"):
            t = t[3:]
        return self._add(t, list(inputs), name, **attrs)

    def init_layers(self):
        if self.executor is None:
            raise RuntimeError("call compile() first")

    def reset_metrics(self):
        self.executor.zero_metrics()

    def get_perf_metrics(self):
        return self.executor.perf_metrics()

    def compute_metrics(self):
        return self.get_perf_metrics()

    def create_data_loader(self, batch_tensor, full_array):
        return SingleDataLoader(self, batch_tensor, full_array, full_array.shape[0])

    def _feeds_from(self, batch_inputs: Dict[str, np.ndarray]):
        return {k: torch.as_tensor(v) for k, v in batch_inputs.items()}

    # ---- Legion-trace equivalent: hipGraph capture of a traced iteration.
    # ``ffconfig.begin_trace(id) ... forward/zero_gradients/backward/update
    # ... ffconfig.end_trace(id)`` (flexflow_cffi.py:562-566, used around
    # every iteration of the reference's training loops) runs the first
    # traced iteration eagerly (autotuning, allocator warm-up), captures the
    # second one into a hipGraph and replays it from then on: forward() feeds
    # the batch into the graph's static buffers and replays the whole
    # iteration; backward()/update()/zero_gradients() inside the trace are
    # then already done.
    def _trace_begin(self, trace_id: int):
        st = self._traces.setdefault(trace_id, {"count": 0, "step": None})
        st["count"] += 1
        st["done"] = False
        self._active_trace = st

    def _trace_end(self, trace_id: int):
        self._active_trace = None

    def _traced(self) -> bool:
        st = self._active_trace
        return bool(st and st.get("done"))

    def _graph_capable(self) -> bool:
        ex = self.executor
        return (ex is not None and ex.cfg.device.type == "cuda" and ex.cfg.grad_clip <= 0
                and self.dist.world == 1)

    def forward(self, seq_length=None):
        feeds = dict(self._pending_feeds)
        st = self._active_trace
        if st is not None and self._graph_capable() and "label" in feeds:
            lab = torch.as_tensor(feeds.pop("label"))
            tfeeds = self._feeds_from({k: v for k, v in feeds.items() if k in self.executor.inputs})
            if st["step"] is None and st["count"] >= 2:
                st["step"] = self.executor.make_graphed_train_step(tfeeds, lab, warmup=0)
            if st["step"] is not None:
                st["step"](tfeeds, lab)
                st["done"] = True
                return
        feeds = {k: v for k, v in feeds.items() if k in self.executor.inputs}
        self.executor.forward(self._feeds_from(feeds), training=True)

    def backward(self, seq_length=None):
        if self._traced():
            return
        lab = self._pending_feeds.get("label")
        g = self.executor.compute_loss(torch.as_tensor(lab) if lab is not None else None)
        self.executor.backward(g)

    def update(self):
        if self._traced():
            return
        self.executor.update(lr=self._optimizer.cfg.lr)

    def zero_gradients(self):
        if self._traced():
            return
        self.executor.zero_gradients()

    def _input_name(self, t):
        return t.name

    def fit(self, x=None, y=None, batch_size=None, epochs=1, batch_hooks=None):
        """Training loop over data loaders (or arrays).  Prints the
        reference's ``ELAPSED TIME = ..., THROUGHPUT = ... samples/s``.
        ``batch_hooks`` = (begin(it), end(it)) callables run around every
        iteration (the keras frontend's per-batch callbacks)."""
        ex = self.executor
        xs = x if isinstance(x, (list, tuple)) else [x]
        bs = batch_size or self.ffconfig.batch_size
        if getattr(self, "local_backing", None) is not None:
            return self._fit_local(xs, y, bs, epochs, batch_hooks)
        mb = max(1, int(getattr(self.ffconfig, "micro_batches", 1) or 1))
        native = self._native_loader(xs, y, bs) if mb == 1 else None
        if native is not None:
            return self._fit_native(native, epochs, batch_hooks)
        loaders = [d if isinstance(d, SingleDataLoader) else SingleDataLoader(self, self._inputs[i], d)
                   for i, d in enumerate(xs)]
        ylo = y if isinstance(y, SingleDataLoader) else SingleDataLoader(self, self._label_tensor, y)
        for l in loaders + [ylo]:
            l.batch_size = bs
        num_samples = ylo.num_samples
        iters = num_samples // bs
        use_graph = bool(self.ffconfig.enable_hipgraph) and self._graph_capable() and mb == 1
        graphed = None
        pending = []    # micro-batches of the current optimizer step (mb > 1)
        start_epoch, start_it = self._resume_fit(iters)
        ex.zero_metrics()
        if ex.cfg.device.type == "cuda":
            torch.cuda.synchronize()
        t0 = time.time()
        first = True
        for epoch in range(start_epoch, epochs):
            for l in loaders + [ylo]:
                l.reset()
            ex.zero_metrics()
            skip = start_it if epoch == start_epoch else 0
            for _ in range(skip):   # resumed mid-epoch: the batches already trained on
                for l in loaders + [ylo]:
                    l.next_batch()
            for it in range(skip, iters):
                if batch_hooks:
                    batch_hooks[0](it)
                feeds = {self._inputs[i].name: torch.as_tensor(l.next_batch()) for i, l in enumerate(loaders)}
                labels = torch.as_tensor(ylo.next_batch())
                if mb > 1:
                    # FFConfig.micro_batches: mb batches per optimizer step, in
                    # GPipe order over the searched pipeline stages
                    pending.append((feeds, labels))
                    if len(pending) == mb or it == iters - 1:
                        ex.train_step_pipelined([f for f, _ in pending], [l for _, l in pending],
                                                lr=self._optimizer.cfg.lr)
                        pending = []
                elif use_graph and not first:
                    # the first iteration ran eagerly (autotune / allocator
                    # warm-up); capture the next one and replay it from then on
                    if graphed is None:
                        graphed = ex.make_graphed_train_step(feeds, labels, warmup=0)
                    graphed(feeds, labels)
                else:
                    ex.train_step(feeds, labels, lr=self._optimizer.cfg.lr)
                first = False
                if not pending:   # checkpoints only between optimizer steps
                    self._after_fit_step(epoch, it, iters)
                if batch_hooks:
                    batch_hooks[1](it)
                # perf_metrics() all-reduces across ranks: every rank calls it, rank 0 prints
                if self.ffconfig.print_freq and (it + 1) % self.ffconfig.print_freq == 0:
                    pm = ex.perf_metrics()
                    if self.dist.rank == 0:
                        print(f"epoch {epoch} iter {it + 1}/{iters}: {pm}", flush=True)
            if iters:
                pm = ex.perf_metrics()
                if self.dist.rank == 0:
                    print(f"epoch {epoch}: {pm}", flush=True)
        if ex.cfg.device.type == "cuda":
            torch.cuda.synchronize()
        elapsed = time.time() - t0
        thr = num_samples * epochs / max(elapsed, 1e-9)
        if self.dist.rank == 0:
            print(f"ELAPSED TIME = {elapsed:.4f}s, THROUGHPUT = {thr:.2f} samples/s", flush=True)
        self.last_throughput = thr
        return thr

    # ------------------------------------------------------------ fault tolerance
    def _resume_fit(self, iters: int):
        """FFConfig.checkpoint_dir: load the newest complete step checkpoint
        and return the (epoch, iteration) fit() continues from."""
        d = self.ffconfig.checkpoint_dir
        if not d:
            return 0, 0
        from ..utils.checkpoint import latest_checkpoint, load_checkpoint, read_checkpoint_meta
        path = latest_checkpoint(d)
        if path is None:
            return 0, 0
        # check the progress record BEFORE restoring anything: a checkpoint of
        # a differently-sized epoch is not resumed (no weights, no step count)
        cmeta = read_checkpoint_meta(path)
        prog = cmeta.get("progress") or {}
        if prog.get("iters_per_epoch") != iters:
            import warnings
            warnings.warn(f"{path}: recorded {prog.get('iters_per_epoch')} iterations per epoch, this fit() runs "
                          f"{iters}; not resuming from it (training starts from the current weights)")
            # new checkpoints must sort after the stale one: otherwise the
            # keep-newest rotation deletes them and latest_checkpoint() keeps
            # returning the mismatched directory
            self.executor.step_num = max(self.executor.step_num, int(cmeta.get("step", 0)))
            return 0, 0
        meta = load_checkpoint(self, path)
        epoch, it = int(prog["epoch"]), int(prog["iter"])
        if it >= iters:
            epoch, it = epoch + 1, 0
        if self.dist.rank == 0:
            print(f"resumed from {path}: epoch {epoch} iteration {it} (step {meta['step']})", flush=True)
        return epoch, it

    def _after_fit_step(self, epoch: int, it: int, iters: int):
        """Periodic atomic checkpoint; FF_FAULT_INJECT_STEP=N raises right
        after executor step N (a failed-rank stand-in for the resume tests)."""
        cfg = self.ffconfig
        g = epoch * iters + it + 1
        if cfg.checkpoint_dir and cfg.checkpoint_every > 0 and g % cfg.checkpoint_every == 0:
            from ..utils.checkpoint import save_step_checkpoint
            save_step_checkpoint(self, cfg.checkpoint_dir,
                                 {"epoch": epoch, "iter": it + 1, "iters_per_epoch": iters},
                                 keep=cfg.keep_checkpoints)
        inj = os.environ.get("FF_FAULT_INJECT_STEP")
        if inj and self.executor.step_num == int(inj):
            raise RuntimeError(f"injected fault after step {inj} (FF_FAULT_INJECT_STEP)")

    def _native_loader(self, xs, y, bs):
        """Arrays (not loader objects) on a batch-split layout -> the native
        prefetching loader (runtime/dataloader.py); None -> host loaders."""
        if not self.ffconfig.native_data_loader:
            return None
        if any(isinstance(d, SingleDataLoader) for d in list(xs) + [y]) or y is None:
            return None
        if bs != self.ffconfig.batch_size or len(xs) != len(self._inputs):
            return None
        from ..runtime.dataloader import NativeDataLoader
        arrays = {self._inputs[i].name: np.asarray(d) for i, d in enumerate(xs)}
        arrays["__label__"] = np.asarray(y)
        try:
            return NativeDataLoader(self.executor, arrays, "__label__", bs,
                                    shuffle=bool(self.ffconfig.shuffle_data), seed=self.ffconfig.seed)
        except (ValueError, KeyError):
            return None

    def _init_local_backing(self, loss_type):
        """--local-execution: train through the native C++ CPU executor
        (csrc/ffcore/src/local_exec.cc, the reference's lib/local-execution),
        starting from the executor's initial weights."""
        if self.dist.world != 1 or self.executor.cfg.device.type != "cpu":
            raise RuntimeError("local execution runs on one CPU process (BASELINE config 1)")
        from ..runtime.optimizer import AdamConfig
        oc = self._optimizer.cfg
        kw = dict(lr=oc.lr, weight_decay=oc.weight_decay)
        if isinstance(oc, AdamConfig):
            if oc.decoupled:
                raise RuntimeError("local execution implements the reference Adam (L2 folded into the gradient)")
            kw.update(optimizer="adam", beta1=oc.beta1, beta2=oc.beta2, epsilon=oc.epsilon)
        else:
            kw.update(optimizer="sgd", momentum=oc.momentum, nesterov=oc.nesterov)
        lt = normalize_loss_type(loss_type) if loss_type is not None else "identity"
        b = C.LocalTrainingBacking(self.cg, loss=lt, seed=self.ffconfig.seed, **kw)
        for n in self.executor.parameter_names():
            b.set_weight(n, self.executor.get_parameter(n).numpy())
        self.local_backing = b

    def _fit_local(self, xs, y, bs, epochs, batch_hooks=None):
        b = self.local_backing
        arrays = [np.asarray(d.full if isinstance(d, SingleDataLoader) else d) for d in xs]
        labels = np.asarray(y.full if isinstance(y, SingleDataLoader) else y)
        names = [t.name for t in self._inputs]
        iters = len(labels) // bs
        t0 = time.time()
        for epoch in range(epochs):
            b.reset_metrics()
            for it in range(iters):
                if batch_hooks:
                    batch_hooks[0](it)
                sl = slice(it * bs, (it + 1) * bs)
                for n, a in zip(names, arrays):
                    b.set_input(n, a[sl])
                b.train_step(labels[sl].astype(np.float32))
                if batch_hooks:
                    batch_hooks[1](it)
            mm = b.metrics()
            if self.dist.rank == 0 and iters:
                acc = 100.0 * mm["correct"] / max(mm["samples"], 1)
                print(f"epoch {epoch}: samples={mm['samples']} accuracy={acc:.2f}% "
                      f"loss={mm['loss_sum'] / max(mm['samples'], 1):.4f} (local execution)", flush=True)
        elapsed = time.time() - t0
        for n in self.executor.parameter_names():   # keep the executor's view current
            self.executor.set_parameter(n, torch.from_numpy(np.array(b.get_weight(n))))
        thr = iters * bs * epochs / max(elapsed, 1e-9)
        print(f"ELAPSED TIME = {elapsed:.4f}s, THROUGHPUT = {thr:.2f} samples/s", flush=True)
        self.last_throughput = thr
        return thr

    def _fit_native(self, loader, epochs, batch_hooks=None):
        ex = self.executor
        iters = loader.iters_per_epoch
        num_samples = iters * loader.batch
        use_graph = bool(self.ffconfig.enable_hipgraph) and self._graph_capable()
        graphed = None
        start_epoch, start_it = self._resume_fit(iters)
        if start_epoch or start_it:
            loader.start(start_epoch * iters + start_it)
        if ex.cfg.device.type == "cuda":
            torch.cuda.synchronize()
        t0 = time.time()
        first = True
        try:
            for epoch in range(start_epoch, epochs):
                ex.zero_metrics()
                for it in range(start_it if epoch == start_epoch else 0, iters):
                    if batch_hooks:
                        batch_hooks[0](it)
                    feeds, labels, _ = loader.next()
                    if use_graph and not first:
                        if graphed is None:
                            graphed = ex.make_graphed_train_step(feeds, labels, warmup=0)
                        graphed(feeds, labels)
                    else:
                        ex.train_step(feeds, labels, lr=self._optimizer.cfg.lr)
                    first = False
                    self._after_fit_step(epoch, it, iters)
                    if batch_hooks:
                        batch_hooks[1](it)
                    if self.ffconfig.print_freq and (it + 1) % self.ffconfig.print_freq == 0:
                        pm = ex.perf_metrics()   # a collective: every rank calls it
                        if self.dist.rank == 0:
                            print(f"epoch {epoch} iter {it + 1}/{iters}: {pm}", flush=True)
                if iters:
                    pm = ex.perf_metrics()
                    if self.dist.rank == 0:
                        print(f"epoch {epoch}: {pm}", flush=True)
        finally:
            loader.close()
        if ex.cfg.device.type == "cuda":
            torch.cuda.synchronize()
        elapsed = time.time() - t0
        thr = num_samples * epochs / max(elapsed, 1e-9)
        if self.dist.rank == 0:
            print(f"ELAPSED TIME = {elapsed:.4f}s, THROUGHPUT = {thr:.2f} samples/s", flush=True)
        self.last_throughput = thr
        return thr

    def eval(self, x=None, y=None, batch_size=None):
        ex = self.executor
        xs = x if isinstance(x, (list, tuple)) else [x]
        loaders = [d if isinstance(d, SingleDataLoader) else SingleDataLoader(self, self._inputs[i], d)
                   for i, d in enumerate(xs)]
        ylo = y if isinstance(y, SingleDataLoader) else SingleDataLoader(self, self._label_tensor, y)
        bs = batch_size or self.ffconfig.batch_size
        for l in loaders + [ylo]:
            l.batch_size = bs
            l.reset()
        ex.zero_metrics()
        iters = ylo.num_samples // bs
        for _ in range(iters):
            feeds = {self._inputs[i].name: torch.as_tensor(l.next_batch()) for i, l in enumerate(loaders)}
            labels = torch.as_tensor(ylo.next_batch())
            ex.forward(feeds, training=False)
            # metrics without gradient: run the loss on the logits, discard grads
            if ex.loss is not None:
                ex._env[ex.loss_value] = ex._env.get(ex.loss_value)
                ex.compute_loss(labels)
        pm = ex.perf_metrics()
        if self.dist.rank == 0:
            print(f"eval: {pm}", flush=True)
        return pm

    def _value_key(self, t: Tensor):
        if self.executor is None or t.vref is None:
            return None
        v = self._pcg_value_of(t)
        if v is None:
            return None
        return v

    def _sparse_labels(self) -> bool:
        lt = self.loss_type
        return "SPARSE" in str(getattr(lt, "name", lt)).upper()

    def _label_dims(self):
        lt = self._label_tensor
        if lt is not None and getattr(lt, "_dims", None):
            return list(lt._dims)
        return [self.ffconfig.batch_size, 1]

    def _get_value(self, t: Tensor):
        """Latest value of a tensor as numpy (this rank's piece): a pending
        feed for inputs, else the last forward's activation.  Asking for an
        activation registers it for retention, so the next forward keeps it."""
        key = t.name or (f"input_{t.vref.node}" if t.vref is not None else None)
        if key in self._pending_feeds:
            return np.asarray(self._pending_feeds[key])
        v = self._value_key(t)
        if v is None:
            return None
        ex = self.executor
        ex.retain.add(v)
        x = ex._env.get(v, ex.retained.get(v))
        return None if x is None else x.detach().float().cpu().numpy()

    def _get_gradient(self, t: Tensor):
        """Gradient of the loss w.r.t. an activation from the last backward
        (registered for retention on first request)."""
        v = self._value_key(t)
        if v is None:
            return None
        ex = self.executor
        ex.retain.add(v)
        g = ex.retained_grads.get(v)
        return None if g is None else g.float().cpu().numpy()

    # ------------------------------------------------------------ recompile
    def recompile_on_condition(self, r) -> bool:
        """Reference: FFModel::recompile_on_condition (model.h:107)."""
        if r.ff is None:
            r.ff = self
        if not r.trigger():
            return False
        r.alter()
        self.recompile()
        return True

    def recompile(self):
        """Re-plan the parallelisation (search / import / DP per the current
        FFConfig) and move the training state onto the new executor."""
        old = self.executor
        if old is None:
            raise RuntimeError("call compile() first")
        names = old.parameter_names()
        params = {n: old.get_parameter(n).cpu() for n in names}
        ostate = {n: {k: t.cpu() for k, t in old.get_optimizer_state(n).items()} for n in names}
        step = old.step_num
        opt_steps = max([f["opt"].step_num for f in old.flats] or [0])
        if old.dist.distributed:
            opt_steps = int(old.dist.max_scalar(float(opt_steps)))
        self.executor = None
        self.compile(optimizer=self._optimizer, loss_type=self.loss_type, metrics=self.metrics)
        ex = self.executor
        for n in ex.parameter_names():
            if n in params:
                ex.set_parameter(n, params[n])
                if ostate.get(n):
                    ex.set_optimizer_state(n, ostate[n])
        ex.step_num = step
        for f in ex.flats:
            f["opt"].step_num = opt_steps
        self.recompilations = getattr(self, "recompilations", 0) + 1
        return self

    # ------------------------------------------------------------ checkpoint
    def save_checkpoint(self, path: str):
        from ..utils.checkpoint import save_checkpoint

        save_checkpoint(self, path)

    def load_checkpoint(self, path: str):
        from ..utils.checkpoint import load_checkpoint

        return load_checkpoint(self, path)
