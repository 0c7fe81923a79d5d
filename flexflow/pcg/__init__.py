"""flexflow.pcg — Python bindings over the C ABI (libflexflow_c.so).

Reference: bindings/python/python/flexflow/pcg/high_level.py (+ raw.py), the
new cffi sketch over lib/*/ffi (ComputationGraph / Tensor wrappers; a sketch
with a syntax error there).  Here the wrappers are complete and
go through the shipped C ABI (csrc/ffi/flexflow_c.h) with ctypes, so a
program that only links the C library sees the same graph, serialisation and
search as the Python package.

    from flexflow.pcg import ComputationGraph, DataType, Activation
    cg = ComputationGraph()
    x = cg.create_tensor([64, 784], DataType.FLOAT)
    y = cg.softmax(cg.dense(cg.dense(x, 512, Activation.RELU), 10))
    res = cg.optimize({"num_nodes": 1, "num_gpus_per_node": 8})
    res.cost, res.data_parallel_cost, res.parallel_computation_graph()
"""
from __future__ import annotations

import ctypes
import enum
import json
import os
from typing import Dict, List, Optional, Sequence, Union

_LIB_PATH = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                         "flexflow_train_amd", "lib", "libflexflow_c.so")


class DataType(enum.IntEnum):
    BOOL = 0
    INT32 = 1
    INT64 = 2
    HALF = 3
    BF16 = 4
    FLOAT = 5
    DOUBLE = 6


class Activation(enum.IntEnum):
    NONE = 0
    RELU = 1
    SIGMOID = 2
    TANH = 3
    GELU = 4


class _Tensor(ctypes.Structure):
    _fields_ = [("node", ctypes.c_int), ("idx", ctypes.c_int)]


class FlexFlowError(RuntimeError):
    pass


_lib = None


def _load():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            import sys

            sys.path.insert(0, os.path.dirname(os.path.dirname(_LIB_PATH)))
            from tools.build_native import build

            build(["ffi"])
        lib = ctypes.CDLL(_LIB_PATH)
        lib.flexflow_last_error.restype = ctypes.c_char_p
        lib.flexflow_version.restype = ctypes.c_char_p
        lib.flexflow_free.argtypes = [ctypes.c_void_p]
        _lib = lib
    return _lib


def _check(rc: int):
    if rc != 0:
        raise FlexFlowError(_load().flexflow_last_error().decode())


def _take_str(p: ctypes.c_void_p) -> str:
    s = ctypes.cast(p, ctypes.c_char_p).value.decode()
    _load().flexflow_free(p)
    return s


def _name(n: Optional[str]):
    return n.encode() if n else None


def _i64(xs: Sequence[int]):
    return (ctypes.c_int64 * len(xs))(*[int(v) for v in xs])


def version() -> str:
    return _load().flexflow_version().decode()


class Tensor:
    """A tensor (layer output) of a ComputationGraph."""

    def __init__(self, cg: "ComputationGraph", handle: _Tensor):
        self._cg = cg
        self._h = handle

    @property
    def dims(self) -> tuple:
        n = ctypes.c_int()
        _check(_load().flexflow_tensor_get_num_dims(self._cg._h, self._h, ctypes.byref(n)))
        out = (ctypes.c_int64 * n.value)()
        _check(_load().flexflow_tensor_get_dims(self._cg._h, self._h, out))
        return tuple(out)

    @property
    def datatype(self) -> DataType:
        d = ctypes.c_int()
        _check(_load().flexflow_tensor_get_datatype(self._cg._h, self._h, ctypes.byref(d)))
        return DataType(d.value)

    @property
    def layer(self) -> int:
        return self._h.node

    def __repr__(self):
        return f"Tensor(layer={self._h.node}, idx={self._h.idx}, dims={self.dims}, {self.datatype.name})"


class SearchResult:
    def __init__(self, handle):
        self._h = handle

    def __del__(self):
        if getattr(self, "_h", None) and _lib is not None:
            _lib.flexflow_search_result_destroy(self._h)
            self._h = None

    def _costs(self):
        c, dp = ctypes.c_double(), ctypes.c_double()
        _check(_load().flexflow_search_result_get_cost(self._h, ctypes.byref(c), ctypes.byref(dp)))
        return c.value, dp.value

    @property
    def cost(self) -> float:
        """Simulated seconds per iteration of the searched strategy."""
        return self._costs()[0]

    @property
    def data_parallel_cost(self) -> float:
        return self._costs()[1]

    def report(self) -> Dict:
        p = ctypes.c_void_p()
        _check(_load().flexflow_search_result_get_report_json(self._h, ctypes.byref(p)))
        return json.loads(_take_str(p))

    def parallel_computation_graph(self) -> Dict:
        p = ctypes.c_void_p()
        _check(_load().flexflow_search_result_get_parallel_computation_graph_json(self._h, ctypes.byref(p)))
        return json.loads(_take_str(p))

    def parallel_layer_for(self, t: Union[Tensor, int]) -> int:
        n = ctypes.c_int()
        _check(_load().flexflow_search_result_get_parallel_layer_for_layer(
            self._h, t.layer if isinstance(t, Tensor) else int(t), ctypes.byref(n)))
        return n.value


class ComputationGraph:
    """Builder + container of a computation graph (reference:
    lib/pcg/include/pcg/computation_graph_builder.h)."""

    def __init__(self, _handle=None):
        lib = _load()
        if _handle is None:
            _handle = ctypes.c_void_p()
            _check(lib.flexflow_computation_graph_create(ctypes.byref(_handle)))
        self._h = _handle

    def __del__(self):
        if getattr(self, "_h", None) and _lib is not None:
            _lib.flexflow_computation_graph_destroy(self._h)
            self._h = None

    # ---------------------------------------------------------------- graph I/O
    @classmethod
    def from_model(cls, name: str) -> "ComputationGraph":
        h = ctypes.c_void_p()
        _check(_load().flexflow_computation_graph_from_model(name.encode(), ctypes.byref(h)))
        return cls(h)

    @classmethod
    def deserialize(cls, text: str) -> "ComputationGraph":
        h = ctypes.c_void_p()
        _check(_load().flexflow_computation_graph_deserialize_from_buf(text.encode(), ctypes.byref(h)))
        return cls(h)

    @classmethod
    def load(cls, path: str) -> "ComputationGraph":
        h = ctypes.c_void_p()
        _check(_load().flexflow_computation_graph_deserialize_from_file(path.encode(), ctypes.byref(h)))
        return cls(h)

    def serialize(self) -> str:
        p = ctypes.c_void_p()
        _check(_load().flexflow_computation_graph_serialize_to_buf(self._h, ctypes.byref(p)))
        return _take_str(p)

    def save(self, path: str):
        _check(_load().flexflow_computation_graph_serialize_to_file(self._h, path.encode()))

    def as_dot(self) -> str:
        p = ctypes.c_void_p()
        _check(_load().flexflow_computation_graph_as_dot(self._h, ctypes.byref(p)))
        return _take_str(p)

    @property
    def num_layers(self) -> int:
        n = ctypes.c_int()
        _check(_load().flexflow_computation_graph_num_layers(self._h, ctypes.byref(n)))
        return n.value

    # ---------------------------------------------------------------- builders
    def _one(self, fn: str, *args) -> Tensor:
        out = _Tensor()
        _check(getattr(_load(), fn)(self._h, *args, ctypes.byref(out)))
        return Tensor(self, out)

    def create_tensor(self, dims: Sequence[int], dtype: DataType = DataType.FLOAT, create_grad: bool = True,
                      name: Optional[str] = None) -> Tensor:
        out = _Tensor()
        _check(_load().flexflow_tensor_create(self._h, len(dims), _i64(dims), int(dtype), bool(create_grad),
                                              _name(name), ctypes.byref(out)))
        return Tensor(self, out)

    def dense(self, x: Tensor, out_dim: int, activation: Activation = Activation.NONE, use_bias: bool = True,
              name: Optional[str] = None) -> Tensor:
        return self._one("flexflow_computation_graph_add_op_dense", x._h, ctypes.c_int64(out_dim), int(activation),
                         bool(use_bias), _name(name))

    def _unary(self, op: str, x: Tensor, name=None) -> Tensor:
        return self._one(f"flexflow_computation_graph_add_op_{op}", x._h, _name(name))

    def relu(self, x, name=None):
        return self._unary("relu", x, name)

    def gelu(self, x, name=None):
        return self._unary("gelu", x, name)

    def sigmoid(self, x, name=None):
        return self._unary("sigmoid", x, name)

    def tanh(self, x, name=None):
        return self._unary("tanh", x, name)

    def exp(self, x, name=None):
        return self._unary("exp", x, name)

    def identity(self, x, name=None):
        return self._unary("identity", x, name)

    def rsqrt(self, x, name=None):
        return self._unary("rsqrt", x, name)

    def flat(self, x, name=None):
        return self._unary("flat", x, name)

    def scalar_multiply(self, x: Tensor, s: float, name=None) -> Tensor:
        return self._one("flexflow_computation_graph_add_op_scalar_multiply", x._h, ctypes.c_double(s), _name(name))

    def scalar_add(self, x: Tensor, s: float, name=None) -> Tensor:
        return self._one("flexflow_computation_graph_add_op_scalar_add", x._h, ctypes.c_double(s), _name(name))

    def _binary(self, op: str, a: Tensor, b: Tensor, name=None) -> Tensor:
        return self._one(f"flexflow_computation_graph_add_op_{op}", a._h, b._h, _name(name))

    def add(self, a, b, name=None):
        return self._binary("add", a, b, name)

    def subtract(self, a, b, name=None):
        return self._binary("subtract", a, b, name)

    def multiply(self, a, b, name=None):
        return self._binary("multiply", a, b, name)

    def divide(self, a, b, name=None):
        return self._binary("divide", a, b, name)

    def batch_matmul(self, a, b, name=None):
        return self._binary("batch_matmul", a, b, name)

    def softmax(self, x: Tensor, dim: int = -1, name=None) -> Tensor:
        return self._one("flexflow_computation_graph_add_op_softmax", x._h, int(dim), _name(name))

    def layer_norm(self, x: Tensor, axes: Sequence[int] = (-1,), elementwise_affine: bool = True,
                   eps: float = 1e-5, name=None) -> Tensor:
        return self._one("flexflow_computation_graph_add_op_layer_norm", x._h, len(axes), _i64(axes),
                         bool(elementwise_affine), ctypes.c_double(eps), _name(name))

    def batch_norm(self, x: Tensor, relu: bool = False, name=None) -> Tensor:
        return self._one("flexflow_computation_graph_add_op_batch_norm", x._h, bool(relu), _name(name))

    def embedding(self, x: Tensor, num_entries: int, out_dim: int, aggr: str = "none", name=None) -> Tensor:
        return self._one("flexflow_computation_graph_add_op_embedding", x._h, ctypes.c_int64(num_entries),
                         ctypes.c_int64(out_dim), aggr.encode(), _name(name))

    def conv2d(self, x: Tensor, out_channels: int, kernel_h: int, kernel_w: int, stride_h: int = 1,
               stride_w: int = 1, padding_h: int = 0, padding_w: int = 0,
               activation: Activation = Activation.NONE, groups: int = 1, use_bias: bool = True, name=None) -> Tensor:
        return self._one("flexflow_computation_graph_add_op_conv2d", x._h, ctypes.c_int64(out_channels), kernel_h,
                         kernel_w, stride_h, stride_w, padding_h, padding_w, int(activation), groups, bool(use_bias),
                         _name(name))

    def pool2d(self, x: Tensor, kernel_h: int, kernel_w: int, stride_h: int, stride_w: int, padding_h: int = 0,
               padding_w: int = 0, pool_type: str = "max", name=None) -> Tensor:
        return self._one("flexflow_computation_graph_add_op_pool2d", x._h, kernel_h, kernel_w, stride_h, stride_w,
                         padding_h, padding_w, pool_type.encode(), _name(name))

    def reshape(self, x: Tensor, shape: Sequence[int], name=None) -> Tensor:
        return self._one("flexflow_computation_graph_add_op_reshape", x._h, len(shape), _i64(shape), _name(name))

    def transpose(self, x: Tensor, perm: Sequence[int], name=None) -> Tensor:
        return self._one("flexflow_computation_graph_add_op_transpose", x._h, len(perm), _i64(perm), _name(name))

    def concat(self, xs: Sequence[Tensor], axis: int, name=None) -> Tensor:
        arr = (_Tensor * len(xs))(*[t._h for t in xs])
        out = _Tensor()
        _check(_load().flexflow_computation_graph_add_op_concat(self._h, len(xs), arr, int(axis), _name(name),
                                                                ctypes.byref(out)))
        return Tensor(self, out)

    def split(self, x: Tensor, sizes: Sequence[int], axis: int, name=None) -> List[Tensor]:
        outs = (_Tensor * len(sizes))()
        _check(_load().flexflow_computation_graph_add_op_split(self._h, x._h, len(sizes), _i64(sizes), int(axis),
                                                               _name(name), outs))
        return [Tensor(self, outs[i]) for i in range(len(sizes))]

    def dropout(self, x: Tensor, rate: float, seed: int = 0, name=None) -> Tensor:
        return self._one("flexflow_computation_graph_add_op_dropout", x._h, ctypes.c_double(rate),
                         ctypes.c_int64(seed), _name(name))

    def multihead_attention(self, q: Tensor, k: Tensor, v: Tensor, embed_dim: int, num_heads: int, kdim: int = 0,
                            vdim: int = 0, dropout: float = 0.0, bias: bool = True, causal: bool = False,
                            name=None) -> Tensor:
        out = _Tensor()
        _check(_load().flexflow_computation_graph_add_multihead_attention(
            self._h, q._h, k._h, v._h, ctypes.c_int64(embed_dim), ctypes.c_int64(num_heads), ctypes.c_int64(kdim),
            ctypes.c_int64(vdim), ctypes.c_double(dropout), bool(bias), bool(causal), _name(name), ctypes.byref(out)))
        return Tensor(self, out)

    def add_op(self, attrs: Dict, inputs: Sequence[Tensor], name: Optional[str] = None,
               max_outputs: int = 8) -> List[Tensor]:
        """Any operator by its attribute JSON (``{"op_type": ..., ...}``)."""
        arr = (_Tensor * max(1, len(inputs)))(*[t._h for t in inputs])
        outs = (_Tensor * max_outputs)()
        n = ctypes.c_int()
        _check(_load().flexflow_computation_graph_add_op(self._h, json.dumps(attrs).encode(), len(inputs), arr,
                                                         _name(name), max_outputs, outs, ctypes.byref(n)))
        return [Tensor(self, outs[i]) for i in range(n.value)]

    # ---------------------------------------------------------------- search
    def optimize(self, machine: Dict, search: Optional[Dict] = None) -> SearchResult:
        """Strategy search (MCMC + Unity) on ``machine`` ({"num_nodes",
        "num_gpus_per_node", ...}) -> SearchResult."""
        h = ctypes.c_void_p()
        _check(_load().flexflow_computation_graph_optimize(self._h, json.dumps(machine).encode(),
                                                           json.dumps(search or {}).encode(), ctypes.byref(h)))
        return SearchResult(h)
