"""ONNX -> FFModel importer (python/flexflow/onnx/model.py:74-363).

The ``onnx`` package is not part of this environment, so the ONNX protobuf
subset the importer needs (ModelProto / GraphProto / NodeProto /
AttributeProto / TensorProto / ValueInfoProto) is decoded directly from the
wire format here; ``encode_model`` writes the same subset (used by tests
and by ``export_onnx``-style tooling).  When ``onnx`` is importable a
``ModelProto`` object is accepted as well.

Handlers: Add, Sub, Mul, Concat, Split, AveragePool, GlobalAveragePool,
BatchNormalization, Conv, Dropout, Flatten, Gemm, MatMul, MaxPool, Relu,
Sigmoid, Tanh, Pad (zero pads folded into the following Conv/Pool),
Softmax, Reshape, Cast, Unsqueeze, Identity, Constant, Range, Transpose.
"""
from __future__ import annotations

import struct
from typing import Dict, List, Optional, Tuple

import numpy as np

from ..core import ActiMode, DataType, PoolType

# ----------------------------------------------------------------- wire format
_F32, _I64, _I32, _F64 = 1, 7, 6, 11
_NP = {1: np.float32, 2: np.uint8, 3: np.int8, 6: np.int32, 7: np.int64, 9: np.bool_, 10: np.float16, 11: np.float64}


def _varint(buf, i):
    v, s = 0, 0
    while True:
        b = buf[i]
        i += 1
        v |= (b & 0x7F) << s
        if not b & 0x80:
            return v, i
        s += 7


def _fields(buf: bytes):
    i, n = 0, len(buf)
    while i < n:
        tag, i = _varint(buf, i)
        f, wt = tag >> 3, tag & 7
        if wt == 0:
            v, i = _varint(buf, i)
        elif wt == 1:
            v = buf[i:i + 8]
            i += 8
        elif wt == 2:
            ln, i = _varint(buf, i)
            v = buf[i:i + ln]
            i += ln
        elif wt == 5:
            v = buf[i:i + 4]
            i += 4
        else:
            raise ValueError(f"unsupported wire type {wt}")
        yield f, wt, v


def _signed(v):
    return v - (1 << 64) if v >= 1 << 63 else v


def _packed_ints(v, wt):
    if wt == 0:
        return [_signed(v)]
    out, i = [], 0
    while i < len(v):
        x, i = _varint(v, i)
        out.append(_signed(x))
    return out


def _packed_floats(v, wt):
    if wt == 5:
        return [struct.unpack("<f", v)[0]]
    return list(np.frombuffer(v, dtype="<f4"))


class Tensor:
    def __init__(self):
        self.name, self.dims, self.dtype, self.data = "", [], _F32, None

    @staticmethod
    def decode(buf):
        t = Tensor()
        floats, ints, raw = [], [], None
        for f, wt, v in _fields(buf):
            if f == 1:
                t.dims += _packed_ints(v, wt)
            elif f == 2:
                t.dtype = v
            elif f == 4:
                floats += _packed_floats(v, wt)
            elif f in (5, 7):
                ints += _packed_ints(v, wt)
            elif f == 8:
                t.name = v.decode()
            elif f == 9:
                raw = v
        dt = _NP.get(t.dtype, np.float32)
        if raw is not None:
            arr = np.frombuffer(raw, dtype=dt).copy()
        elif floats:
            arr = np.asarray(floats, dtype=dt)
        else:
            arr = np.asarray(ints, dtype=dt)
        t.data = arr.reshape(t.dims) if t.dims else arr.reshape(())
        return t


class Attr:
    @staticmethod
    def decode(buf):
        name, val, floats, ints, strs = None, None, [], [], []
        for f, wt, v in _fields(buf):
            if f == 1:
                name = v.decode()
            elif f == 2:
                val = struct.unpack("<f", v)[0]
            elif f == 3:
                val = _signed(v)
            elif f == 4:
                val = v.decode()
            elif f == 5:
                val = Tensor.decode(v).data
            elif f == 7:
                floats += _packed_floats(v, wt)
            elif f == 8:
                ints += _packed_ints(v, wt)
        if val is None:
            val = ints if ints else floats
        return name, val


class Node:
    def __init__(self, op_type="", inputs=(), outputs=(), name="", attrs=None):
        self.op_type, self.inputs, self.outputs, self.name = op_type, list(inputs), list(outputs), name
        self.attrs = dict(attrs or {})

    @staticmethod
    def decode(buf):
        n = Node()
        for f, wt, v in _fields(buf):
            if f == 1:
                n.inputs.append(v.decode())
            elif f == 2:
                n.outputs.append(v.decode())
            elif f == 3:
                n.name = v.decode()
            elif f == 4:
                n.op_type = v.decode()
            elif f == 5:
                k, a = Attr.decode(v)
                n.attrs[k] = a
        return n


def _value_info(buf) -> Tuple[str, List[int], int]:
    name, dims, elem = "", [], _F32
    for f, wt, v in _fields(buf):
        if f == 1:
            name = v.decode()
        elif f == 2:
            for f2, _, v2 in _fields(v):           # TypeProto
                if f2 == 1:                          # tensor_type
                    for f3, _, v3 in _fields(v2):
                        if f3 == 1:
                            elem = v3
                        elif f3 == 2:                # TensorShapeProto
                            for f4, _, v4 in _fields(v3):
                                if f4 == 1:
                                    d = None
                                    for f5, _, v5 in _fields(v4):
                                        if f5 == 1:
                                            d = _signed(v5)
                                    dims.append(d if d is not None else -1)
    return name, dims, elem


class Graph:
    def __init__(self):
        self.nodes: List[Node] = []
        self.initializers: Dict[str, np.ndarray] = {}
        self.inputs: List[Tuple[str, List[int], int]] = []
        self.outputs: List[Tuple[str, List[int], int]] = []

    @staticmethod
    def decode_model(buf: bytes) -> "Graph":
        for f, wt, v in _fields(buf):
            if f == 7:
                return Graph.decode(v)
        raise ValueError("ModelProto has no graph")

    @staticmethod
    def decode(buf):
        g = Graph()
        for f, wt, v in _fields(buf):
            if f == 1:
                g.nodes.append(Node.decode(v))
            elif f == 5:
                t = Tensor.decode(v)
                g.initializers[t.name] = t.data
            elif f == 11:
                g.inputs.append(_value_info(v))
            elif f == 12:
                g.outputs.append(_value_info(v))
        return g


# encoder (subset) ---------------------------------------------------------
def _ev(x):
    out = bytearray()
    x &= (1 << 64) - 1
    while True:
        b = x & 0x7F
        x >>= 7
        if x:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _fld(f, wt, payload):
    if wt == 0:
        return _ev(f << 3) + _ev(payload)
    if wt == 2:
        return _ev(f << 3 | 2) + _ev(len(payload)) + payload
    if wt == 5:
        return _ev(f << 3 | 5) + payload
    raise ValueError


def _enc_tensor(name, arr: np.ndarray) -> bytes:
    dt = {np.dtype(np.float32): _F32, np.dtype(np.int64): _I64, np.dtype(np.int32): _I32}[arr.dtype]
    b = b"".join(_fld(1, 0, d) for d in arr.shape) + _fld(2, 0, dt) + _fld(8, 2, name.encode())
    return b + _fld(9, 2, np.ascontiguousarray(arr).tobytes())


def _enc_attr(k, v) -> bytes:
    b = _fld(1, 2, k.encode())
    if isinstance(v, float):
        return b + _fld(2, 5, struct.pack("<f", v)) + _fld(20, 0, 1)
    if isinstance(v, (int, np.integer)):
        return b + _fld(3, 0, int(v)) + _fld(20, 0, 2)
    if isinstance(v, str):
        return b + _fld(4, 2, v.encode()) + _fld(20, 0, 3)
    if isinstance(v, np.ndarray):
        return b + _fld(5, 2, _enc_tensor(k, v)) + _fld(20, 0, 4)
    if isinstance(v, (list, tuple)) and v and isinstance(v[0], float):
        return b + b"".join(_fld(7, 5, struct.pack("<f", x)) for x in v) + _fld(20, 0, 6)
    return b + b"".join(_fld(8, 0, int(x)) for x in v) + _fld(20, 0, 7)


def _enc_vi(name, dims, elem=_F32) -> bytes:
    shape = b"".join(_fld(1, 2, _fld(1, 0, d)) for d in dims)
    tt = _fld(1, 0, elem) + _fld(2, 2, shape)
    return _fld(1, 2, name.encode()) + _fld(2, 2, _fld(1, 2, tt))


def encode_model(nodes: List[Node], initializers: Dict[str, np.ndarray], inputs: List[Tuple[str, List[int]]],
                 outputs: List[Tuple[str, List[int]]], opset: int = 13) -> bytes:
    g = b""
    for n in nodes:
        nb = b"".join(_fld(1, 2, i.encode()) for i in n.inputs) + b"".join(_fld(2, 2, o.encode()) for o in n.outputs)
        nb += _fld(3, 2, n.name.encode()) + _fld(4, 2, n.op_type.encode())
        nb += b"".join(_fld(5, 2, _enc_attr(k, v)) for k, v in n.attrs.items())
        g += _fld(1, 2, nb)
    g += _fld(2, 2, b"graph")
    for k, a in initializers.items():
        g += _fld(5, 2, _enc_tensor(k, a))
    for nm, d in inputs:
        g += _fld(11, 2, _enc_vi(nm, d))
    for nm, d in outputs:
        g += _fld(12, 2, _enc_vi(nm, d))
    opset_b = _fld(1, 2, b"") + _fld(2, 0, opset)
    return _fld(1, 0, 8) + _fld(2, 2, b"flexflow_train_amd") + _fld(8, 2, opset_b) + _fld(7, 2, g)


# -------------------------------------------------------------------- importer
class ONNXModel:
    def __init__(self, model):
        if isinstance(model, (bytes, bytearray)):
            self.graph = Graph.decode_model(bytes(model))
        elif isinstance(model, str):
            with open(model, "rb") as f:
                self.graph = Graph.decode_model(f.read())
        else:  # an onnx.ModelProto
            self.graph = Graph.decode_model(model.SerializeToString())
        self.weights: Dict[str, Tuple[str, np.ndarray]] = {}

    def apply(self, ffmodel, input_tensors):
        g = self.graph
        env: Dict[str, object] = {}
        consts: Dict[str, np.ndarray] = dict(g.initializers)
        real_inputs = [n for (n, _, _) in g.inputs if n not in consts]
        for n, t in zip(real_inputs, input_tensors):
            env[n] = t
        pads: Dict[str, Tuple[str, List[int]]] = {}
        for node in g.nodes:
            self._handle(ffmodel, node, env, consts, pads)
        outs = [env[n] for (n, _, _) in g.outputs]
        return outs[0] if len(outs) == 1 else outs

    def _handle(self, ff, node: Node, env, consts, pads):
        op, a, name = node.op_type, node.attrs, node.name or node.outputs[0]
        x = env.get(node.inputs[0]) if node.inputs else None
        o = node.outputs[0]

        def const(i):
            return consts[node.inputs[i]]

        if op in ("Add", "Sub", "Mul"):
            fn = {"Add": ff.add, "Sub": ff.subtract, "Mul": ff.multiply}[op]
            if node.inputs[1] in consts:
                c = const(1)
                if c.size == 1:
                    sfn = {"Add": ff.scalar_add, "Sub": ff.scalar_sub, "Mul": ff.scalar_multiply}[op]
                    env[o] = sfn(x, float(c.reshape(())), name=name)
                    return
                raise NotImplementedError(f"{op} with a non-scalar constant")
            env[o] = fn(x, env[node.inputs[1]], name=name)
        elif op == "Concat":
            env[o] = ff.concat([env[i] for i in node.inputs], int(a.get("axis", 1)), name=name)
        elif op == "Split":
            axis = int(a.get("axis", 0))
            sizes = list(a["split"]) if "split" in a else (list(const(1)) if len(node.inputs) > 1 else None)
            if sizes is None:
                k = len(node.outputs)
                sizes = [x.dims[axis] // k] * k
            outs = ff.split(x, [int(s) for s in sizes], axis, name=name)
            for oname, t in zip(node.outputs, outs):
                env[oname] = t
        elif op in ("MaxPool", "AveragePool"):
            k = a["kernel_shape"]
            s = a.get("strides", [1, 1])
            p = list(a.get("pads", [0, 0, 0, 0]))
            if node.inputs[0] in pads:
                x = env[pads[node.inputs[0]][0]]
                pp = pads[node.inputs[0]][1]
                p = [p[0] + pp[2], p[1] + pp[3]]
            pt = PoolType.POOL_MAX if op == "MaxPool" else PoolType.POOL_AVG
            env[o] = ff.pool2d(x, k[0], k[1], s[0], s[1], p[0], p[1], pt, name=name)
        elif op == "GlobalAveragePool":
            h, w = x.dims[2], x.dims[3]
            env[o] = ff.pool2d(x, h, w, 1, 1, 0, 0, PoolType.POOL_AVG, name=name)
        elif op == "BatchNormalization":
            env[o] = ff.batch_norm(x, False, name=name)
            self.weights[name + ".gamma"] = ("copy", const(1))
            self.weights[name + ".beta"] = ("copy", const(2))
        elif op == "Conv":
            w = const(1)
            k = a.get("kernel_shape", list(w.shape[2:]))
            s = a.get("strides", [1, 1])
            p = list(a.get("pads", [0, 0, 0, 0]))
            if node.inputs[0] in pads:
                x = env[pads[node.inputs[0]][0]]
                pp = pads[node.inputs[0]][1]
                p = [p[0] + pp[2], p[1] + pp[3]]
            bias = len(node.inputs) > 2
            env[o] = ff.conv2d(x, w.shape[0], k[0], k[1], s[0], s[1], p[0], p[1], ActiMode.AC_MODE_NONE,
                               int(a.get("group", 1)), bias, name=name)
            self.weights[name + ".kernel"] = ("copy", w)
            if bias:
                self.weights[name + ".bias"] = ("copy", const(2))
        elif op == "Dropout":
            env[o] = ff.dropout(x, float(a.get("ratio", 0.5)), 0, name=name)
        elif op == "Flatten":
            env[o] = ff.flat(x, name=name)
        elif op in ("Gemm", "MatMul"):
            w = const(1)
            if op == "Gemm" and int(a.get("transB", 0)):
                w = w.T
            bias = op == "Gemm" and len(node.inputs) > 2
            env[o] = ff.dense(x, w.shape[1], ActiMode.AC_MODE_NONE, bias, name=name)
            self.weights[name + ".kernel"] = ("copy", np.ascontiguousarray(w))
            if bias:
                self.weights[name + ".bias"] = ("copy", const(2))
        elif op in ("Relu", "Sigmoid", "Tanh", "Identity"):
            fn = {"Relu": ff.relu, "Sigmoid": ff.sigmoid, "Tanh": ff.tanh, "Identity": ff.identity}[op]
            env[o] = fn(x, name=name)
        elif op == "Pad":
            p = list(a["pads"]) if "pads" in a else list(const(1))
            if any(v < 0 for v in p) or a.get("mode", "constant") not in ("constant", b"constant"):
                raise NotImplementedError("Pad: only non-negative zero padding")
            env[o] = x
            pads[o] = (node.inputs[0], p)   # folded into the consumer conv / pool
        elif op == "Softmax":
            env[o] = ff.softmax(x, int(a.get("axis", -1)), name=name)
        elif op == "Reshape":
            shape = [int(s) for s in const(1)]
            total = int(np.prod(x.dims))
            shape = [x.dims[i] if s == 0 else s for i, s in enumerate(shape)]
            if -1 in shape:
                k = int(np.prod([s for s in shape if s != -1]))
                shape = [total // k if s == -1 else s for s in shape]
            env[o] = ff.reshape(x, shape, name=name)
        elif op == "Cast":
            to = {1: DataType.DT_FLOAT, 6: DataType.DT_INT32, 7: DataType.DT_INT64}[int(a["to"])]
            env[o] = ff.cast(x, to, name=name)
        elif op == "Unsqueeze":
            axes = list(a["axes"]) if "axes" in a else [int(v) for v in const(1)]
            shape = list(x.dims)
            for ax in sorted(axes):
                shape.insert(ax if ax >= 0 else len(shape) + ax + 1, 1)
            env[o] = ff.reshape(x, shape, name=name)
        elif op == "Transpose":
            env[o] = ff.transpose(x, [int(p) for p in a["perm"]], name=name)
        elif op == "Constant":
            consts[o] = np.asarray(a["value"])
        elif op == "Range":
            s, e, d = (float(const(i).reshape(())) for i in range(3))
            consts[o] = np.arange(s, e, d)
        else:
            raise NotImplementedError(f"ONNX op {op}")

    def copy_weights(self, ffmodel):
        import torch

        ex = ffmodel.executor
        names = set(ex.parameter_names())
        for pname, (_, arr) in self.weights.items():
            if pname in names:
                ex.set_parameter(pname, torch.as_tensor(np.asarray(arr, dtype=np.float32)))
