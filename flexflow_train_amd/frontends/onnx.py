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
def _fuse_matmul_add(nodes: List[Node], consts, shapes) -> List[Node]:
    """MatMul(x, W) whose only consumer is Add(., bias) with a constant 1-D
    bias -> one Gemm(x, W, bias) (the keras2onnx form of a Dense layer)."""
    users: Dict[str, List[Node]] = {}
    for n in nodes:
        for i in n.inputs:
            users.setdefault(i, []).append(n)
    out, skip = [], set()
    for n in nodes:
        if id(n) in skip:
            continue
        if n.op_type == "MatMul" and len(users.get(n.outputs[0], [])) == 1:
            u = users[n.outputs[0]][0]
            other = [i for i in u.inputs if i != n.outputs[0]]
            if (u.op_type == "Add" and len(other) == 1 and
                    (other[0] in consts and consts[other[0]].ndim == 1 or len(shapes.get(other[0], [])) == 1)):
                out.append(Node("Gemm", [n.inputs[0], n.inputs[1], other[0]], u.outputs, n.name or u.name, {}))
                skip.add(id(u))
                continue
        out.append(n)
    return out


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
        """Replay the graph into ``ffmodel``.  ``input_tensors``: a list (the
        graph's non-initializer inputs in order) or a {input name: tensor}
        dict as in the reference (``apply(ffmodel, {"input.1": t})``).
        Returns the output tensor (one output) or the list of them."""
        g = self.graph
        consts: Dict[str, np.ndarray] = dict(g.initializers)
        # parameters exported as graph inputs (export_params=False) are known
        # by shape only: FlexFlow initialises them itself
        self.shapes: Dict[str, List[int]] = {n: list(d) for (n, d, _) in g.inputs}
        if isinstance(input_tensors, dict):
            env: Dict[str, object] = dict(input_tensors)
        else:
            real_inputs = [n for (n, _, _) in g.inputs if n not in consts]
            env = dict(zip(real_inputs, input_tensors))
        pads: Dict[str, Tuple[str, List[int]]] = {}
        for node in _fuse_matmul_add(g.nodes, consts, self.shapes):
            self._handle(ffmodel, node, env, consts, pads)
        outs = [env[n] for (n, _, _) in g.outputs]
        return outs[0] if len(outs) == 1 else outs

    def _shape(self, consts, name) -> List[int]:
        if name in consts:
            return list(consts[name].shape)
        return list(self.shapes[name])

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
            if node.inputs[1] in consts:
                self.weights[name + ".gamma"] = ("copy", const(1))
            if node.inputs[2] in consts:
                self.weights[name + ".beta"] = ("copy", const(2))
        elif op == "Conv":
            w = consts.get(node.inputs[1])
            wshape = self._shape(consts, node.inputs[1])
            k = a.get("kernel_shape", wshape[2:])
            s = a.get("strides", [1, 1])
            p = list(a.get("pads", [0, 0, 0, 0]))
            if node.inputs[0] in pads:
                x = env[pads[node.inputs[0]][0]]
                pp = pads[node.inputs[0]][1]
                p = [p[0] + pp[2], p[1] + pp[3]]
            bias = len(node.inputs) > 2
            env[o] = ff.conv2d(x, wshape[0], k[0], k[1], s[0], s[1], p[0], p[1], ActiMode.AC_MODE_NONE,
                               int(a.get("group", 1)), bias, name=name)
            if w is not None:
                self.weights[name + ".kernel"] = ("copy", w)
            if bias and node.inputs[2] in consts:
                self.weights[name + ".bias"] = ("copy", const(2))
        elif op == "Dropout":
            env[o] = ff.dropout(x, float(a.get("ratio", 0.5)), 0, name=name)
        elif op == "Flatten":
            env[o] = ff.flat(x, name=name)
        elif op in ("Gemm", "MatMul"):
            w = consts.get(node.inputs[1])
            wshape = self._shape(consts, node.inputs[1])
            tb = op == "Gemm" and int(a.get("transB", 0))
            if tb:
                w = None if w is None else w.T
                wshape = wshape[::-1]
            bias = op == "Gemm" and len(node.inputs) > 2
            env[o] = ff.dense(x, wshape[1], ActiMode.AC_MODE_NONE, bias, name=name)
            if w is not None:
                self.weights[name + ".kernel"] = ("copy", np.ascontiguousarray(w))
            if bias and node.inputs[2] in consts:
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


class ONNXModelKeras(ONNXModel):
    """A keras-exported ONNX file (reference onnx/model.py ONNXModelKeras:
    Dense layers as MatMul + Add, channels-first images)."""

    def __init__(self, model, ffconfig=None, ffmodel=None):
        super().__init__(model)
        self.ffconfig, self.ffmodel = ffconfig, ffmodel


# ------------------------------------------------------------------ exporters
def _save(data: bytes, path):
    if path:
        with open(path, "wb") as f:
            f.write(data)
    return data


def export_torch(module, example_inputs, path: Optional[str] = None, export_params: bool = True,
                 input_names: Optional[List[str]] = None) -> bytes:
    """nn.Module -> ONNX (the ``torch.onnx.export`` role; the ``onnx``
    package is not available here).  torch.fx traces the module; leaf
    modules Linear, Conv2d, BatchNorm2d, ReLU, Sigmoid, Tanh, MaxPool2d,
    AvgPool2d, AdaptiveAvgPool2d(1), Flatten, Softmax, Dropout, Identity and
    the functions add / mul / sub / cat / flatten / relu / softmax / view /
    reshape map to ONNX nodes.  Inputs are named ``input.1``, ``input.2``,
    ... as torch's exporter names them.  ``export_params=False`` lists the
    parameters as shaped graph inputs instead of initializers."""
    import operator

    import torch
    import torch.nn as nn
    import torch.nn.functional as F
    from torch.fx.passes.shape_prop import ShapeProp

    gm = torch.fx.symbolic_trace(module)
    ex = tuple(example_inputs) if isinstance(example_inputs, (tuple, list)) else (example_inputs,)
    was = module.training
    module.eval()
    with torch.no_grad():
        ShapeProp(gm).propagate(*ex)
    module.train(was)
    nodes: List[Node] = []
    inits: Dict[str, np.ndarray] = {}
    param_inputs: List[Tuple[str, List[int]]] = []
    inputs: List[Tuple[str, List[int]]] = []
    outputs: List[Tuple[str, List[int]]] = []
    names: Dict[object, str] = {}

    def shp(n):
        return [int(d) for d in n.meta["tensor_meta"].shape]

    def param(pname, t):
        arr = t.detach().cpu().float().numpy()
        if export_params:
            inits[pname] = np.ascontiguousarray(arr)
        else:
            param_inputs.append((pname, list(arr.shape)))
        return pname

    def emit(op, ins, n, **attrs):
        names[n] = n.name
        nodes.append(Node(op, ins, [n.name], n.name, attrs))

    def pair(v):
        return list(v) if isinstance(v, (tuple, list)) else [v, v]

    for n in gm.graph.nodes:
        if n.op == "placeholder":
            nm = (input_names or [])[len(inputs)] if input_names and len(inputs) < len(input_names) else \
                f"input.{len(inputs) + 1}"
            names[n] = nm
            inputs.append((nm, shp(n)))
        elif n.op == "call_module":
            m = gm.get_submodule(n.target)
            x = names[n.args[0]]
            if isinstance(m, nn.Linear):
                ins = [x, param(f"{n.target}.weight", m.weight)]
                if m.bias is not None:
                    ins.append(param(f"{n.target}.bias", m.bias))
                emit("Gemm", ins, n, transB=1)
            elif isinstance(m, nn.Conv2d):
                if m.padding_mode != "zeros" or isinstance(m.padding, str):
                    raise NotImplementedError("Conv2d: explicit zero padding only")
                ins = [x, param(f"{n.target}.weight", m.weight)]
                if m.bias is not None:
                    ins.append(param(f"{n.target}.bias", m.bias))
                ph, pw = pair(m.padding)
                emit("Conv", ins, n, kernel_shape=pair(m.kernel_size), strides=pair(m.stride),
                     pads=[ph, pw, ph, pw], group=int(m.groups), dilations=pair(m.dilation))
            elif isinstance(m, nn.BatchNorm2d):
                ins = [x, param(f"{n.target}.weight", m.weight), param(f"{n.target}.bias", m.bias),
                       param(f"{n.target}.running_mean", m.running_mean),
                       param(f"{n.target}.running_var", m.running_var)]
                emit("BatchNormalization", ins, n, epsilon=float(m.eps), momentum=float(1 - (m.momentum or 0.1)))
            elif isinstance(m, (nn.ReLU, nn.Sigmoid, nn.Tanh, nn.Identity)):
                emit({nn.ReLU: "Relu", nn.Sigmoid: "Sigmoid", nn.Tanh: "Tanh", nn.Identity: "Identity"}[type(m)],
                     [x], n)
            elif isinstance(m, (nn.MaxPool2d, nn.AvgPool2d)):
                if m.ceil_mode:
                    raise NotImplementedError("pooling with ceil_mode")
                ph, pw = pair(m.padding)
                emit("MaxPool" if isinstance(m, nn.MaxPool2d) else "AveragePool", [x], n,
                     kernel_shape=pair(m.kernel_size), strides=pair(m.stride or m.kernel_size), pads=[ph, pw, ph, pw])
            elif isinstance(m, nn.AdaptiveAvgPool2d):
                if pair(m.output_size) != [1, 1]:
                    raise NotImplementedError("AdaptiveAvgPool2d to a size other than 1")
                emit("GlobalAveragePool", [x], n)
            elif isinstance(m, nn.Flatten):
                emit("Flatten", [x], n, axis=int(m.start_dim))
            elif isinstance(m, nn.Softmax):
                emit("Softmax", [x], n, axis=int(m.dim if m.dim is not None else -1))
            elif isinstance(m, nn.Dropout):
                emit("Dropout", [x], n, ratio=float(m.p))
            else:
                raise NotImplementedError(f"export_torch: module {type(m).__name__}")
        elif n.op in ("call_function", "call_method"):
            t = n.target
            a0 = n.args[0] if n.args else None
            if t in (operator.add, operator.iadd, torch.add, "add", "add_"):
                emit("Add", [names[a0], names[n.args[1]]], n)
            elif t in (operator.mul, torch.mul, "mul"):
                emit("Mul", [names[a0], names[n.args[1]]], n)
            elif t in (operator.sub, torch.sub, "sub"):
                emit("Sub", [names[a0], names[n.args[1]]], n)
            elif t is torch.cat:
                dim = n.args[1] if len(n.args) > 1 else n.kwargs.get("dim", 0)
                emit("Concat", [names[v] for v in a0], n, axis=int(dim))
            elif t in (torch.flatten, "flatten"):
                emit("Flatten", [names[a0]], n, axis=int(n.args[1] if len(n.args) > 1 else n.kwargs.get("start_dim", 0)))
            elif t in (torch.relu, F.relu, "relu"):
                emit("Relu", [names[a0]], n)
            elif t in (F.softmax, torch.softmax, "softmax"):
                dim = n.args[1] if len(n.args) > 1 else n.kwargs.get("dim", -1)
                emit("Softmax", [names[a0]], n, axis=int(dim))
            elif t in ("view", "reshape", torch.reshape):
                out = shp(n)
                cname = f"{n.name}.shape"
                inits[cname] = np.asarray([0] + out[1:], dtype=np.int64)   # 0: keep the batch dimension
                emit("Reshape", [names[a0], cname], n)
            else:
                raise NotImplementedError(f"export_torch: function {t}")
        elif n.op == "output":
            res = n.args[0]
            for r in (res if isinstance(res, (tuple, list)) else [res]):
                outputs.append((names[r], shp(r)))
        else:
            raise NotImplementedError(f"export_torch: {n.op} {n.target}")
    return _save(encode_model(nodes, inits, inputs + param_inputs, outputs), path)


def export_keras(model, path: Optional[str] = None, export_params: bool = True) -> bytes:
    """flexflow.keras Model -> ONNX in keras2onnx's form (Dense = MatMul +
    Add, activations as their own nodes, channels-first images; the
    ``keras2onnx.convert_keras`` role).  Inputs are named ``input_1``,
    ``input_2``, ...  Weights come from the compiled model when
    ``export_params`` (the model must have been compiled)."""
    from .keras.layers import (Activation, Add, AveragePooling2D, BatchNormalization, Concatenate, Conv2D, Dense,
                               Dropout, Flatten, InputLayer, MaxPooling2D, Multiply, Permute, Reshape, Subtract)
    from .keras.models import _graph_order

    ff = model.ffmodel if export_params else None
    if export_params and ff is None:
        raise RuntimeError("export_keras: compile the model first (or pass export_params=False)")
    nodes: List[Node] = []
    inits: Dict[str, np.ndarray] = {}
    extra_inputs: List[Tuple[str, List[int]]] = []
    names: Dict[int, str] = {}
    acts = {"relu": "Relu", "sigmoid": "Sigmoid", "tanh": "Tanh", "softmax": "Softmax"}

    def dims(t):
        return [1 if d is None else int(d) for d in t.shape]

    def weights(layer, shapes):
        if ff is None:
            ws = [np.zeros(s, np.float32) for s in shapes]
        else:
            ws = [np.asarray(w, np.float32) for w in layer.get_weights(ff)]
        out = []
        for i, w in enumerate(ws):
            nm = f"{layer.name}/w{i}"
            if export_params:
                inits[nm] = np.ascontiguousarray(w)
            else:
                extra_inputs.append((nm, list(w.shape)))
            out.append(nm)
        return out

    inputs = []
    for i, t in enumerate(model.inputs):
        names[id(t)] = f"input_{i + 1}"
        inputs.append((names[id(t)], dims(t)))
    for t in _graph_order(model.outputs):
        if id(t) in names:
            continue
        L = t.layer
        ins = [names[id(i)] for i in t.inputs]
        o = f"{L.name}/out{len([1 for n in nodes if n.name.startswith(L.name)])}"
        act = None
        if isinstance(L, Dense):
            fin = t.inputs[0].shape[-1]
            w = weights(L, [(fin, L.units)] + ([(L.units,)] if L.use_bias else []))
            mm = o + "/matmul"
            nodes.append(Node("MatMul", [ins[0], w[0]], [mm if L.use_bias else o], L.name, {}))
            if L.use_bias:
                nodes.append(Node("Add", [mm, w[1]], [o], L.name + "/bias", {}))
            act = L.activation
        elif isinstance(L, Conv2D):
            cin = t.inputs[0].shape[1]
            w = weights(L, [(L.filters, cin // L.groups, *L.k)] + ([(L.filters,)] if L.use_bias else []))
            ph, pw = L._pad()
            nodes.append(Node("Conv", [ins[0]] + w, [o], L.name,
                              {"kernel_shape": list(L.k), "strides": list(L.s), "pads": [ph, pw, ph, pw],
                               "group": int(L.groups)}))
            act = L.activation
        elif isinstance(L, (MaxPooling2D, AveragePooling2D)):
            nodes.append(Node("MaxPool" if isinstance(L, MaxPooling2D) else "AveragePool", ins, [o], L.name,
                              {"kernel_shape": list(L.p), "strides": list(L.s),
                               "pads": [L.pad[0], L.pad[1], L.pad[0], L.pad[1]]}))
        elif isinstance(L, Flatten):
            nodes.append(Node("Flatten", ins, [o], L.name, {"axis": 1}))
        elif isinstance(L, Activation):
            if L.activation in (None, "linear"):
                nodes.append(Node("Identity", ins, [o], L.name, {}))
            else:
                nodes.append(Node(acts[L.activation], ins, [o], L.name,
                                  {"axis": -1} if L.activation == "softmax" else {}))
        elif isinstance(L, Concatenate):
            nodes.append(Node("Concat", ins, [o], L.name, {"axis": int(L.axis)}))
        elif isinstance(L, (Add, Subtract, Multiply)):
            op = {Add: "Add", Subtract: "Sub", Multiply: "Mul"}[type(L)]
            cur = ins[0]
            for j, x in enumerate(ins[1:]):
                nxt = o if j == len(ins) - 2 else f"{o}/{j}"
                nodes.append(Node(op, [cur, x], [nxt], f"{L.name}/{j}", {}))
                cur = nxt
        elif isinstance(L, Dropout):
            nodes.append(Node("Dropout", ins, [o], L.name, {"ratio": float(L.rate)}))
        elif isinstance(L, BatchNormalization):
            c = t.inputs[0].shape[1]
            w = weights(L, [(c,), (c,)])
            mean, var = f"{L.name}/mean", f"{L.name}/var"
            inits[mean], inits[var] = np.zeros(c, np.float32), np.ones(c, np.float32)
            nodes.append(Node("BatchNormalization", [ins[0], w[0], w[1], mean, var], [o], L.name,
                              {"epsilon": float(L.epsilon)}))
        elif isinstance(L, Reshape):
            cname = f"{L.name}/shape"
            inits[cname] = np.asarray([0] + list(t.shape[1:]), np.int64)
            nodes.append(Node("Reshape", [ins[0], cname], [o], L.name, {}))
        elif isinstance(L, Permute):
            nodes.append(Node("Transpose", ins, [o], L.name, {"perm": list(L.perm)}))
        elif isinstance(L, InputLayer):
            raise ValueError(f"export_keras: {L.name} is not a model input")
        else:
            raise NotImplementedError(f"export_keras: layer {type(L).__name__}")
        if act not in (None, "linear"):
            pre = o
            o = pre + "/" + act
            nodes[-1].outputs = [pre]
            nodes.append(Node(acts[act], [pre], [o], f"{L.name}/{act}", {"axis": -1} if act == "softmax" else {}))
        names[id(t)] = o
    outputs = [(names[id(t)], dims(t)) for t in model.outputs]
    return _save(encode_model(nodes, inits, inputs + extra_inputs, outputs), path)

