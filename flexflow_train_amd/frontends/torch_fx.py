"""PyTorch -> FFModel importer (torch.fx) and the ``.ff`` text IR.

Parity: python/flexflow/torch/model.py — ``PyTorchModel(model, ...)``,
``torch_to_ff(ffmodel, inputs)`` (:2496-2538), ``torch_to_file(path)``
(:2597-2604) and ``file_to_ff(path, ffmodel, inputs)`` (:2540-2574).  The
``.ff`` format is one node per line::

    name; in1,in2,; out1,; OPTYPE; arg1; arg2; ...

(``IR_DELIMITER = "; "``, ``INOUT_NODE_DELIMITER = ","``), with the
reference's op names and argument orders for the shared ops (LINEAR:
out_features, acti, bias; CONV2D: out, kh, kw, sh, sw, ph, pw, acti, groups,
bias; POOL2D: kernel, stride, padding, pool_type, acti; ...) and enum
integers from core.types.

Design: fx nodes are lowered through a table of small converters that each
emit one FFModel call *and* one IR line, so the in-memory path and the file
path share a single mapping.  ``copy_weights(ffmodel)`` moves the torch
parameters into the compiled model (the reference has no weight transfer;
it is what makes the importer testable against torch numerics).
"""
from __future__ import annotations

import operator
from typing import Callable, Dict, List, Optional, Sequence

import torch
import torch.fx
import torch.nn as nn
import torch.nn.functional as F

from ..core.types import ActiMode, AggrMode, PoolType

IR_DELIMITER = "; "
INOUT_NODE_DELIMITER = ","


def _acti_int(a: ActiMode = ActiMode.AC_MODE_NONE) -> str:
    return str(a.value)


class _Emitter:
    """Builds FFModel tensors (if ``ffmodel``) and IR lines for fx nodes."""

    def __init__(self, ffmodel=None):
        self.ff = ffmodel
        self.lines: List[str] = []
        self.out: Dict[str, object] = {}      # node name -> FF tensor (or tuple of tensors)
        self.weights: Dict[str, tuple] = {}    # FF layer name -> (weight name -> torch param)

    def line(self, name, ins, outs, op, *args):
        s = [name, INOUT_NODE_DELIMITER.join(ins) + (INOUT_NODE_DELIMITER if ins else ""),
             INOUT_NODE_DELIMITER.join(outs) + (INOUT_NODE_DELIMITER if outs else ""), op]
        s += [str(a) for a in args]
        self.lines.append(IR_DELIMITER.join(s))


def _args_nodes(args) -> List[str]:
    out = []
    for a in args:
        if isinstance(a, torch.fx.Node):
            out.append(a.name)
        elif isinstance(a, (list, tuple)):
            out += _args_nodes(a)
    return out


class PyTorchModel:
    """Wraps an ``nn.Module`` for conversion to FlexFlow."""

    def __init__(self, model: nn.Module, is_hf_model: bool = False, input_names: Optional[Sequence[str]] = None,
                 batch_size: int = 1, seq_length: Optional[int] = None):
        self.model = model.eval()
        self.is_hf_model = is_hf_model
        self.input_names = list(input_names or [])
        self.batch_size = batch_size
        self.seq_length = seq_length
        # Hugging Face models (and anything torch.fx cannot trace) go through
        # torch.export + the ATen lowering (torch_export.py) at torch_to_ff
        # time, with example inputs shaped like the FF input tensors: the
        # reference's transformers.utils.fx tracer is gone in transformers 5
        self.graph = None
        self.trace_error = None
        if not is_hf_model:
            try:
                self.graph = torch.fx.symbolic_trace(self.model)
            except Exception as e:   # data-dependent control flow etc.
                self.trace_error = e
        self.modules = dict(self.model.named_modules())

    def _export_to_ff(self, ffmodel, input_tensors: Sequence, verbose: bool):
        from .torch_export import ATenImporter, HFWrapper, _TORCH_DT

        ex = []
        for t in input_tensors:
            dt = _TORCH_DT.get(t.data_type, torch.float32)
            ex.append(torch.ones(list(t.dims), dtype=dt) if not dt.is_floating_point
                      else torch.randn(list(t.dims), dtype=dt))
        mod = HFWrapper(self.model, self.input_names) if self.is_hf_model else self.model
        imp = ATenImporter(mod, ex)
        outs = imp.to_ff(ffmodel, list(input_tensors))
        self._importer = imp
        if verbose:
            print(imp.ep.graph_module.graph)
        return outs

    # ------------------------------------------------------------------ API
    def torch_to_ff(self, ffmodel, input_tensors: Sequence, verbose: bool = False):
        if self.graph is None:
            return self._export_to_ff(ffmodel, input_tensors, verbose)
        em = _Emitter(ffmodel)
        outs = self._lower(em, list(input_tensors))
        self._last_emitter = em
        ffmodel._torch_weights = getattr(ffmodel, "_torch_weights", {})
        ffmodel._torch_weights.update(em.weights)
        if verbose:
            print("\n".join(em.lines))
        return outs

    def weights(self) -> Dict[str, dict]:
        """FF layer name -> {weight name: (layout, torch parameter)} for
        ``copy_weights`` (the same names ``torch_to_ff``/``file_to_ff`` use)."""
        if self.graph is None:
            imp = getattr(self, "_importer", None)
            if imp is None:
                raise RuntimeError("call torch_to_ff first (torch.export path)")
            return imp.weights
        em = _Emitter(None)
        self._lower(em, None)
        return em.weights

    def torch_to_string(self) -> List[str]:
        if self.graph is None:
            raise NotImplementedError("the .ff text IR covers torch.fx-traceable modules; import this model with "
                                      "torch_to_ff (torch.export path)" +
                                      (f" (fx: {self.trace_error})" if self.trace_error else ""))
        em = _Emitter(None)
        self._lower(em, None)
        return em.lines

    def torch_to_file(self, path: str):
        with open(path, "w") as f:
            f.write("\n".join(self.torch_to_string()) + "\n")

    @staticmethod
    def file_to_ff(path: str, ffmodel, input_tensors: Sequence):
        with open(path) as f:
            return string_to_ff([ln for ln in f.read().splitlines() if ln.strip()], ffmodel, input_tensors)

    # ------------------------------------------------------------ lowering
    def _lower(self, em: _Emitter, inputs: Optional[List]):
        placeholders = [n for n in self.graph.graph.nodes if n.op == "placeholder"]
        if inputs is not None and len(inputs) != len(placeholders):
            raise ValueError(f"model has {len(placeholders)} inputs, got {len(inputs)} tensors")
        outputs = []
        for node in self.graph.graph.nodes:
            if node.op == "placeholder":
                k = placeholders.index(node)
                em.line(node.name, [], [u.name for u in node.users], "INPUT")
                if inputs is not None:
                    em.out[node.name] = inputs[k]
            elif node.op == "output":
                res = node.args[0]
                names = _args_nodes([res])
                em.line(node.name, names, [], "OUTPUT")
                outputs = [em.out.get(n) for n in names] if em.ff is not None else names
            elif node.op == "call_module":
                self._module(em, node, self.modules[node.target])
            elif node.op in ("call_function", "call_method"):
                _function(em, node)
            elif node.op == "get_attr":
                raise NotImplementedError(f"get_attr {node.target} (module attributes are not supported)")
        return list(outputs)   # a list, as the reference's torch_to_ff / file_to_ff return

    def _module(self, em: _Emitter, node, mod: nn.Module):
        ins = _args_nodes(node.args)
        outs = [u.name for u in node.users]
        x = em.out.get(ins[0]) if ins else None
        ff = em.ff
        name = node.name

        def emit(op, *args, fn: Optional[Callable] = None, weights=None):
            em.line(name, ins, outs, op, *args)
            if weights:
                em.weights[name] = weights
            if ff is not None and fn is not None:
                em.out[name] = fn()

        if isinstance(mod, nn.Linear):
            emit("LINEAR", mod.out_features, _acti_int(), int(mod.bias is not None),
                 fn=lambda: ff.dense(x, mod.out_features, ActiMode.AC_MODE_NONE, mod.bias is not None, name=name),
                 weights={"kernel": ("linear_t", mod.weight), **({"bias": ("copy", mod.bias)} if mod.bias is not None
                                                                  else {})})
        elif isinstance(mod, nn.Conv2d):
            kh, kw = mod.kernel_size
            sh, sw = mod.stride
            ph, pw = mod.padding
            emit("CONV2D", mod.out_channels, kh, kw, sh, sw, ph, pw, _acti_int(), mod.groups, int(mod.bias is not None),
                 fn=lambda: ff.conv2d(x, mod.out_channels, kh, kw, sh, sw, ph, pw, ActiMode.AC_MODE_NONE, mod.groups,
                                      mod.bias is not None, name=name),
                 weights={"kernel": ("copy", mod.weight), **({"bias": ("copy", mod.bias)} if mod.bias is not None
                                                              else {})})
        elif isinstance(mod, (nn.MaxPool2d, nn.AvgPool2d)):
            k = mod.kernel_size if isinstance(mod.kernel_size, int) else mod.kernel_size[0]
            s = mod.stride if isinstance(mod.stride, int) else mod.stride[0]
            p = mod.padding if isinstance(mod.padding, int) else mod.padding[0]
            pt = PoolType.POOL_MAX if isinstance(mod, nn.MaxPool2d) else PoolType.POOL_AVG
            emit("POOL2D", k, s, p, pt.value, _acti_int(),
                 fn=lambda: ff.pool2d(x, k, k, s, s, p, p, pt, name=name))
        elif isinstance(mod, nn.AdaptiveAvgPool2d):
            out_hw = mod.output_size if isinstance(mod.output_size, int) else mod.output_size[0]
            emit("ADAPTIVE_POOL2D", out_hw, PoolType.POOL_AVG.value, _acti_int(), fn=lambda: _adaptive_pool(ff, x, out_hw, name))
        elif isinstance(mod, nn.BatchNorm2d):
            emit("BATCH_NORM", fn=lambda: ff.batch_norm(x, False, name=name),
                 weights={"gamma": ("copy", mod.weight), "beta": ("copy", mod.bias)})
        elif isinstance(mod, nn.LayerNorm):
            emit("LAYER_NORM", fn=lambda: ff.layer_norm(x, [-1], mod.elementwise_affine, mod.eps, name=name),
                 weights={"gamma": ("copy", mod.weight), "beta": ("copy", mod.bias)} if mod.elementwise_affine else None)
        elif isinstance(mod, nn.Embedding):
            emit("EMBEDDING", mod.num_embeddings, mod.embedding_dim, AggrMode.AGGR_MODE_NONE.value,
                 fn=lambda: ff.embedding(x, mod.num_embeddings, mod.embedding_dim, AggrMode.AGGR_MODE_NONE, name=name),
                 weights={"weight": ("copy", mod.weight)})
        elif isinstance(mod, nn.Dropout):
            emit("DROPOUT", mod.p, fn=lambda: ff.dropout(x, mod.p, 0, name=name))
        elif isinstance(mod, nn.Flatten):
            emit("FLAT", fn=lambda: ff.flat(x, name=name))
        elif isinstance(mod, nn.Softmax):
            emit("SOFTMAX", mod.dim if mod.dim is not None else -1,
                 fn=lambda: ff.softmax(x, mod.dim if mod.dim is not None else -1, name=name))
        elif isinstance(mod, (nn.ReLU, nn.GELU, nn.Sigmoid, nn.Tanh, nn.ELU, nn.Identity)):
            op = {nn.ReLU: "RELU", nn.GELU: "GELU", nn.Sigmoid: "SIGMOID", nn.Tanh: "TANH", nn.ELU: "ELU",
                  nn.Identity: "IDENTITY"}[type(mod)]
            emit(op, fn=lambda: _unary(ff, op, x, name))
        elif isinstance(mod, nn.MultiheadAttention):
            if not mod.batch_first:
                raise NotImplementedError("nn.MultiheadAttention must be batch_first")
            q, k, v = (em.out.get(n) for n in ins[:3])
            emit("MULTIHEAD_ATTENTION", mod.embed_dim, mod.num_heads, mod.dropout,
                 # torch returns (output, attention weights); weights are not materialized
                 fn=lambda: (ff.multihead_attention(q, k, v, mod.embed_dim, mod.num_heads,
                                                    bias=mod.in_proj_bias is not None, name=name), None),
                 weights={"weight": ("mha", mod)})
        else:
            raise NotImplementedError(f"module {type(mod).__name__} ({node.target})")


def _unary(ff, op, x, name):
    return {"RELU": lambda: ff.relu(x, name=name), "GELU": lambda: ff.gelu(x, name=name),
            "SIGMOID": lambda: ff.sigmoid(x, name=name), "TANH": lambda: ff.tanh(x, name=name),
            "ELU": lambda: ff.elu(x, name=name), "IDENTITY": lambda: ff.identity(x, name=name),
            "EXP": lambda: ff.exp(x, name=name), "SIN": lambda: ff.sin(x, name=name),
            "COS": lambda: ff.cos(x, name=name), "RSQRT": lambda: ff.rsqrt(x, name=name)}[op]()


def _adaptive_pool(ff, x, out_hw, name):
    h = x.dims[-1]
    if h % out_hw:
        raise NotImplementedError("adaptive pooling with a non-divisible output size")
    k = h // out_hw
    return ff.pool2d(x, k, k, k, k, 0, 0, PoolType.POOL_AVG, name=name)


_BINARY = {operator.add: "ADD", torch.add: "ADD", operator.sub: "SUBTRACT", torch.sub: "SUBTRACT",
           operator.mul: "MULTIPLY", torch.mul: "MULTIPLY", operator.truediv: "DIVIDE", torch.div: "DIVIDE",
           "add": "ADD", "sub": "SUBTRACT", "mul": "MULTIPLY", "div": "DIVIDE", "truediv": "DIVIDE"}
_SCALAR = {"ADD": "SCALAR_ADD", "SUBTRACT": "SCALAR_SUB", "MULTIPLY": "SCALAR_MULTIPLY", "DIVIDE": "SCALAR_TRUEDIV"}
_UNARY_FN = {F.relu: "RELU", torch.relu: "RELU", F.gelu: "GELU", torch.sigmoid: "SIGMOID", F.sigmoid: "SIGMOID",
             torch.tanh: "TANH", F.tanh: "TANH", F.elu: "ELU", torch.exp: "EXP", torch.sin: "SIN", torch.cos: "COS",
             torch.rsqrt: "RSQRT", "relu": "RELU", "sigmoid": "SIGMOID", "tanh": "TANH", "exp": "EXP",
             "contiguous": "IDENTITY", "float": "IDENTITY"}


def _function(em: _Emitter, node):
    ff = em.ff
    name = node.name
    tgt = node.target
    ins = _args_nodes(node.args)
    outs = [u.name for u in node.users]
    get = em.out.get

    def emit(op, *args, fn=None):
        em.line(name, ins, outs, op, *args)
        if ff is not None and fn is not None:
            em.out[name] = fn()

    if tgt in _BINARY:
        op = _BINARY[tgt]
        a, b = node.args[0], node.args[1]
        if isinstance(a, torch.fx.Node) and isinstance(b, torch.fx.Node):
            fns = {"ADD": "add", "SUBTRACT": "subtract", "MULTIPLY": "multiply", "DIVIDE": "divide"}
            emit(op, fn=lambda: getattr(ff, fns[op])(get(a.name), get(b.name), name=name))
        else:
            x, s = (a, b) if isinstance(a, torch.fx.Node) else (b, a)
            sop = _SCALAR[op]
            if not isinstance(a, torch.fx.Node) and op in ("SUBTRACT", "DIVIDE"):
                raise NotImplementedError(f"scalar {op} with the scalar on the left")
            fns = {"SCALAR_ADD": "scalar_add", "SCALAR_SUB": "scalar_sub", "SCALAR_MULTIPLY": "scalar_multiply",
                   "SCALAR_TRUEDIV": "scalar_true_divide"}
            emit(sop, float(s), fn=lambda: getattr(ff, fns[sop])(get(x.name), float(s), name=name))
    elif tgt in _UNARY_FN:
        op = _UNARY_FN[tgt]
        emit(op, fn=lambda: _unary(ff, op, get(ins[0]), name))
    elif tgt in (torch.cat, torch.concat):
        axis = node.kwargs.get("dim", node.args[1] if len(node.args) > 1 else 0)
        emit("CONCAT", axis, fn=lambda: ff.concat([get(n) for n in ins], axis, name=name))
    elif tgt in (torch.flatten,) or tgt == "flatten":
        emit("FLAT", fn=lambda: ff.flat(get(ins[0]), name=name))
    elif tgt in (F.softmax, torch.softmax) or tgt == "softmax":
        dim = node.kwargs.get("dim", node.args[1] if len(node.args) > 1 else -1)
        emit("SOFTMAX", dim, fn=lambda: ff.softmax(get(ins[0]), dim, name=name))
    elif tgt in (torch.matmul, torch.bmm) or tgt in ("matmul", "bmm"):
        emit("BATCH_MATMUL", fn=lambda: ff.batch_matmul(get(ins[0]), get(ins[1]), name=name))
    elif tgt in ("view", "reshape") or tgt is torch.reshape:
        shape = [int(s) for s in (node.args[1:] if not isinstance(node.args[1], (list, tuple)) else node.args[1])]
        emit("RESHAPE", *shape, fn=lambda: ff.reshape(get(ins[0]), _resolve_shape(get(ins[0]), shape), name=name))
    elif tgt in ("permute",) or tgt is torch.permute:
        perm = [int(p) for p in (node.args[1:] if not isinstance(node.args[1], (list, tuple)) else node.args[1])]
        emit("PERMUTE", *perm, fn=lambda: ff.transpose(get(ins[0]), perm, name=name))
    elif tgt in ("transpose",) or tgt is torch.transpose:
        d0, d1 = int(node.args[1]), int(node.args[2])

        def tr():
            x = get(ins[0])
            perm = list(range(len(x.dims)))
            perm[d0], perm[d1] = perm[d1], perm[d0]
            return ff.transpose(x, perm, name=name)
        emit("TRANSPOSE", d0, d1, fn=tr)
    elif tgt in ("mean",) or tgt is torch.mean:
        dims = node.args[1] if len(node.args) > 1 else node.kwargs.get("dim")
        dims = [dims] if isinstance(dims, int) else list(dims)
        keep = bool(node.kwargs.get("keepdim", False))
        emit("MEAN", *dims, int(keep), fn=lambda: ff.mean(get(ins[0]), dims, keep, name=name))
    elif tgt in (torch.split, torch.chunk) or tgt in ("split", "chunk"):
        sizes = node.args[1]
        dim = node.kwargs.get("dim", node.args[2] if len(node.args) > 2 else 0)

        def sp():
            x = get(ins[0])
            n = x.dims[dim]
            if tgt in (torch.chunk, "chunk"):
                k = int(sizes)
                sz = [n // k] * k
            elif isinstance(sizes, int):
                sz = [sizes] * (n // sizes)
            else:
                sz = list(sizes)
            return tuple(ff.split(x, sz, dim, name=name))
        emit("SPLIT", sizes, dim, fn=sp)
    elif tgt is operator.getitem:
        idx = node.args[1]
        emit("GETITEM", idx, fn=lambda: get(ins[0])[idx])
    elif tgt is F.dropout:
        p = node.kwargs.get("p", node.args[1] if len(node.args) > 1 else 0.5)
        emit("DROPOUT", p, fn=lambda: ff.dropout(get(ins[0]), p, 0, name=name))
    else:
        raise NotImplementedError(f"fx target {tgt}")


def _resolve_shape(x, shape):
    total = 1
    for d in x.dims:
        total *= d
    if -1 in shape:
        known = 1
        for s in shape:
            if s != -1:
                known *= s
        shape = [total // known if s == -1 else s for s in shape]
    return shape


def string_to_ff(lines: Sequence[str], ffmodel, input_tensors: Sequence):
    """Replay a ``.ff`` IR into ``ffmodel`` (reference: file_to_ff)."""
    env: Dict[str, object] = {}
    inputs = list(input_tensors)
    out = []
    for ln in lines:
        items = [i.strip() for i in ln.split(";")]
        name = items[0]
        ins = [s.strip() for s in items[1].split(INOUT_NODE_DELIMITER) if s.strip()] if len(items) > 1 else []
        op = items[3] if len(items) > 3 else items[1]
        a = items[4:]
        x = env.get(ins[0]) if ins else None
        f = ffmodel
        if op == "INPUT":
            env[name] = inputs.pop(0)
        elif op == "OUTPUT":
            out = [env[n] for n in ins]
        elif op == "LINEAR":
            env[name] = f.dense(x, int(a[0]), ActiMode(int(a[1])), bool(int(a[2])), name=name)
        elif op == "CONV2D":
            env[name] = f.conv2d(x, int(a[0]), int(a[1]), int(a[2]), int(a[3]), int(a[4]), int(a[5]), int(a[6]),
                                 ActiMode(int(a[7])), int(a[8]), bool(int(a[9])), name=name)
        elif op == "POOL2D":
            k, s, p = int(a[0]), int(a[1]), int(a[2])
            env[name] = f.pool2d(x, k, k, s, s, p, p, PoolType(int(a[3])), ActiMode(int(a[4])), name=name)
        elif op == "ADAPTIVE_POOL2D":
            env[name] = _adaptive_pool(f, x, int(a[0]), name)
        elif op == "BATCH_NORM":
            env[name] = f.batch_norm(x, False, name=name)
        elif op == "LAYER_NORM":
            env[name] = f.layer_norm(x, [-1], name=name)
        elif op == "EMBEDDING":
            env[name] = f.embedding(x, int(a[0]), int(a[1]), AggrMode(int(a[2])), name=name)
        elif op == "DROPOUT":
            env[name] = f.dropout(x, float(a[0]), 0, name=name)
        elif op == "FLAT":
            env[name] = f.flat(x, name=name)
        elif op == "SOFTMAX":
            env[name] = f.softmax(x, int(a[0]) if a else -1, name=name)
        elif op in ("RELU", "GELU", "SIGMOID", "TANH", "ELU", "IDENTITY", "EXP", "SIN", "COS", "RSQRT"):
            env[name] = _unary(f, op, x, name)
        elif op in ("ADD", "SUBTRACT", "MULTIPLY", "DIVIDE"):
            fn = {"ADD": f.add, "SUBTRACT": f.subtract, "MULTIPLY": f.multiply, "DIVIDE": f.divide}[op]
            env[name] = fn(env[ins[0]], env[ins[1]], name=name)
        elif op in ("SCALAR_ADD", "SCALAR_SUB", "SCALAR_MULTIPLY", "SCALAR_TRUEDIV"):
            fn = {"SCALAR_ADD": f.scalar_add, "SCALAR_SUB": f.scalar_sub, "SCALAR_MULTIPLY": f.scalar_multiply,
                  "SCALAR_TRUEDIV": f.scalar_true_divide}[op]
            env[name] = fn(x, float(a[0]), name=name)
        elif op == "CONCAT":
            env[name] = f.concat([env[n] for n in ins], int(a[0]), name=name)
        elif op == "BATCH_MATMUL":
            env[name] = f.batch_matmul(env[ins[0]], env[ins[1]], name=name)
        elif op == "RESHAPE":
            env[name] = f.reshape(x, _resolve_shape(x, [int(v) for v in a]), name=name)
        elif op == "PERMUTE":
            env[name] = f.transpose(x, [int(v) for v in a], name=name)
        elif op == "TRANSPOSE":
            perm = list(range(len(x.dims)))
            d0, d1 = int(a[0]), int(a[1])
            perm[d0], perm[d1] = perm[d1], perm[d0]
            env[name] = f.transpose(x, perm, name=name)
        elif op == "MEAN":
            env[name] = f.mean(x, [int(v) for v in a[:-1]], bool(int(a[-1])), name=name)
        elif op == "MULTIHEAD_ATTENTION":
            q, k, v = (env[n] for n in ins[:3])
            env[name] = f.multihead_attention(q, k, v, int(a[0]), int(a[1]), name=name)
        elif op == "SPLIT":
            import ast

            sizes, dim = ast.literal_eval(a[0]), int(a[1])
            n = x.dims[dim]
            sz = [sizes] * (n // sizes) if isinstance(sizes, int) else list(sizes)
            env[name] = tuple(f.split(x, sz, dim, name=name))
        elif op == "GETITEM":
            env[name] = x[int(a[0])]
        else:
            raise NotImplementedError(f".ff op {op}")
    return list(out)


def copy_weights(ffmodel, torch_weights: Optional[Dict] = None):
    """Copy torch parameters recorded by ``torch_to_ff`` into the compiled
    model (Linear kernels are stored [in, out] in FlexFlow)."""
    ex = ffmodel.executor
    tw = torch_weights if torch_weights is not None else getattr(ffmodel, "_torch_weights", {})
    names = set(ex.parameter_names())
    for layer, ws in tw.items():
        for wname, (kind, t) in ws.items():
            pname = f"{layer}.{wname}"
            if pname not in names:
                continue
            if kind == "linear_t":
                val = t.detach().t().contiguous()
            elif kind == "mha":
                val = _mha_logical_weight(t)
            else:
                val = t.detach()
            ex.set_parameter(pname, val.float().reshape(ex.get_parameter(pname).shape))
        if any(k == "mha" for k, _ in ws.values()):
            mod = next(t for k, t in ws.values() if k == "mha")
            if mod.in_proj_bias is not None:
                E, H = mod.embed_dim, mod.num_heads
                d = E // H
                b = mod.in_proj_bias.detach().view(3, H, d).permute(0, 2, 1).reshape(3 * d, H)
                if f"{layer}.input_bias" in names:
                    ex.set_parameter(f"{layer}.input_bias", b.float())
                if f"{layer}.output_bias" in names:
                    ex.set_parameter(f"{layer}.output_bias", mod.out_proj.bias.detach().float())


def _mha_logical_weight(mod: nn.MultiheadAttention) -> torch.Tensor:
    """torch in_proj/out_proj -> FlexFlow [q|k|v|o per head, heads] layout."""
    E, H = mod.embed_dim, mod.num_heads
    d = E // H
    W = mod.in_proj_weight.detach()           # [3E, E]  (y = x W^T)
    cols = []
    for h in range(H):
        parts = []
        for j in range(3):
            Wj = W[j * E + h * d: j * E + (h + 1) * d]   # [d, E]
            parts.append(Wj.t().reshape(-1))             # [E, d]
        Wo = mod.out_proj.weight.detach()[:, h * d:(h + 1) * d]  # [E, d] -> per-head [d, E]
        parts.append(Wo.t().reshape(-1))
        cols.append(torch.cat(parts))
    return torch.stack(cols, dim=1)
