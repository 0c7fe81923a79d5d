"""torch.export (ATen IR) -> FFModel importer.

The reference imports Hugging Face models by tracing them with
``transformers.utils.fx`` (python/flexflow/torch/model.py:2427-2494,
``PyTorchModel(is_hf_model=True)``).  That tracer no longer exists in
transformers 5, and symbolic fx tracing does not get through modern HF
control flow anyway, so models that torch.fx cannot trace are exported with
``torch.export`` instead and the ATen graph is lowered here:

* every value is an FF tensor, a constant, or a parameter;
* a node none of whose inputs is an FF tensor or a parameter is evaluated
  eagerly (constant folding: position-bucket arithmetic, causal masks,
  aranges ...);
* ``aten.linear`` / ``aten.embedding`` become Linear / Embedding layers whose
  weights are copied from the module (``copy_weights``); any other use of a
  parameter (RMS-norm scales, biases added by hand) becomes a standalone
  trainable weight; non-scalar constants that meet an FF tensor become
  constant inputs of the executor;
* ``aten.scaled_dot_product_attention`` is lowered to batch_matmul /
  softmax / batch_matmul with the additive mask.
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

from ..core import ActiMode, AggrMode, DataType

aten = torch.ops.aten


class FFV:
    """An FF tensor in the lowering environment."""

    def __init__(self, t, shape=None):
        self.t = t
        self.shape = tuple(shape if shape is not None else t.dims)


class Param:
    def __init__(self, name: str, tensor: torch.Tensor):
        self.name, self.tensor = name, tensor


_DT = {torch.float32: DataType.DT_FLOAT, torch.float16: DataType.DT_HALF, torch.bfloat16: DataType.DT_BFLOAT16,
       torch.int32: DataType.DT_INT32, torch.int64: DataType.DT_INT64, torch.bool: DataType.DT_BOOLEAN}
_TORCH_DT = {DataType.DT_FLOAT: torch.float32, DataType.DT_INT32: torch.int32, DataType.DT_INT64: torch.int64,
             DataType.DT_HALF: torch.float16, DataType.DT_BFLOAT16: torch.bfloat16, DataType.DT_DOUBLE: torch.float64,
             DataType.DT_BOOLEAN: torch.bool}


def _safe(name: str) -> str:
    return name.replace(".", "_")


class ATenImporter:
    """Lower an ``ExportedProgram`` of ``module(*example_inputs)`` into an
    FFModel.  ``weights`` records {FF layer: {weight: (kind, tensor)}} for
    ``torch_fx.copy_weights`` (the same structure the fx importer uses)."""

    def __init__(self, module: torch.nn.Module, example_inputs: Sequence[torch.Tensor]):
        was = module.training
        module.eval()
        with torch.no_grad():
            ep = torch.export.export(module, tuple(example_inputs), strict=False)
            self.ep = ep.run_decompositions({})
        module.train(was)
        self.weights: Dict[str, Dict[str, tuple]] = {}
        self._n = 0

    # ------------------------------------------------------------------ API
    def to_ff(self, ff, input_tensors: Sequence) -> List:
        self.ff = ff
        self._wcache: Dict[str, FFV] = {}
        ep = self.ep
        state = dict(ep.state_dict)
        consts = dict(getattr(ep, "constants", {}) or {})
        env: Dict[str, object] = {}
        user = list(input_tensors)
        specs = ep.graph_signature.input_specs
        ui = 0
        for spec in specs:
            nm = spec.arg.name
            kind = spec.kind.name
            if kind == "USER_INPUT":
                if ui >= len(user):
                    raise ValueError("fewer FF input tensors than the module's inputs")
                env[nm] = FFV(user[ui])
                ui += 1
            elif kind == "PARAMETER":
                env[nm] = Param(spec.target, state[spec.target].detach())
            elif kind in ("BUFFER", "CONSTANT_TENSOR"):
                src = state.get(spec.target, consts.get(spec.target))
                env[nm] = src.detach() if isinstance(src, torch.Tensor) else src
            else:
                raise NotImplementedError(f"export input kind {kind}")
        outs: List = []
        for node in ep.graph_module.graph.nodes:
            if node.op == "placeholder":
                continue
            if node.op == "output":
                res = node.args[0]
                for r in (res if isinstance(res, (tuple, list)) else [res]):
                    v = self._val(env, r)
                    outs.append(v.t if isinstance(v, FFV) else v)
                continue
            if node.op != "call_function":
                raise NotImplementedError(f"export node {node.op}")
            args = [self._val(env, a) for a in node.args]
            kwargs = {k: self._val(env, v) for k, v in node.kwargs.items()}
            env[node.name] = self._call(node, args, kwargs)
        ff._torch_weights = getattr(ff, "_torch_weights", {})
        ff._torch_weights.update(self.weights)
        return outs

    # ----------------------------------------------------------- machinery
    def _val(self, env, a):
        if isinstance(a, torch.fx.Node):
            return env[a.name]
        if isinstance(a, (list, tuple)):
            return type(a)(self._val(env, x) for x in a)
        return a

    @staticmethod
    def _has(x, kinds) -> bool:
        if isinstance(x, kinds):
            return True
        if isinstance(x, (list, tuple)):
            return any(ATenImporter._has(v, kinds) for v in x)
        return False

    def _name(self, node) -> str:
        self._n += 1
        return f"{node.name}"

    def _weight(self, p: Param) -> FFV:
        """A parameter used outside Linear / Embedding: a standalone weight."""
        if p.name not in self._wcache:
            from .. import _ffcore as C
            from ..core.model import Tensor
            layer = _safe(p.name)
            dt = C.datatype_from_string("float")
            v = self.ff.cg.create_weight(C.TensorShape(list(p.tensor.shape), dt), '{"type":"zero"}', True,
                                         layer + ".w")
            self.weights[layer] = {"w": ("copy", p.tensor)}
            self._wcache[p.name] = FFV(Tensor(self.ff, v, layer + ".w"), p.tensor.shape)
        return self._wcache[p.name]

    def _const(self, c: torch.Tensor, node) -> FFV:
        """A constant that meets an FF tensor: a constant input."""
        c = c.detach()
        if c.dtype == torch.float64:
            c = c.float()
        if c.dtype == torch.bool:
            c = c.to(torch.float32)
        t = self.ff.create_constant_array(np.ascontiguousarray(c.cpu().numpy()), name=f"{node.name}_const")
        return FFV(t, c.shape)

    def _ffv(self, x, node) -> FFV:
        if isinstance(x, FFV):
            return x
        if isinstance(x, Param):
            return self._weight(x)
        if isinstance(x, torch.Tensor):
            return self._const(x, node)
        return self._const(torch.tensor(x, dtype=torch.float32), node)

    @staticmethod
    def _scalar(x) -> Optional[float]:
        if isinstance(x, (int, float, bool)) and not isinstance(x, FFV):
            return float(x)
        if isinstance(x, torch.Tensor) and x.numel() == 1:
            return float(x.reshape(()).item())
        return None

    # ------------------------------------------------------------ lowering
    def _call(self, node, args, kwargs):
        t = node.target
        if t in (aten._assert_tensor_metadata.default, aten._assert_scalar.default) or \
                str(t).startswith("aten.sym_constrain_range"):
            return None
        if not self._has(list(args) + list(kwargs.values()), (FFV, Param)):
            with torch.no_grad():
                return t(*args, **kwargs)            # constant folding
        ff, name = self.ff, self._name(node)
        a0 = args[0] if args else None

        if t == aten.linear.default:
            x, w = args[0], args[1]
            b = args[2] if len(args) > 2 else kwargs.get("bias")
            if not isinstance(w, Param):
                raise NotImplementedError("linear with a non-parameter weight")
            x = self._ffv(x, node)
            out_f = w.tensor.shape[0]
            y = ff.dense(x.t, out_f, ActiMode.AC_MODE_NONE, b is not None, name=name)
            self.weights[name] = {"kernel": ("linear_t", w.tensor)}
            if b is not None:
                self.weights[name]["bias"] = ("copy", b.tensor if isinstance(b, Param) else b)
            return FFV(y)
        if t == aten.embedding.default:
            w, ids = args[0], args[1]
            if not isinstance(w, Param):
                raise NotImplementedError("embedding with a non-parameter table")
            ids = self._ffv(ids, node)
            V, D = w.tensor.shape
            y = ff.embedding(ids.t, V, D, AggrMode.AGGR_MODE_NONE, name=name)
            self.weights[name] = {"weight": ("copy", w.tensor)}
            return FFV(y)
        if t in (aten.add.Tensor, aten.sub.Tensor, aten.mul.Tensor, aten.div.Tensor, aten.rsub.Scalar,
                 aten.add.Scalar, aten.sub.Scalar, aten.mul.Scalar, aten.div.Scalar):
            return self._binary(t, args, kwargs, node, name)
        if t in (aten.view.default, aten.reshape.default, aten._unsafe_view.default):
            x = self._ffv(a0, node)
            shape = list(args[1])
            n = int(np.prod(x.shape))
            if -1 in shape:
                k = int(np.prod([s for s in shape if s != -1]))
                shape[shape.index(-1)] = n // k
            return FFV(ff.reshape(x.t, shape, name=name), shape)
        if t in (aten.unsqueeze.default, aten.squeeze.dim, aten.squeeze.dims):
            x = self._ffv(a0, node)
            shape = list(x.shape)
            if t == aten.unsqueeze.default:
                d = args[1] % (len(shape) + 1)
                shape.insert(d, 1)
            else:
                dims = args[1] if isinstance(args[1], (list, tuple)) else [args[1]]
                dims = sorted({d % len(shape) for d in dims}, reverse=True)
                for d in dims:
                    if shape[d] == 1:
                        shape.pop(d)
            return FFV(ff.reshape(x.t, shape, name=name), shape)
        if t == aten.transpose.int:
            x = self._ffv(a0, node)
            perm = list(range(len(x.shape)))
            d0, d1 = args[1] % len(perm), args[2] % len(perm)
            perm[d0], perm[d1] = perm[d1], perm[d0]
            return FFV(ff.transpose(x.t, perm, name=name))
        if t == aten.permute.default:
            x = self._ffv(a0, node)
            return FFV(ff.transpose(x.t, [p % len(x.shape) for p in args[1]], name=name))
        if t == aten.expand.default:
            # consumers broadcast: the FF tensor keeps its own (broadcastable) shape
            return self._ffv(a0, node)
        if t in (aten.clone.default, aten.alias.default, aten.contiguous.default, aten.detach.default,
                 aten.lift_fresh_copy.default):
            return self._ffv(a0, node)
        if t == aten._to_copy.default:
            x = self._ffv(a0, node)
            dt = kwargs.get("dtype")
            if dt == torch.bool:
                dt = torch.float32      # masks: 0 / 1 floats (inputs are 0 / 1 already)
            cur = _TORCH_DT.get(x.t.data_type)
            if dt is None or dt == cur:
                return x
            return FFV(ff.cast(x.t, _DT[dt], name=name), x.shape)
        if t == aten.index.Tensor:
            return self._index(args, node, name)
        if t in (aten.__and__.Tensor, aten.logical_and.default, aten.bitwise_and.Tensor):
            return self._binary(aten.mul.Tensor, [self._maskf(args[0]), self._maskf(args[1])], {}, node, name)
        if t in (aten.where.self, aten.where.ScalarOther, aten.where.ScalarSelf, aten.where.Scalar):
            return self._where(args, node, name)
        if t in (aten.dropout.default, aten.native_dropout.default):
            x = self._ffv(a0, node)
            return x if t == aten.dropout.default else (x, None)
        if t == aten.pow.Tensor_Scalar:
            return FFV(ff.pow(self._ffv(a0, node).t, float(args[1]), name=name))
        if t == aten.mean.dim:
            x = self._ffv(a0, node)
            dims = [d % len(x.shape) for d in (args[1] if isinstance(args[1], (list, tuple)) else [args[1]])]
            keep = bool(args[2]) if len(args) > 2 else bool(kwargs.get("keepdim", False))
            return FFV(ff.mean(x.t, dims, keep, name=name))
        if t in (aten.sum.dim_IntList,):
            x = self._ffv(a0, node)
            dims = [d % len(x.shape) for d in args[1]]
            keep = bool(args[2]) if len(args) > 2 else bool(kwargs.get("keepdim", False))
            return FFV(ff.reduce_sum(x.t, dims, keep, name=name))
        unary = {aten.rsqrt.default: ff.rsqrt, aten.tanh.default: ff.tanh, aten.relu.default: ff.relu,
                 aten.sigmoid.default: ff.sigmoid, aten.exp.default: ff.exp, aten.sin.default: ff.sin,
                 aten.cos.default: ff.cos}
        if t in unary:
            return FFV(unary[t](self._ffv(a0, node).t, name=name))
        if t == aten.gelu.default:
            return FFV(ff.gelu(self._ffv(a0, node).t, name=name))
        if t == aten.neg.default:
            return FFV(ff.scalar_multiply(self._ffv(a0, node).t, -1.0, name=name))
        if t in (aten._softmax.default, aten.softmax.int):
            x = self._ffv(a0, node)
            return FFV(ff.softmax(x.t, args[1] % len(x.shape), name=name))
        if t in (aten.bmm.default, aten.matmul.default):
            return FFV(ff.batch_matmul(self._ffv(a0, node).t, self._ffv(args[1], node).t, name=name))
        if t == aten.scaled_dot_product_attention.default:
            return self._sdpa(args, kwargs, node, name)
        raise NotImplementedError(f"torch.export lowering: {t}")

    def _binary(self, t, args, kwargs, node, name):
        ff = self.ff
        a, b = args[0], args[1]
        alpha = kwargs.get("alpha", 1)
        kind = {aten.add.Tensor: "add", aten.add.Scalar: "add", aten.sub.Tensor: "sub", aten.sub.Scalar: "sub",
                aten.mul.Tensor: "mul", aten.mul.Scalar: "mul", aten.div.Tensor: "div", aten.div.Scalar: "div",
                aten.rsub.Scalar: "rsub"}[t]
        if kind == "rsub":           # other - a * alpha
            kind, a, b = "sub", b, a
        if alpha != 1:
            sb = self._scalar(b)
            if sb is not None:
                b = sb * alpha
            else:
                b = FFV(ff.scalar_multiply(self._ffv(b, node).t, float(alpha), name=name + "_alpha"))
        sa, sb = self._scalar(a), self._scalar(b)
        if sb is not None and not isinstance(a, (int, float)):
            x = self._ffv(a, node).t
            if kind == "add":
                return FFV(ff.scalar_add(x, sb, name=name))
            if kind == "sub":
                return FFV(ff.scalar_sub(x, sb, name=name))
            if kind == "mul":
                return FFV(ff.scalar_multiply(x, sb, name=name))
            return FFV(ff.scalar_true_divide(x, sb, name=name))
        if sa is not None:
            y = self._ffv(b, node).t
            if kind == "add":
                return FFV(ff.scalar_add(y, sa, name=name))
            if kind == "mul":
                return FFV(ff.scalar_multiply(y, sa, name=name))
            if kind == "sub":        # s - y
                neg = ff.scalar_multiply(y, -1.0, name=name + "_neg")
                return FFV(ff.scalar_add(neg, sa, name=name))
            raise NotImplementedError("scalar / tensor")
        x, y = self._ffv(a, node).t, self._ffv(b, node).t
        fn = {"add": ff.add, "sub": ff.subtract, "mul": ff.multiply, "div": ff.divide}[kind]
        return FFV(fn(x, y, name=name))

    @staticmethod
    def _maskf(x):
        return x.to(torch.float32) if isinstance(x, torch.Tensor) and x.dtype == torch.bool else x

    def _index(self, args, node, name):
        """x[i0, i1, ...] where each index is a constant arange over its own
        dimension broadcast into a larger shape (how HF builds (B, 1, 1, S)
        masks): a reshape to the broadcast shape."""
        x, idx = self._ffv(args[0], node), args[1]
        if any(not isinstance(i, torch.Tensor) for i in idx) or len(idx) != len(x.shape):
            raise NotImplementedError("aten.index with data-dependent indices")
        out = torch.broadcast_shapes(*[i.shape for i in idx])
        pos = []
        for k, i in enumerate(idx):
            nz = [d for d, n in enumerate(i.shape) if n != 1]
            ok = (i.numel() == x.shape[k] and torch.equal(i.reshape(-1).cpu(), torch.arange(x.shape[k])) and
                  len(nz) <= 1 and len(i.shape) == len(out))
            if not ok:
                raise NotImplementedError("aten.index other than an arange gather")
            pos.append(nz[0] if nz else -1)
        if [p for p in pos if p >= 0] != sorted(p for p in pos if p >= 0):
            raise NotImplementedError("aten.index that permutes dimensions")
        return FFV(self.ff.reshape(x.t, list(out), name=name), tuple(out))

    def _where(self, args, node, name):
        """where(c, x, y) on a 0 / 1 mask c as x c + y (1 - c), each term
        formed so nothing cancels (a -1e30 fill never meets the kept
        values); infinite / finfo-min fills are clamped to -+1e30, finite in
        the bf16 compute dtype."""
        ff = self.ff
        c = self._ffv(self._maskf(args[0]), node).t
        x, y = args[1], args[2]

        def fin(v):
            if isinstance(v, torch.Tensor) and v.is_floating_point():
                return v.float().clamp(-1e30, 1e30)
            if isinstance(v, float):
                return max(-1e30, min(1e30, v))
            return v
        x, y = fin(x), fin(y)
        sx, sy = self._scalar(x), self._scalar(y)
        terms = []
        if sx is None:
            terms.append(ff.multiply(c, self._ffv(x, node).t, name=name + "_x"))
        elif sx != 0.0:
            terms.append(ff.scalar_multiply(c, sx, name=name + "_x"))
        if sy is None:
            yt = self._ffv(y, node).t
            terms.append(ff.subtract(yt, ff.multiply(yt, c, name=name + "_yc"), name=name + "_y"))
        elif sy != 0.0:   # y (1 - c) = (c - 1) (-y)
            terms.append(ff.scalar_multiply(ff.scalar_sub(c, 1.0, name=name + "_c1"), -sy, name=name + "_y"))
        if not terms:
            return FFV(ff.scalar_multiply(c, 0.0, name=name))
        out = terms[0]
        for k, t in enumerate(terms[1:]):
            out = ff.add(out, t, name=name if k == len(terms) - 2 else f"{name}_{k}")
        return FFV(out)

    def _sdpa(self, args, kwargs, node, name):
        """softmax(q k^T * scale + mask) v over (B, H, S, D) tensors."""
        ff = self.ff
        names = ["query", "key", "value", "attn_mask", "dropout_p", "is_causal", "scale"]
        p = dict(zip(names, args))
        p.update(kwargs)
        q, k, v = (self._ffv(p[n], node) for n in ("query", "key", "value"))
        d = q.shape[-1]
        scale = p.get("scale")
        scale = 1.0 / math.sqrt(d) if scale is None else float(scale)
        nd = len(k.shape)
        perm = list(range(nd))
        perm[-1], perm[-2] = perm[-2], perm[-1]
        kt = ff.transpose(k.t, perm, name=name + "_kt")
        s = ff.batch_matmul(q.t, kt, name=name + "_qk")
        if scale != 1.0:
            s = ff.scalar_multiply(s, scale, name=name + "_scale")
        mask = p.get("attn_mask")
        if p.get("is_causal"):
            Sq, Sk = q.shape[-2], k.shape[-2]
            causal = torch.full((Sq, Sk), float("-inf")).triu(1)
            mask = causal if mask is None else mask + causal
        if mask is not None:
            if isinstance(mask, torch.Tensor) and mask.dtype == torch.bool:
                mask = torch.zeros(mask.shape).masked_fill(~mask, float("-inf"))
            if isinstance(mask, torch.Tensor):
                mask = mask.clamp(min=torch.finfo(torch.float32).min)
            s = ff.add(s, self._ffv(mask, node).t, name=name + "_mask")
        pr = ff.softmax(s, nd - 1, name=name + "_softmax")
        return FFV(ff.batch_matmul(pr, v.t, name=name))


class HFWrapper(torch.nn.Module):
    """Positional inputs -> HF keyword inputs; returns the first output
    (logits of an LM head model, the last hidden state of a bare model)."""

    def __init__(self, model, input_names: Sequence[str]):
        super().__init__()
        self.model, self.input_names = model, list(input_names)

    def forward(self, *xs):
        out = self.model(**dict(zip(self.input_names, xs)), use_cache=False, return_dict=True)
        return out[0]
