"""Compile a PyTorch module with FlexFlow and keep training it with an
ordinary PyTorch loop (reference: the designed flow of
docs/plantuml/figures/pytorch-tracing.puml:95-232,305-361 — ``model.compile
(algorithm=..., optimizer=...)`` turns an fx-traced module into a
ComputationGraph, optimises it and returns a CompiledModel; the user then
runs ``loss.backward(); optimizer.step()`` as usual.  The reference only
designed this; it has no implementation).

    cm = flexflow.torch.compile(model, example_inputs)     # fx trace -> CG -> search -> executor
    opt = torch.optim.SGD(model.parameters(), lr=0.1)
    for x, y in data:
        loss = loss_fn(cm(x), y)      # forward on the FlexFlow executor (HIP kernels, the searched strategy)
        loss.backward()               # backward on the executor; grads land in model.parameters()
        opt.step(); opt.zero_grad()   # any torch optimizer; changed weights are synced on the next call

The torch module keeps owning the parameters: the executor's weights are
refreshed from them whenever their version counters moved (an in-place
optimizer update), and backward() hands the executor's weight gradients back
in the torch layouts (Linear [out, in], MultiheadAttention in_proj / out_proj).
Inputs get no gradient (they are data)."""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence, Tuple

import torch
from torch import nn

from ..core import DataType, FFConfig, FFModel, SGDOptimizer
from .torch_fx import PyTorchModel, _mha_logical_weight, copy_weights

_DT = {torch.float32: DataType.DT_FLOAT, torch.float16: DataType.DT_HALF, torch.bfloat16: DataType.DT_BFLOAT16,
       torch.int32: DataType.DT_INT32, torch.int64: DataType.DT_INT64}


def _mha_grad_to_torch(mod: nn.MultiheadAttention, g: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """Inverse of torch_fx._mha_logical_weight for a gradient: FlexFlow
    [q|k|v|o per head, heads] -> (in_proj_weight [3E, E], out_proj.weight [E, E])."""
    E, H = mod.embed_dim, mod.num_heads
    d = E // H
    win = torch.zeros(3 * E, E, dtype=g.dtype, device=g.device)
    wo = torch.zeros(E, E, dtype=g.dtype, device=g.device)
    for h in range(H):
        col = g[:, h]
        for j in range(3):
            win[j * E + h * d: j * E + (h + 1) * d] = col[j * E * d:(j + 1) * E * d].view(E, d).t()
        wo[:, h * d:(h + 1) * d] = col[3 * E * d:4 * E * d].view(d, E).t()
    return win, wo


class CompiledModel:
    """``module`` compiled onto the FlexFlow executor (see module docstring)."""

    def __init__(self, module: nn.Module, example_inputs: Sequence[torch.Tensor],
                 ffconfig: Optional[FFConfig] = None, algorithm: Optional[str] = None):
        self.module = module
        cfg = ffconfig or FFConfig()
        ex_in = [torch.as_tensor(t) for t in example_inputs]
        cfg.batch_size = int(ex_in[0].shape[0])
        if algorithm is not None:
            if algorithm in ("data_parallel", "dp"):
                cfg.only_data_parallel = True
            else:
                cfg.search_algorithm = algorithm
        self.ff = FFModel(cfg)
        was_training = module.training
        self.pm = PyTorchModel(module)     # traces in eval mode
        module.train(was_training)         # the caller's mode decides dropout / BN per call
        self.input_tensors = [self.ff.create_tensor(list(t.shape), _DT[t.dtype], name=f"input{i}")
                              for i, t in enumerate(ex_in)]
        self.pm.torch_to_ff(self.ff, self.input_tensors)
        self.ff.compile(optimizer=SGDOptimizer(self.ff, lr=0.0))
        self.ex = self.ff.executor
        self.weights = self.pm.weights()
        # executor parameter name -> (kind, torch object), and the torch
        # parameters in a fixed order (the autograd Function's extra inputs)
        names = set(self.ex.parameter_names())
        self.pmap: Dict[str, Tuple[str, object]] = {}
        for layer, ws in self.weights.items():
            for wname, (kind, t) in ws.items():
                if f"{layer}.{wname}" in names:
                    self.pmap[f"{layer}.{wname}"] = (kind, t)
                if kind == "mha":
                    for extra in ("input_bias", "output_bias"):
                        if f"{layer}.{extra}" in names:
                            self.pmap[f"{layer}.{extra}"] = ("mha_" + extra, t)
        self.params: List[nn.Parameter] = [p for p in module.parameters() if p.requires_grad]
        self._versions: Optional[List[int]] = None
        self._sync_weights(force=True)

    # ---------------------------------------------------------------- weights
    def _sync_weights(self, force: bool = False):
        vers = [p._version for p in self.params]
        if force or vers != self._versions:
            copy_weights(self.ff, self.weights)
            self._versions = vers

    def _grads_to_torch(self) -> Dict[nn.Parameter, torch.Tensor]:
        out: Dict[nn.Parameter, torch.Tensor] = {}

        def put(p, g):
            # always a copy: the executor's gradient buffers are overwritten by
            # the next backward(), possibly before autograd has summed this one
            g = g.reshape(p.shape).to(device=p.device, dtype=p.dtype, copy=True)
            out[p] = out[p] + g if p in out else g

        for pname, (kind, t) in self.pmap.items():
            g = self.ex.get_parameter_grad(pname)
            if kind == "linear_t":
                put(t, g.t())
            elif kind == "mha":
                win, wo = _mha_grad_to_torch(t, g)
                put(t.in_proj_weight, win)
                put(t.out_proj.weight, wo)
            elif kind == "mha_input_bias":
                E, H = t.embed_dim, t.num_heads
                put(t.in_proj_bias, g.view(3, E // H, H).permute(0, 2, 1).reshape(3 * E))
            elif kind == "mha_output_bias":
                put(t.out_proj.bias, g)
            elif isinstance(t, torch.Tensor):
                put(t, g)
        return out

    # ---------------------------------------------------------------- call
    def __call__(self, *inputs: torch.Tensor) -> torch.Tensor:
        self._sync_weights()
        training = self.module.training
        if not torch.is_grad_enabled():
            # inference (torch.no_grad / inference_mode): nothing is saved
            # for a backward; module.eval() turns dropout off and uses running
            # statistics, as in eager PyTorch
            out = self._run(inputs, training, save=False)
            return out.detach().to(device=inputs[0].device, dtype=torch.float32).clone()
        return _FlexFlowFunction.apply(self, training, len(inputs), *inputs, *self.params)

    def _run(self, inputs, training: bool, save: bool) -> torch.Tensor:
        feeds = {t.name: inputs[i] for i, t in enumerate(self.input_tensors)}
        return self.ex.forward(feeds, training=training, keep_outputs=True, save=save)

    forward = __call__


class _FlexFlowFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, cm: CompiledModel, training: bool, n_in: int, *args):
        out = cm._run(args[:n_in], training, save=True)
        ctx.cm, ctx.n_in = cm, n_in
        ctx.out_dtype = out.dtype
        # this call's saved activations: the executor keeps one set, which the
        # next forward() replaces, so several forwards may be pending a
        # backward (f(x1) + f(x2), micro-batches accumulated before backward)
        ctx.exec_state = (cm.ex._saved, cm.ex._env)
        dev = args[0].device
        return out.detach().to(device=dev, dtype=torch.float32).clone()

    @staticmethod
    def backward(ctx, gout):
        cm = ctx.cm
        if ctx.exec_state is None:
            raise RuntimeError("flexflow: backward through the same compiled call twice "
                               "(retain_graph=True is not supported)")
        cm.ex._saved, cm.ex._env = ctx.exec_state
        ctx.exec_state = None
        # an autograd.Function's backward runs with grad mode off; the
        # executor's host fallbacks differentiate with torch autograd
        with torch.enable_grad():
            cm.ex.backward(gout.to(device=cm.ex.cfg.device, dtype=ctx.out_dtype).contiguous())
        grads = cm._grads_to_torch()
        return (None, None, None) + (None,) * ctx.n_in + tuple(grads.get(p) for p in cm.params)


def compile(module: nn.Module, example_inputs: Sequence[torch.Tensor], ffconfig: Optional[FFConfig] = None,
            algorithm: Optional[str] = None) -> CompiledModel:
    """fx-trace ``module`` at the shapes of ``example_inputs``, build its
    ComputationGraph, search a strategy (``algorithm``: "unity" | "mcmc" |
    "data_parallel"; default FFConfig's) and return the CompiledModel."""
    return CompiledModel(module, example_inputs, ffconfig, algorithm)


# ----------------------------------------------------------------- dynamo
# torch.compile(model, backend="flexflow"): dynamo hands the backend a flat
# graph whose parameters are PLACEHOLDERS (nn.Parameter example inputs) used by
# functional ops (torch._C._nn.linear, torch.conv2d, F.layer_norm, ...).  The
# backend rebinds each such op to an nn.Module holding the SAME Parameter
# objects (so gradients still reach the user's parameters), drops the
# parameter placeholders, and compiles the resulting module-structured graph
# with CompiledModel.  Graphs with ops the importer does not map run eagerly.
def _rebind_parameter_ops(gm: torch.fx.GraphModule, example_inputs) -> Tuple[torch.fx.GraphModule, List[int]]:
    import copy

    import torch.nn.functional as F

    # work on a copy: dynamo passes the caller's arguments by the ORIGINAL
    # graph's placeholders
    gm = torch.fx.GraphModule(gm, copy.deepcopy(gm.graph))
    phs = [n for n in gm.graph.nodes if n.op == "placeholder"]
    is_param = {n: isinstance(e, nn.Parameter) for n, e in zip(phs, example_inputs)}
    pval = {n: e for n, e in zip(phs, example_inputs) if is_param[n]}
    root = nn.Module()
    k = 0

    def param_of(a):
        if a is None:
            return None
        if isinstance(a, torch.fx.Node) and is_param.get(a):
            return pval[a]
        raise NotImplementedError("a parameter op whose weight is not a module parameter")

    for node in list(gm.graph.nodes):
        if node.op != "call_function":
            continue
        t, args = node.target, list(node.args)
        if t in (torch._C._nn.linear, F.linear):
            x, w = args[0], param_of(args[1])
            b = param_of(args[2] if len(args) > 2 else node.kwargs.get("bias"))
            m = nn.Linear(w.shape[1], w.shape[0], bias=b is not None)
            m.weight = w
            if b is not None:
                m.bias = b
        elif t in (torch.conv2d, F.conv2d):
            x, w = args[0], param_of(args[1])
            b = param_of(args[2] if len(args) > 2 else node.kwargs.get("bias"))
            stride, padding, dilation, groups = (list(args[3:7]) + [1, 0, 1, 1][len(args[3:7]):])
            m = nn.Conv2d(w.shape[1] * groups, w.shape[0], tuple(w.shape[2:]), stride=stride, padding=padding,
                          dilation=dilation, groups=groups, bias=b is not None)
            m.weight = w
            if b is not None:
                m.bias = b
        elif t is F.layer_norm:
            x, shape = args[0], args[1]
            w = param_of(args[2] if len(args) > 2 else node.kwargs.get("weight"))
            b = param_of(args[3] if len(args) > 3 else node.kwargs.get("bias"))
            eps = args[4] if len(args) > 4 else node.kwargs.get("eps", 1e-5)
            m = nn.LayerNorm(shape, eps=eps, elementwise_affine=w is not None)
            if w is not None:
                m.weight, m.bias = w, b
        elif t in (F.max_pool2d, torch.max_pool2d, F.avg_pool2d, torch._C._nn.avg_pool2d):
            x = args[0]
            ks = args[1] if len(args) > 1 else node.kwargs["kernel_size"]
            st = args[2] if len(args) > 2 else node.kwargs.get("stride", None)
            pd = args[3] if len(args) > 3 else node.kwargs.get("padding", 0)
            cls = nn.MaxPool2d if t in (F.max_pool2d, torch.max_pool2d) else nn.AvgPool2d
            m = cls(ks, stride=st or ks, padding=pd)
        elif t in (F.embedding, torch.embedding):
            x, w = (args[0], param_of(args[1])) if t is F.embedding else (args[1], param_of(args[0]))
            m = nn.Embedding(w.shape[0], w.shape[1])
            m.weight = w
        else:
            if any(isinstance(a, torch.fx.Node) and is_param.get(a) for a in args):
                raise NotImplementedError(f"parameter used by {t}")
            continue
        name = f"ff_mod{k}"
        k += 1
        root.add_module(name, m)
        gm.add_submodule(name, m)
        with gm.graph.inserting_before(node):
            new = gm.graph.call_module(name, (x,))
        node.replace_all_uses_with(new)
        gm.graph.erase_node(node)
    data_pos = [i for i, n in enumerate(phs) if not is_param[n]]
    for n in phs:
        if is_param[n]:
            if n.users:
                raise NotImplementedError("a parameter is used outside a module-mapped op")
            gm.graph.erase_node(n)
    gm.graph.lint()
    return torch.fx.GraphModule(root, gm.graph), data_pos


COMPILED: List[CompiledModel] = []   # graphs the backend compiled (introspection / tests)


def flexflow_backend(gm: torch.fx.GraphModule, example_inputs, ffconfig: Optional[FFConfig] = None):
    """The ``backend="flexflow"`` entry point for torch.compile."""
    import warnings

    try:
        mod, data_pos = _rebind_parameter_ops(gm, example_inputs)
        cm = CompiledModel(mod, [example_inputs[i] for i in data_pos], ffconfig)
    except Exception as e:  # noqa: BLE001 — unsupported graph: dynamo runs it eagerly
        warnings.warn(f"flexflow backend: running this graph eagerly ({type(e).__name__}: {e})")
        return gm.forward

    def run(*args):
        out = cm(*[args[i] for i in data_pos])
        return (out,)

    run.compiled_model = cm
    COMPILED.append(cm)
    return run


def backend(**config):
    """A configured backend: ``torch.compile(m, backend=flexflow.torch.backend(
    cpu_only=True, search_algorithm="mcmc"))`` (FFConfig fields)."""
    def _be(gm, example_inputs):
        cfg = FFConfig()
        for k, v in config.items():
            if not hasattr(cfg, k):
                raise AttributeError(f"FFConfig has no field {k}")
            setattr(cfg, k, v)
        return flexflow_backend(gm, example_inputs, cfg)
    return _be


def _register_dynamo_backend():
    try:
        from torch._dynamo import register_backend
    except Exception:  # noqa: BLE001 — dynamo unavailable
        return
    try:
        register_backend(name="flexflow")(flexflow_backend)
    except Exception:  # noqa: BLE001 — already registered
        pass


_register_dynamo_backend()
