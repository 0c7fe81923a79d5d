"""Per-rank executor of a ParallelComputationGraph.

This is the MI355X replacement of the reference's Legion runtime
(lib/runtime: FFModel/LegionBacking/FFMapper/NCCL communicators) and of the
single-device LocalTrainingBacking (lib/local-execution/src/
local_training_backing.cc:50-163):

* one process per GPU; the PCG is lowered ONCE into a flat list of steps for
  this rank (compute steps on local shards, redistribution steps for the
  parallel operators and for machine-view changes), executed on the current
  HIP stream; hipGraph capture of a whole iteration replaces Legion tracing;
* weights: the WEIGHT -> Repartition/Replicate chains of the PCG are folded
  into the parameter's resident layout; all parameter pieces of a rank live
  in ONE flat fp32 master buffer (+ bf16 compute copy + fp32 gradient buffer)
  per gradient-sync group; gradients are reduced with bucketed RCCL
  all-reduces launched as soon as the backward pass finalises each bucket
  (overlapped with the rest of the backward — the reference simulator's
  "overlap backward and update" mode, simulator.cc:914-955);
* the optimizer update is one fused launch per flat buffer;
* loss + metrics are fused with the trailing softmax (loss.py).
"""
from __future__ import annotations

import contextlib
import dataclasses
import gc
import hashlib
import json
import math
import os
import time
from typing import Any, Callable, Dict, List, Optional, Sequence, Tuple

import torch

from .. import _ffcore as C
from .. import kernels as K
from .. import ops as _ops_pkg  # noqa: F401  (registers operator impls)
from ..ops import base as opbase
from ..ops.loss import N_SLOTS, LossFunction, PerfMetrics
from ..parallel.comm import DistContext, Redistributor
from ..parallel.layout import Layout, layout_from_pshape, placement
from ..parallel.halo import HaloGroup, HaloPlan
from ..parallel.sequence import SeqGroup
from ..ops.moe import ExpertGroup
from .optimizer import AdamConfig, FlatOptimizer, SGDConfig, ShardedOptimizer
from .graphs import SegmentRecorder
from .graphs import _native_module as _native_replay_module
from .initializers import make_initializer_tensor
from ..utils.tracing import Tracer

Value = Tuple[int, int]
_PAR_OPS = {"REPARTITION", "COMBINE", "REPLICATE", "REDUCTION", "ALLTOALL", "FUSED_PARALLEL"}
_TORCH_DT = {"float": torch.float32, "double": torch.float64, "half": torch.float16, "bfloat16": torch.bfloat16,
             "int32": torch.int32, "int64": torch.int64, "bool": torch.bool}


@dataclasses.dataclass
class ExecConfig:
    compute_dtype: torch.dtype = torch.float32
    device: torch.device = torch.device("cpu")
    seed: int = 0
    bucket_bytes: int = 64 << 20
    fuse_add_layernorm: bool = True
    profiling: bool = False
    grad_clip: float = 0.0
    overlap_grad_sync: bool = True
    # single-device gradient buckets: run each bucket's optimizer update on a
    # side stream as soon as the backward pass finalises it (train_step only).
    # Off by default: measured neutral on BERT-large / GPT-3 medium
    # (profiles/ab_overlap_update_r2.txt) — the backward GEMMs occupy every CU,
    # so the memory-bound update cannot run beside them.
    overlap_update: bool = dataclasses.field(default_factory=lambda: os.environ.get("FF_OVERLAP_UPDATE", "0") != "0")
    bf16_weight_grads: bool = True
    # weight-gradient GEMMs (LINEAR / attention projections) on a second HIP
    # stream: the dW GEMM of a layer runs beside the input-gradient chain
    # (dX GEMM, activation / LayerNorm / attention backward) instead of in
    # series with it; joined before every gradient collective and at the end
    # of the backward pass.  Off by default: measured 2 % slower on BERT-large
    # and GPT-3 medium (profiles/ab_wgrad_stream_r2.txt) — concurrent GEMMs
    # contend for the CUs, and residual gradients read by a queued dW GEMM
    # cannot be accumulated in place (one extra add each).
    wgrad_stream: bool = dataclasses.field(default_factory=lambda: os.environ.get("FF_WGRAD_STREAM", "0") != "0")
    # debug mode (the AMD_SERIALIZE_KERNEL / HIP_LAUNCH_BLOCKING
    # analogue at operator granularity): synchronise the device after every
    # operator's forward and backward and re-raise a device fault naming the
    # operator that launched it.  Not usable inside a hipGraph capture.
    sync_debug: bool = dataclasses.field(default_factory=lambda: os.environ.get("FF_SYNC_DEBUG", "0") != "0")
    # --enable-inplace-optimizations: element-wise activations / scalar ops
    # whose input has no other reader overwrite that input instead of
    # allocating an output (_plan_inplace)
    inplace: bool = False
    # row-sparse SGD update of embedding tables (plain SGD only; exact)
    sparse_embedding_update: bool = True
    # "counter": every rank generates only its own piece from a counter-based
    # RNG keyed by the global element index (on-device on GPU);
    # "host": full weight from a torch.Generator on every rank, then sliced.
    init_mode: str = "counter"
    # ZeRO-style sharded optimizer: gradients are reduce-scattered, each rank
    # of a data-parallel group updates (and keeps Adam state for) one shard
    # of every bucket, and the updated weights are all-gathered.
    shard_optimizer: bool = False
    # gradient synchronisation of replicated weights: "nccl" = bucketed RCCL
    # all-reduce + update on every replica; "ps" = parameter server (the
    # reference's ParamSync::PS): reduce to the group leader, the leader
    # updates, the updated weights are broadcast.
    param_sync: str = "nccl"
    # reference-parity mode for SOFTMAX backward: the reference's softmax
    # backward is an identity copy (lib/kernels/src/cuda/ops/softmax_kernels.cu:
    # 63-72), correct only under a fused cross-entropy loss.  Off: the true
    # softmax Jacobian-vector product (docs/PARITY.md, "Deliberate divergences").
    softmax_identity_backward: bool = dataclasses.field(
        default_factory=lambda: os.environ.get("FF_SOFTMAX_IDENTITY_BWD", "0") != "0")


@dataclasses.dataclass
class ParamPiece:
    name: str
    node: int
    terminal: Value
    layout: Layout
    logical_shape: Tuple[int, ...]
    initializer: dict
    group: Tuple[int, ...]
    trainable: bool
    consumer_op: str = ""
    consumer_attrs: dict = dataclasses.field(default_factory=dict)
    # kernel regularizer of a LINEAR weight: ("l1" | "l2", lambda)
    regularizer: Optional[Tuple[str, float]] = None
    offset: int = 0
    numel: int = 0
    flat_id: int = 0
    final_step: int = -1          # forward index of first consumer
    n_consumers: int = 0
    grad_dtype: torch.dtype = torch.float32
    sparse: bool = False          # row-sparse SGD update (embedding tables)
    master: Optional[torch.Tensor] = None
    compute: Optional[torch.Tensor] = None
    grad: Optional[torch.Tensor] = None


_INPLACE_OPS = frozenset({"RELU", "SIGMOID", "TANH", "EXP", "SCALAR_MULTIPLY", "SCALAR_ADD", "SCALAR_SUB",
                          "SCALAR_TRUE_DIV"})


@dataclasses.dataclass
class Step:
    kind: str                      # "compute" | "comm"
    node: int
    op_type: str
    inputs: List[Value]
    outputs: List[Value]
    weights: List[Optional[ParamPiece]] = dataclasses.field(default_factory=list)
    src: Optional[Layout] = None
    dst: Optional[Layout] = None
    ctx: Optional[opbase.OpContext] = None
    active: bool = True            # this rank participates
    name: str = ""


def _stable_seed(*parts) -> int:
    h = hashlib.sha256(("/".join(str(p) for p in parts)).encode()).digest()
    return int.from_bytes(h[:8], "little") & ((1 << 62) - 1)


class Executor:
    def __init__(self, pcg, dist_ctx: DistContext, cfg: ExecConfig, views: Optional[Dict[int, Sequence[int]]] = None,
                 loss_type=None, metrics: Sequence[str] = (), optimizer=None, output: Optional[Value] = None,
                 label_dtype: Optional[torch.dtype] = None, valid_classes: Optional[int] = None):
        self.pcg = pcg
        self.dist = dist_ctx
        self.cfg = cfg
        # constant inputs: name -> host array (FFModel.create_constant*), and
        # their device pieces, built on the first forward (per executor)
        self.constants: Dict[str, object] = {}
        self._const_env: Optional[Dict] = None
        self.world = dist_ctx.world
        # PCG node -> placement (device tuple in task order, search/machine
        # mapping); nodes without one run on every rank
        self.views = {int(k): placement(v, self.world) for k, v in (views or {}).items()}
        self.rank = dist_ctx.rank
        self.redist = Redistributor(dist_ctx)
        self.metrics_names = list(metrics)
        self.optimizer_cfg = optimizer or SGDConfig()
        self.valid_classes = valid_classes
        self.step_num = 0
        self.tracer = Tracer(self.cfg.device, self.rank, enabled=self.cfg.profiling)
        self._ce_loss = loss_type in ("categorical_crossentropy", "sparse_categorical_crossentropy")
        self._build(output)
        self.loss = LossFunction(loss_type, self._global_rows(), valid_cols=valid_classes) if loss_type else None
        self.metrics_buf = torch.zeros(N_SLOTS, device=cfg.device, dtype=torch.float32)
        self.metrics_start = time.time()
        self._saved: Dict[int, Any] = {}
        # values whose latest forward value / gradient the API asked to keep
        # (Tensor.get_tensor / get_gradients on activations)
        self.retain: set = set()
        self.retained: Dict[Value, torch.Tensor] = {}
        self.retained_grads: Dict[Value, torch.Tensor] = {}
        self._env: Dict[Value, torch.Tensor] = {}
        self._works = []
        self._upd_stream = None
        self._ov_flats = set()
        self._overlap_lr = None

    # ------------------------------------------------------------------ build
    def _view(self, node: int) -> Tuple[int, ...]:
        v = self.views.get(node)
        return v if v is not None else tuple(range(self.world))

    def _layout(self, v: Value, node_for_view: Optional[int] = None) -> Layout:
        devs = self._view(v[0] if node_for_view is None else node_for_view)
        return layout_from_pshape(self.pcg.shape(C.ValueRef(v[0], v[1])), devices=devs)

    def _build(self, output: Optional[Value]):
        pcg = self.pcg
        order = list(pcg.topo_order())
        self.order = order
        optype = {n: pcg.layer_op(n).op_type for n in order}
        attrs = {n: dict(pcg.layer_op(n).items()) for n in order}
        names = {n: pcg.layer_name(n) for n in order}
        inputs_of = {n: [(v.node, v.idx) for v in pcg.layer_inputs(n)] for n in order}
        nout = {n: pcg.num_outputs(n) for n in order}
        uses: Dict[Value, List[Tuple[int, int]]] = {}
        for n in order:
            for slot, v in enumerate(inputs_of[n]):
                uses.setdefault(v, []).append((n, slot))
        self._uses = uses
        weight_path = {n: pcg.is_weight_path(n) for n in order}

        def follow_chain(v: Value) -> List[Value]:
            """Terminal values reached from v through parallel ops only."""
            terms = []
            for (c, _) in uses.get(v, []):
                if optype[c] in _PAR_OPS and nout[c] == 1:
                    terms.extend(follow_chain((c, 0)))
                else:
                    terms.append(v)
            return sorted(set(terms))

        # ---- parameters (folded weight paths)
        self.params: List[ParamPiece] = []
        self.param_of_value: Dict[Value, ParamPiece] = {}
        folded = set()
        for n in order:
            if optype[n] != "WEIGHT":
                continue
            terms = follow_chain((n, 0))
            if len(terms) != 1:
                terms = [(n, 0)]  # shared weight with several layouts: keep the source layout
            t = terms[0]
            # fold the chain nodes
            cur = t
            while cur[0] != n:
                folded.add(cur[0])
                cur = inputs_of[cur[0]][0]
            consumers = [c for (c, _) in uses.get(t, [])]
            cnode = consumers[0] if consumers else n
            lay = dataclasses.replace(self._layout(t, node_for_view=cnode), copy_outer=True)
            init = json.loads(attrs[n].get("initializer") or '{"type":"zero"}')
            cattrs = dict(attrs[cnode])
            if cnode != n:  # data-input feature sizes (physical weight layouts depend on them)
                cattrs["_in_features"] = [int(pcg.shape(C.ValueRef(v.node, v.idx)).shard_dims[-1].size)
                                          for v in pcg.layer_data_inputs(cnode)]
            piece = ParamPiece(name=names[n] or f"weight_{n}", node=n, terminal=t, layout=lay,
                               logical_shape=tuple(lay.sizes), initializer=init, group=(), trainable=bool(
                                   pcg.create_grad(C.ValueRef(n, 0))),
                               consumer_op=optype[cnode], consumer_attrs=cattrs)
            reg = str(cattrs.get("regularizer", "none"))
            if (optype[cnode] == "LINEAR" and reg in ("l1", "l2") and float(cattrs.get("regularizer_lambda", 0.0)) != 0
                    and [(w.node, w.idx) for w in pcg.layer_weights(cnode)][:1] == [tuple(t)]):
                piece.regularizer = (reg, float(cattrs["regularizer_lambda"]))
            self.params.append(piece)
            self.param_of_value[t] = piece
            folded.add(n)

        # ---- data inputs (folded repartition chains)
        self.inputs: Dict[str, Tuple[Value, Layout, torch.dtype]] = {}
        self.input_terminal: Dict[Value, str] = {}
        for n in order:
            if optype[n] != "INPUT":
                continue
            terms = follow_chain((n, 0))
            if len(terms) != 1:
                terms = [(n, 0)]
            t = terms[0]
            cur = t
            while cur[0] != n:
                folded.add(cur[0])
                cur = inputs_of[cur[0]][0]
            consumers = [c for (c, _) in uses.get(t, [])]
            lay = self._layout(t, node_for_view=consumers[0] if consumers else n)
            dt = _TORCH_DT.get(attrs[n].get("data_type", "float"), torch.float32)
            nm = names[n] or f"input_{n}"
            self.inputs[nm] = (t, lay, dt)
            self.input_terminal[t] = nm
            folded.add(n)

        # ---- steps
        self.steps: List[Step] = []
        self._sp_groups: set = set()
        self.value_layout: Dict[Value, Layout] = {}
        for nm, (t, lay, _) in self.inputs.items():
            self.value_layout[t] = lay
        for p in self.params:
            self.value_layout[p.terminal] = p.layout
        for n in order:
            if n in folded or weight_path.get(n) and n in folded:
                continue
            t = optype[n]
            if t in ("INPUT", "WEIGHT"):
                continue
            ins = inputs_of[n]
            if t in _PAR_OPS:
                src = self.value_layout[ins[0]]
                devs = self._view(n)
                dst = layout_from_pshape(pcg.shape(C.ValueRef(n, 0)), devices=devs)
                self.steps.append(Step("comm", n, t, [ins[0]], [(n, 0)], src=src, dst=dst, name=names[n]))
                self.value_layout[(n, 0)] = dst
                continue
            nw = C.num_weights(pcg.layer_op(n))
            data_ins, w_ins = ins[:len(ins) - nw], ins[len(ins) - nw:]
            devs = self._view(n)
            # implicit view changes for data inputs
            real_ins = []
            for v in data_ins:
                want = layout_from_pshape(pcg.shape(C.ValueRef(*v)), devices=devs)
                have = self.value_layout[v]
                if have != want:
                    nv = (-(len(self.steps) + 1) * 1000 - v[0], v[1])  # synthetic value id
                    self.steps.append(Step("comm", n, "VIEW_CHANGE", [v], [nv], src=have, dst=want,
                                           name=f"{names[n]}.view"))
                    self.value_layout[nv] = want
                    v = nv
                real_ins.append(v)
            wpieces = []
            for v in w_ins:
                if v not in self.param_of_value:
                    raise NotImplementedError(f"{names[n]}: weight input {v} is not a folded parameter")
                wpieces.append(self.param_of_value[v])
            outs = [(n, i) for i in range(nout[n])]
            for o in outs:
                self.value_layout[o] = layout_from_pshape(pcg.shape(C.ValueRef(*o)), devices=devs)
            olay = self.value_layout[outs[0]]
            coord = olay.coord(self.rank)
            in0 = pcg.shape(C.ValueRef(*data_ins[0])) if data_ins else None
            ctx = opbase.OpContext(
                op_type=t, attrs=attrs[n], name=names[n],
                sum_index=coord.a if coord else 0, sum_degree=olay.a_deg,
                copy_index=coord.b if coord else 0,
                input_copy_degree=int(in0.discard_copy_degree) if in0 is not None else 1,
                input_sum_degree=int(in0.sum_degree) if in0 is not None else 1,
                compute_dtype=self.cfg.compute_dtype, device=self.cfg.device,
                seed=_stable_seed(self.cfg.seed, names[n], self.rank // max(1, olay.reps) if coord else 0),
                output_shapes=[self.value_layout[o].piece_shape for o in outs])
            if t == "MULTIHEAD_ATTENTION" and len(olay.degrees) >= 2 and olay.degrees[1] > 1:
                # sequence-parallel attention: the ranks holding the other
                # sequence chunks of the same (batch, head) slice
                def _seq_ranks(c, lay=olay):
                    return [lay.rank_of(dataclasses.replace(c, shard=(c.shard[0], j) + tuple(c.shard[2:])))
                            for j in range(lay.degrees[1])]
                for r in range(self.world):
                    cr = olay.coord(r)
                    if cr is not None:
                        self._sp_groups.add(tuple(sorted(_seq_ranks(cr))))
                if coord is not None:
                    ctx.extra["seq_group"] = SeqGroup(self.dist, _seq_ranks(coord), coord.shard[1])
            if (t == "EXPERTS" and attrs[n].get("expert_parallel_mode") == "alltoall"
                    and int(attrs[n].get("expert_degree", 1)) > 1 and wpieces):
                # all-to-all expert parallelism: ranks holding the other expert
                # shards of the same weight replica exchange tokens
                wl = wpieces[0].layout

                def _ep_ranks(c, lay=wl):
                    return [lay.rank_of(dataclasses.replace(c, shard=(e,) + tuple(c.shard[1:])))
                            for e in range(lay.degrees[0])]
                for r in range(self.world):
                    cr = wl.coord(r)
                    if cr is not None:
                        self._sp_groups.add(tuple(sorted(_ep_ranks(cr))))
                cw = wl.coord(self.rank)
                if cw is not None:
                    ctx.extra["ep_group"] = ExpertGroup(self.dist, _ep_ranks(cw), cw.shard[0])
            if t in ("CONV2D", "POOL2D") and in0 is not None and len(in0.shard_dims) == 4 \
                    and int(in0.shard_dims[2].degree) > 1:
                # attribute (spatial) parallelism: the ranks holding the other
                # H bands of the same (batch, channel) slice exchange halos
                ilay = self.value_layout[real_ins[0]]
                a_n = attrs[n]

                def _band_ranks(c, lay=ilay):
                    return [lay.rank_of(dataclasses.replace(c, shard=tuple(c.shard[:2]) + (j,) + tuple(c.shard[3:])))
                            for j in range(lay.degrees[2])]
                for r in range(self.world):
                    cr = ilay.coord(r)
                    if cr is not None:
                        self._sp_groups.add(tuple(sorted(_band_ranks(cr))))
                ci = ilay.coord(self.rank)
                if ci is not None:
                    plan = HaloPlan(int(in0.shard_dims[2].size), int(a_n["kernel_h"]), int(a_n.get("stride_h", 1)),
                                    int(a_n.get("padding_h", 0)), int(in0.shard_dims[2].degree))
                    ctx.extra["halo"] = HaloGroup(self.dist, _band_ranks(ci), ci.shard[2], plan)
            if t in ("REDUCE_MEAN", "MEAN") and in0 is not None:
                axes = [int(a) % len(in0.shard_dims) for a in attrs[n].get("axes", [])]
                deg = math.prod(int(in0.shard_dims[a].degree) for a in axes)
                if deg > 1:
                    ctx.extra["mean_scale"] = 1.0 / deg
            self.steps.append(Step("compute", n, t, real_ins, outs, weights=wpieces, ctx=ctx,
                                   active=coord is not None, name=names[n]))

        # ---- output / loss value
        if output is None:
            last = [s for s in self.steps if s.kind == "compute"][-1]
            output = last.outputs[0]
        self.output_value = output
        self.loss_value = output
        self.softmax_fused_step: Optional[Step] = None
        prod_step = next((s for s in self.steps if output in s.outputs), None)
        if prod_step is not None and prod_step.op_type == "SOFTMAX":
            self.softmax_fused_step = prod_step
            # a trailing softmax fused with a cross-entropy loss: the loss
            # gradient (softmax - onehot) is taken at the logits.  Without such
            # a loss (none, MSE, identity) backward() starts at the softmax
            # OUTPUT and runs the softmax backward.
            if self._ce_loss:
                self.loss_value = prod_step.inputs[0]
        if self.cfg.fuse_add_layernorm:
            self._fuse_add_layernorm()
            self._fuse_conv_bn()
            if os.environ.get("FF_FUSE_DACT", "1") != "0":
                self._fuse_linear_dact()
        if self.cfg.softmax_identity_backward:
            for s in self.steps:
                if s.kind == "compute" and s.op_type == "SOFTMAX":
                    s.ctx.extra["identity_backward"] = True
        self._inplace_prod: Dict[int, int] = {}
        if self.cfg.inplace:
            self._plan_inplace()
        self._mark_requires_grad()
        self._assign_params_to_buffers()

    def _plan_inplace(self):
        """--enable-inplace-optimizations (reference FFModel::compile:
        Op::can_inplace_output / do_inplace_output, model.cc).  An element-wise
        activation (RELU / SIGMOID / TANH / EXP: backward from the output) or
        scalar op (backward needs no activation) whose input is read by
        nothing else writes its output over the input: no allocation, half
        the activation memory of the pair.  Static conditions here: one
        reader, not a fed input / constant / parameter, not the loss or
        output value, same layout in and out.  The storage check at run time
        (_inplace_ok) covers the dynamic ones: the producer kept the tensor
        for its own backward, or it is a view of a live tensor."""
        uses: Dict[Value, int] = {}
        for st in self.steps:
            for v in st.inputs:
                uses[v] = uses.get(v, 0) + 1
        fed = {v[0] for v in self.inputs.values()}
        terminals = {p.terminal for p in self.params if p.group}
        prod = {o: i for i, st in enumerate(self.steps) for o in st.outputs}
        for i, st in enumerate(self.steps):
            if st.kind != "compute" or st.op_type not in _INPLACE_OPS or len(st.inputs) != 1:
                continue
            v = st.inputs[0]
            j = prod.get(v)
            if (j is None or self.steps[j].kind != "compute" or uses.get(v, 0) != 1 or v in fed or v in terminals
                    or v in (self.loss_value, self.output_value)
                    or self.value_layout.get(v) != self.value_layout.get(st.outputs[0])):
                continue
            st.ctx.extra["inplace"] = True
            self._inplace_prod[i] = j

    def _inplace_ok(self, i: int, s: Step, x: Optional[torch.Tensor]) -> bool:
        if x is None or s.inputs[0] in self.retain or not x.is_floating_point():
            return False
        ptr = x.untyped_storage().data_ptr()
        j = self._inplace_prod[i]
        # what may still be read: the producer's saved tensors, its other
        # outputs and its inputs (x may be a view of one: FLAT / RESHAPE)
        prod = self.steps[j]
        held = [self._saved.get(j)] + [self._env_out.get(o) for o in prod.outputs if o != s.inputs[0]] + \
            [self._env_out.get(v) for v in prod.inputs]
        stack = list(held)
        while stack:
            t = stack.pop()
            if isinstance(t, torch.Tensor):
                if t.untyped_storage().data_ptr() == ptr:
                    return False
            elif isinstance(t, (tuple, list)):
                stack.extend(t)
            elif isinstance(t, dict):
                stack.extend(t.values())
        return True

    def _fuse_add_layernorm(self):
        by_out = {o: s for s in self.steps for o in s.outputs}
        keep = []
        # id(dropped EW_ADD step) -> the fused step that takes its place
        moves: Dict[int, Step] = {}
        uses: Dict[Value, List[Step]] = {}
        for s in self.steps:
            for v in s.inputs:
                uses.setdefault(v, []).append(s)
        for s in self.steps:
            if s.kind == "compute" and s.op_type == "LAYERNORM" and len(s.inputs) == 1:
                v = s.inputs[0]
                prod = by_out.get(v)
                if (prod is not None and prod.kind == "compute" and prod.op_type == "EW_ADD" and id(prod) not in moves
                        and v != self.loss_value
                        and self.value_layout[prod.inputs[0]] == self.value_layout[prod.inputs[1]]
                        and self.value_layout[v] == self.value_layout[prod.inputs[0]]
                        and tuple(self.value_layout[v].piece_shape)
                        == tuple(self.value_layout[prod.inputs[0]].piece_shape)):
                    s.op_type = "FUSED_ADD_LAYERNORM"
                    s.ctx.op_type = "FUSED_ADD_LAYERNORM"
                    s.inputs = list(prod.inputs)
                    if len(uses.get(v, [])) > 1:
                        # pre-LN residual stream: the sum also feeds the next
                        # residual add; the fused kernel writes it as a second output
                        s.outputs = [s.outputs[0], v]
                        s.ctx.extra["emit_sum"] = True
                    moves[id(prod)] = s
        # The fused step runs where the add ran: every other consumer of the
        # sum (a residual add, a redistribution on the residual edge) may sit
        # between the add and the norm in topological order, so it must see the
        # sum already written in forward, and in backward (reverse order) its
        # gradient contribution to the sum must land before the fused step's
        # backward reads it.  The norm's remaining inputs are weights, always
        # ready at the add's position.
        moved = {id(s) for s in moves.values()}
        for s in self.steps:
            if id(s) in moves:
                keep.append(moves[id(s)])
            elif id(s) not in moved:
                keep.append(s)
        self.steps = keep
        self._fuse_linear_bias_into_ln()

    def _fuse_linear_bias_into_ln(self):
        """LINEAR(+bias, no activation) -> FUSED_ADD_LAYERNORM: the input
        gradient of the add+norm IS the Linear's output gradient, so the norm
        backward accumulates its column sums straight into the Linear's bias
        gradient (layernorm_bwd dsum) and the Linear skips its own column-sum
        pass over the same tensor.  Taken at run time only on the HIP path."""
        by_out = {o: s for s in self.steps for o in s.outputs}
        uses: Dict[Value, List[Step]] = {}
        for s in self.steps:
            for v in s.inputs:
                uses.setdefault(v, []).append(s)
        for s in self.steps:
            if s.kind != "compute" or s.op_type != "FUSED_ADD_LAYERNORM":
                continue
            for v in s.inputs:
                prod = by_out.get(v)
                if prod is None or prod.kind != "compute" or prod.ctx.sum_degree != 1:
                    continue
                # (producer, index of its output-bias weight)
                if (prod.op_type == "LINEAR" and prod.ctx.a("activation", "none") == "none"
                        and len(prod.weights) > 1):
                    widx = 1
                elif prod.op_type == "MULTIHEAD_ATTENTION" and len(prod.weights) > 2:
                    widx = 2
                else:
                    continue
                if (len(uses.get(v, [])) == 1 and v != self.loss_value
                        and self.value_layout[v] == self.value_layout[s.inputs[0]]):
                    s.ctx.extra["dbias_src"] = (prod, widx)
                    break

    def _fuse_conv_bn(self):
        """CNN fusions (the reference's FusedOp grouping, lib/runtime/src/ops/fused.cc,
        done as real kernel fusion):
        * CONV2D whose only consumer is a BATCHNORM on the same layout emits the
          per-channel statistics from its epilogue (``emit_bn_stats``);
        * BATCHNORM(relu=False) -> EW_ADD -> RELU (the residual block tail) becomes
          one BATCHNORM step computing relu(bn(x) + residual), placed where the add
          was (both operands are available there)."""
        by_out = {o: s for s in self.steps for o in s.outputs}
        uses: Dict[Value, List[Step]] = {}
        for s in self.steps:
            for v in s.inputs:
                uses.setdefault(v, []).append(s)
        lay = self.value_layout
        for s in self.steps:
            if s.kind != "compute" or s.op_type != "BATCHNORM" or len(s.inputs) != 1:
                continue
            prod = by_out.get(s.inputs[0])
            if (prod is not None and prod.kind == "compute" and prod.op_type == "CONV2D"
                    and len(uses.get(s.inputs[0], [])) == 1 and s.inputs[0] != self.loss_value
                    and prod.ctx.sum_degree == 1 and s.ctx.sum_degree == 1):
                prod.ctx.extra["emit_bn_stats"] = True
        drop = set()
        moves = {}
        for s in self.steps:
            if (s.kind != "compute" or s.op_type != "BATCHNORM" or len(s.inputs) != 1 or s.ctx.a("relu", False)
                    or len(s.outputs) != 1):
                continue
            v = s.outputs[0]
            u = uses.get(v, [])
            if len(u) != 1 or u[0].kind != "compute" or u[0].op_type != "EW_ADD" or v == self.loss_value:
                continue
            add = u[0]
            if id(add) in moves:  # both add operands are BN outputs: fuse one of them
                continue
            a = add.outputs[0]
            ua = uses.get(a, [])
            if len(ua) != 1 or ua[0].kind != "compute" or ua[0].op_type != "RELU" or a == self.loss_value:
                continue
            relu = ua[0]
            other = add.inputs[1] if add.inputs[0] == v else add.inputs[0]
            if other == v or not (lay[other] == lay[v] == lay[a] == lay[relu.outputs[0]]):
                continue
            if tuple(lay[other].piece_shape) != tuple(lay[v].piece_shape):
                continue
            s.inputs = [s.inputs[0], other]
            s.outputs = list(relu.outputs)
            s.ctx.extra["residual_relu"] = True
            drop.add(id(relu))
            moves[id(add)] = s
        keep = []
        moved = {id(s) for s in moves.values()}
        for s in self.steps:
            if id(s) in moves:
                keep.append(moves[id(s)])
            elif id(s) in drop or id(s) in moved:
                continue
            else:
                keep.append(s)
        self.steps = keep
        # * BATCHNORM (no residual) whose only consumer is a CONV2D on the same
        #   layout: that conv's dgrad epilogue reduces the BN's backward sums
        #   (``emit_bn_bwd_sums``), so the BN backward skips its reduction pass
        uses = {}
        for s in self.steps:
            for v in s.inputs:
                uses.setdefault(v, []).append(s)
        for s in self.steps:
            if (s.kind != "compute" or s.op_type != "BATCHNORM" or len(s.inputs) != 1 or len(s.outputs) != 1
                    or s.ctx.extra.get("residual_relu") or s.ctx.sum_degree != 1):
                continue
            v = s.outputs[0]
            u = uses.get(v, [])
            if (len(u) == 1 and u[0].kind == "compute" and u[0].op_type == "CONV2D" and v != self.loss_value
                    and u[0].ctx.sum_degree == 1 and u[0].inputs[0] == v and lay[v] == lay[s.inputs[0]]):
                u[0].ctx.extra["emit_bn_bwd_sums"] = True
                s.ctx.extra["bn_sums_from_conv"] = True

    def _fuse_linear_dact(self):
        """LINEAR(act) -> LINEAR: the second layer's input-gradient GEMM
        applies the first layer's activation derivative and accumulates its
        bias gradient in its epilogue (gemmp act_bwd + dbias), so the first
        layer's backward starts from the pre-activation gradient and skips its
        own activation-backward / bias-gradient pass (colsum_act: a read of the
        gradient and the pre-activation plus a write).  Decided per step at
        run time (GPU bf16 operands the kernel supports); otherwise both
        layers run unfused."""
        by_out = {o: s for s in self.steps for o in s.outputs}
        uses: Dict[Value, List[Step]] = {}
        for s in self.steps:
            for v in s.inputs:
                uses.setdefault(v, []).append(s)
        for s in self.steps:
            if s.kind != "compute" or s.op_type != "LINEAR" or not s.inputs:
                continue
            v = s.inputs[0]
            prod = by_out.get(v)
            if (prod is None or prod.kind != "compute" or prod.op_type != "LINEAR"
                    or prod.ctx.a("activation", "none") not in ("relu", "sigmoid", "tanh", "gelu")
                    or len(uses.get(v, [])) != 1 or v == self.loss_value or prod.ctx.sum_degree != 1
                    or self.value_layout[v] != self.value_layout[prod.outputs[0]]):
                continue
            s.ctx.extra["dact_src"] = prod

    def _mark_requires_grad(self):
        rg: Dict[Value, bool] = {}
        for p in self.params:
            rg[p.terminal] = p.trainable
        for nm, (t, _, dt) in self.inputs.items():
            rg[t] = False
        for idx, s in enumerate(self.steps):
            need = any(rg.get(v, False) for v in s.inputs) or any(p.trainable for p in s.weights)
            for o in s.outputs:
                rg[o] = need
            for p in s.weights:
                p.n_consumers += 1
                if p.final_step < 0:
                    p.final_step = idx
        self.requires_grad = rg

    def _assign_params_to_buffers(self):
        dev = self.cfg.device
        # gradient-sync group: same shard piece, same partial index, same
        # implicit replica; all discard-copy indices (their grads add up).
        for p in self.params:
            lay = p.layout
            c = lay.coord(self.rank)
            if c is None:
                p.group = ()
                continue
            grp = []
            for b in range(lay.b_deg):
                grp.append(lay.rank_of(dataclasses.replace(c, b=b)))
            p.group = tuple(sorted(grp))
        held = [p for p in self.params if p.group]
        # flat order = the order in which backward finalises gradients
        held.sort(key=lambda p: (-p.final_step, p.node))
        cd = self.cfg.compute_dtype
        # GEMM weights (written once by their dW GEMM) keep bf16 gradients when
        # computing in bf16: the bf16-output GEMM runs ~1.6x faster than the
        # fp32-output one on hipBLASLt and the DP all-reduce moves half the
        # bytes; atomically-accumulated gradients (biases, norms, embeddings)
        # stay fp32.  Master weights and optimizer state are always fp32.
        for p in held:
            p.grad_dtype = torch.float32
            if (self.cfg.bf16_weight_grads and cd == torch.bfloat16 and p.n_consumers == 1
                    and p.consumer_op in ("LINEAR", "MULTIHEAD_ATTENTION") and self._weight_index(p) == 0):
                p.grad_dtype = torch.bfloat16
        # Embedding tables under plain SGD (the reference's DLRM optimizer:
        # no momentum / weight decay) that no other rank holds: a row the batch
        # did not touch has a zero gradient and stays unchanged, so the update
        # (and the gradient reset) visits only the touched rows instead of
        # sweeping gigabytes of table every step.  Exact, not an approximation.
        oc = self.optimizer_cfg
        plain_sgd = isinstance(oc, SGDConfig) and not oc.momentum and not oc.weight_decay
        for p in held:
            p.sparse = bool(self.cfg.sparse_embedding_update and plain_sgd and p.consumer_op == "EMBEDDING"
                            and p.n_consumers == 1 and len(p.group) <= 1 and p.layout.degrees[0] == 1
                            and self._weight_index(p) == 0 and len(p.layout.piece_shape) == 2)
        groups: Dict[Tuple, List[ParamPiece]] = {}
        for p in held:
            groups.setdefault((p.group, str(p.grad_dtype), p.sparse), []).append(p)
        self.flats = []
        for fid, ((g, gdt, sparse), plist) in enumerate(sorted(groups.items(), key=lambda kv: kv[0])):
            multi = len(g) > 1 or (self.dist.force_collectives and len(g) == 1)
            zero = self.cfg.shard_optimizer and multi
            esize = torch.tensor([], dtype=plist[0].grad_dtype).element_size()
            # buckets: contiguous param ranges, finalised in backward order
            buckets, cur, cur_bytes = [], [], 0
            for p in plist:
                p.numel = int(math.prod(p.layout.piece_shape))
                cur.append(p)
                cur_bytes += p.numel * esize
                if cur_bytes >= self.cfg.bucket_bytes:
                    buckets.append(cur)
                    cur, cur_bytes = [], 0
            if cur:
                buckets.append(cur)
            # sharded optimizer: every bucket splits evenly over the group
            unit = 64 * (len(g) if zero else 1)
            off = 0
            binfo = []
            for b in buckets:
                lo = off
                for p in b:
                    p.offset = off
                    p.flat_id = fid
                    off += (p.numel + 63) // 64 * 64
                off = (off + unit - 1) // unit * unit
                info = {"params": b, "lo": lo, "hi": off, "pending": 0}
                if zero:
                    S = (off - lo) // len(g)
                    gi = g.index(self.rank)
                    info["shard"] = (lo + gi * S, lo + (gi + 1) * S)
                binfo.append(info)
            master = torch.zeros(off, dtype=torch.float32, device=dev)
            grad = torch.zeros(off, dtype=plist[0].grad_dtype, device=dev)
            compute = torch.zeros(off, dtype=cd, device=dev) if cd != torch.float32 else None
            for p in plist:
                shp = p.layout.piece_shape
                p.master = master[p.offset:p.offset + p.numel].view(shp)
                p.grad = grad[p.offset:p.offset + p.numel].view(shp)
                p.compute = (compute[p.offset:p.offset + p.numel].view(shp) if compute is not None else p.master)
            if zero:
                opt = ShardedOptimizer(self.optimizer_cfg, master, grad, compute, [b["shard"] for b in binfo])
            else:
                opt = FlatOptimizer(self.optimizer_cfg, master, grad, compute)
            self.flats.append({"group": g, "params": plist, "master": master, "grad": grad, "compute": compute,
                               "buckets": binfo, "opt": opt, "zero": zero, "sparse": sparse,
                               "ps": (not zero) and self.cfg.param_sync == "ps" and multi})
        for p in self.params:
            if p.sparse and 0 <= p.final_step < len(self.steps):
                self.steps[p.final_step].ctx.extra["track_rows"] = True
        self._param_bucket = {}
        for f in self.flats:
            for bi, b in enumerate(f["buckets"]):
                for p in b["params"]:
                    self._param_bucket[id(p)] = (f, b)
        # create every sub-communicator collectively, in a deterministic order
        if self.dist.distributed:
            all_groups = set()
            for p in self.params:
                lay = p.layout
                for r in range(self.world):
                    c = lay.coord(r)
                    if c is None:
                        continue
                    all_groups.add(tuple(sorted(lay.rank_of(dataclasses.replace(c, b=b)) for b in range(lay.b_deg))))
            all_groups |= self._sp_groups
            for g in sorted(all_groups):
                if self.dist.syncs(g):
                    self.dist.group(g)
            for s in self.steps:
                if s.kind == "comm":
                    self.redist.plan(s.src, s.dst)
                    self.redist.plan(s.dst.dual(), s.src.dual())

    # ------------------------------------------------------------ weights
    def init_parameters(self):
        """Deterministic initialisation: every rank generates the full logical
        weight from a seed derived from the weight name, then keeps its piece
        (identical across replicas without any broadcast)."""
        if self.cfg.init_mode == "counter":
            self._init_counter()
            return
        for p in self.params:
            if not p.group:
                continue
            gen = torch.Generator().manual_seed(_stable_seed(self.cfg.seed, p.name))
            impl = None
            try:
                impl = opbase.get_impl(p.consumer_op)
            except NotImplementedError:
                pass
            full = None
            if impl is not None:
                ctx = opbase.OpContext(op_type=p.consumer_op, attrs=p.consumer_attrs, name=p.name)
                widx = self._weight_index(p)
                full = impl.init_weight(ctx, widx, p.logical_shape, p.initializer, gen)
            if full is None:
                full = make_initializer_tensor(p.initializer, p.logical_shape, gen)
            self._set_piece(p, full)
        for f in self.flats:
            if f["compute"] is not None:
                f["compute"].copy_(f["master"])

    def _init_counter(self):
        from .initializers import counter_init_piece, counter_spec
        for p in self.params:
            if not p.group:
                continue
            impl = self._impl_of(p)
            spec = None
            if impl is not None:
                ctx = opbase.OpContext(op_type=p.consumer_op, attrs=p.consumer_attrs, name=p.name)
                spec = impl.init_spec(ctx, self._weight_index(p), p.logical_shape, p.initializer or {})
            if spec is None:
                spec = counter_spec(p.initializer, p.logical_shape)
            box = p.layout.box(p.layout.coord(self.rank).shard)
            piece = counter_init_piece(spec, p.logical_shape, box, _stable_seed(self.cfg.seed, p.name),
                                       p.master.device)
            p.master.copy_(self._to_physical(p, piece))
            if p.compute is not p.master:
                p.compute.copy_(p.master)
        for f in self.flats:
            if f["compute"] is not None:
                f["compute"].copy_(f["master"])

    def _weight_index(self, p: ParamPiece) -> int:
        for s in self.steps:
            for i, w in enumerate(s.weights):
                if w is p:
                    return i
        return 0

    def _impl_of(self, p: ParamPiece):
        try:
            return opbase.get_impl(p.consumer_op)
        except NotImplementedError:
            return None

    def _to_physical(self, p: ParamPiece, piece: torch.Tensor) -> torch.Tensor:
        impl = self._impl_of(p)
        if impl is None:
            return piece
        return impl.to_physical(p.consumer_attrs, self._weight_index(p), piece).reshape(piece.shape)

    def _to_logical(self, p: ParamPiece, piece: torch.Tensor) -> torch.Tensor:
        impl = self._impl_of(p)
        if impl is None:
            return piece
        return impl.to_logical(p.consumer_attrs, self._weight_index(p), piece).reshape(piece.shape)

    def _set_piece(self, p: ParamPiece, full: torch.Tensor):
        c = p.layout.coord(self.rank)
        box = p.layout.box(c.shard)
        sl = tuple(slice(lo, hi) for lo, hi in box)
        p.master.copy_(self._to_physical(p, full.reshape(p.logical_shape)[sl].to(torch.float32)))
        if p.compute is not p.master:
            p.compute.copy_(p.master)

    def get_parameter(self, name: str) -> torch.Tensor:
        """Full logical weight (gathered across ranks)."""
        self._gather_masters()
        p = next(pp for pp in self.params if pp.name == name)
        full = torch.zeros(p.logical_shape, dtype=torch.float32, device=self.cfg.device)
        c = p.layout.coord(self.rank)
        owner = c is not None and c.b == 0 and c.rep == 0 and c.a == 0
        if owner:
            box = p.layout.box(c.shard)
            full[tuple(slice(lo, hi) for lo, hi in box)] = self._to_logical(p, p.master)
        if self.dist.distributed:
            import torch.distributed as dist
            dist.all_reduce(full)
        return full

    def get_parameter_grad(self, name: str) -> torch.Tensor:
        """Full logical gradient of a weight after backward() (summed over the
        data-parallel replicas once the gradient sync ran), fp32."""
        p = next(pp for pp in self.params if pp.name == name)
        full = torch.zeros(p.logical_shape, dtype=torch.float32, device=self.cfg.device)
        if p.grad is None or not p.group:
            return full
        if self.flats[p.flat_id]["zero"]:
            raise RuntimeError("get_parameter_grad: gradients are reduce-scattered under the sharded optimizer")
        c = p.layout.coord(self.rank)
        if c is not None and c.b == 0 and c.rep == 0 and c.a == 0:
            box = p.layout.box(c.shard)
            full[tuple(slice(lo, hi) for lo, hi in box)] = self._to_logical(p, p.grad.float())
        if self.dist.distributed:
            import torch.distributed as dist
            dist.all_reduce(full)
        return full

    def _opt_state_keys(self) -> List[str]:
        if isinstance(self.optimizer_cfg, AdamConfig):
            return ["m", "v"]
        return ["mom"] if getattr(self.optimizer_cfg, "momentum", 0.0) else []

    def get_optimizer_state(self, name: str) -> Dict[str, torch.Tensor]:
        """Full logical optimizer state of one weight ({"m", "v"} for Adam,
        {"mom"} for momentum SGD), gathered across ranks; {} when the
        optimizer is sharded (ZeRO) — its state stays rank-local."""
        if self.cfg.shard_optimizer:
            return {}
        p = next(pp for pp in self.params if pp.name == name)
        out = {}
        for key in self._opt_state_keys():
            full = torch.zeros(p.logical_shape, dtype=torch.float32, device=self.cfg.device)
            c = p.layout.coord(self.rank)
            if c is not None and c.b == 0 and c.rep == 0 and c.a == 0 and p.group:
                flat = getattr(self.flats[p.flat_id]["opt"], key)
                piece = flat[p.offset:p.offset + p.numel].view(p.layout.piece_shape)
                box = p.layout.box(c.shard)
                full[tuple(slice(lo, hi) for lo, hi in box)] = self._to_logical(p, piece)
            if self.dist.distributed:
                import torch.distributed as dist
                dist.all_reduce(full)
            out[key] = full
        return out

    def set_optimizer_state(self, name: str, state: Dict[str, torch.Tensor]):
        p = next(pp for pp in self.params if pp.name == name)
        if not p.group or self.cfg.shard_optimizer:
            return
        c = p.layout.coord(self.rank)
        box = p.layout.box(c.shard)
        for key, full in state.items():
            flat = getattr(self.flats[p.flat_id]["opt"], key, None)
            if flat is None:
                continue
            piece = full.to(self.cfg.device).float().reshape(p.logical_shape)[tuple(slice(lo, hi) for lo, hi in box)]
            flat[p.offset:p.offset + p.numel].view(p.layout.piece_shape).copy_(self._to_physical(p, piece))

    def set_parameter(self, name: str, value: torch.Tensor):
        p = next(pp for pp in self.params if pp.name == name)
        if p.group:
            self._set_piece(p, value.to(self.cfg.device).float())

    def parameter_names(self) -> List[str]:
        return [p.name for p in self.params]

    # --------------------------------------------------------------- inputs
    def local_input_shape(self, name: str) -> Tuple[int, ...]:
        return self.inputs[name][1].piece_shape

    def _local_piece(self, name: str, x: torch.Tensor) -> Optional[torch.Tensor]:
        t, lay, dt = self.inputs[name]
        c = lay.coord(self.rank)
        if c is None:
            return None
        if tuple(x.shape) == tuple(lay.piece_shape) and tuple(lay.sizes) != tuple(lay.piece_shape):
            piece = x  # already the local piece
        elif tuple(x.shape) == tuple(lay.sizes):
            piece = x[tuple(slice(lo, hi) for lo, hi in lay.box(c.shard))]
        else:
            raise ValueError(f"input {name}: shape {tuple(x.shape)} is neither global {lay.sizes} "
                             f"nor local {lay.piece_shape}")
        piece = piece.to(self.cfg.device, non_blocking=True)
        if piece.is_floating_point():
            piece = piece.to(self.cfg.compute_dtype)
        return piece.contiguous()

    def _global_rows(self) -> int:
        lay = self.value_layout[self.loss_value]
        return int(math.prod(lay.sizes[:-1])) if len(lay.sizes) > 1 else int(lay.sizes[0])

    def label_layout(self) -> Layout:
        lay = self.value_layout[self.loss_value]
        return lay

    def local_labels(self, y: torch.Tensor) -> Optional[torch.Tensor]:
        lay = self._loss_layout()
        c = lay.coord(self.rank)
        if c is None:
            return None
        box = lay.box(c.shard)
        sparse = self.loss is not None and self.loss.loss_type == "sparse_categorical_crossentropy"
        gshape = tuple(lay.sizes[:-1]) if sparse else tuple(lay.sizes)
        lshape = tuple(lay.piece_shape[:-1]) if sparse else tuple(lay.piece_shape)
        nb = box[:-1] if sparse else box
        if y.numel() == math.prod(gshape):
            y = y.reshape(gshape)[tuple(slice(lo, hi) for lo, hi in nb)]
        elif y.numel() == math.prod(lshape):
            y = y.reshape(lshape)
        else:
            raise ValueError(f"labels of shape {tuple(y.shape)} match neither global {gshape} nor local {lshape}")
        return y.to(self.cfg.device, non_blocking=True).contiguous()

    def _loss_layout(self) -> Layout:
        lay = self.value_layout[self.loss_value]
        if lay.degrees[-1] != 1 or lay.a_deg != 1:
            degs = tuple(lay.degrees[:-1]) + (1,)
            lay = dataclasses.replace(lay, degrees=degs, a_deg=1)
        return lay

    # -------------------------------------------------------------- execution
    def forward(self, feeds: Dict[str, torch.Tensor], training: bool = True, keep_outputs: bool = False,
                save: Optional[bool] = None, free_env: bool = False):
        """Forward pass.  ``training`` selects training-mode op semantics
        (dropout masks, batch statistics); ``save`` (default: ``training``)
        keeps each step's saved tensors for a following backward();
        ``free_env`` (the training step's own forward) lets each value go
        after its last forward reader instead of holding every activation
        to the end of the step."""
        if save is None:
            save = training
        env: Dict[Value, torch.Tensor] = {}
        for name, x in feeds.items():
            if name not in self.inputs:
                raise KeyError(f"unknown input {name}; inputs are {list(self.inputs)}")
            piece = self._local_piece(name, x)
            if piece is not None:
                env[self.inputs[name][0]] = piece
        if self.constants:
            # constant inputs (FFModel.create_constant*): placed on the device
            # once, never fed; the same tensors every step (graph-capture safe)
            if self._const_env is None:
                self._const_env = {}
                for name, x in self.constants.items():
                    piece = self._local_piece(name, torch.as_tensor(x))
                    if piece is not None:
                        self._const_env[self.inputs[name][0]] = piece
            for v, piece in self._const_env.items():
                env.setdefault(v, piece)
        for p in self.params:
            if p.group:
                env[p.terminal] = p.compute
        self._saved = {}
        prof = self.cfg.profiling
        # with a backward to follow, a value leaves the environment after its
        # last forward consumer: from then on only the saved tensors that the
        # backward reads keep it, so the backward frees activations as it goes
        # (kept to the end of the step, ResNet-50's peak was every activation
        # plus the largest gradients: 13.7 vs 12.0 GB planned)
        drop = self._env_drop_plan() if free_env and save and os.environ.get("FF_FREE_ENV", "1") != "0" else None
        for i, s in enumerate(self.steps):
            if drop is not None and i:
                for v in drop[i - 1]:
                    if v not in self.retain:
                        env.pop(v, None)
            if training and s is self.softmax_fused_step and self.loss is not None and self.loss.fuses_softmax:
                continue
            if s.kind == "comm":
                x = env.get(s.inputs[0])
                t0 = self.tracer.begin(f"{s.name}:fwd", "comm", self.step_num) if prof else None
                env[s.outputs[0]] = self.redist(x, s.src, s.dst, self._dtype_of(s.inputs[0], x), self.cfg.device)
                self.tracer.end(t0)
                continue
            if not s.active:
                continue
            s.ctx.training = training
            s.ctx.step = self.step_num
            ins = [env[v] for v in s.inputs]
            ws = [p.compute for p in s.weights]
            if i in self._inplace_prod:
                self._env_out = env
                s.ctx.extra["inplace_ok"] = self._inplace_ok(i, s, ins[0])
            impl = opbase.get_impl(s.op_type)
            t0 = self.tracer.begin(f"{s.name}:fwd", "compute", self.step_num) if prof else None
            outs, saved = impl.forward(s.ctx, ins, ws)
            self.tracer.end(t0)
            if self.cfg.sync_debug:
                self._debug_sync(s, "forward")
            for o, t in zip(s.outputs, outs):
                env[o] = t
                if o in self.retain:
                    self.retained[o] = t
            if save:
                self._saved[i] = saved
        if drop is not None and self.steps:
            for v in drop[-1]:
                if v not in self.retain:
                    env.pop(v, None)
        self._env = env
        return env.get(self.output_value) if keep_outputs or not training else env.get(self.loss_value)

    def _env_drop_plan(self) -> List[List[Value]]:
        """Per step, the values whose last forward reader it is (a value no
        step reads goes right after its producer).  Kept to the end: the loss
        and output values, parameter terminals, and the inputs / outputs of an
        in-place step's producer (its in-place check looks them up)."""
        key = (len(self.steps), id(self.softmax_fused_step), len(self._inplace_prod))
        cached = getattr(self, "_env_drop", None)
        if cached is not None and cached[0] == key:
            return cached[1]
        last: Dict[Value, int] = {}
        for i, st in enumerate(self.steps):
            for o in st.outputs:
                last.setdefault(o, i)
            for v in st.inputs:
                last[v] = max(i, last.get(v, i))
        keep = {self.loss_value, self.output_value}
        keep.update(p.terminal for p in self.params if p.group)
        for j in set(self._inplace_prod.values()):
            keep.update(self.steps[j].inputs)
            keep.update(self.steps[j].outputs)
        plan: List[List[Value]] = [[] for _ in self.steps]
        for v, i in last.items():
            if v not in keep:
                plan[i].append(v)
        self._env_drop = (key, plan)
        return plan

    def _dtype_of(self, v: Value, x: Optional[torch.Tensor]) -> torch.dtype:
        if x is not None:
            return x.dtype
        ps = self.pcg.shape(C.ValueRef(*v)) if v[0] >= 0 else None
        if ps is not None and C.datatype_to_string(ps.dtype) in ("int32", "int64"):
            return _TORCH_DT[C.datatype_to_string(ps.dtype)]
        return self.cfg.compute_dtype

    def compute_loss(self, labels: Optional[torch.Tensor]) -> Optional[torch.Tensor]:
        logits = self._env.get(self.loss_value)
        lay = self.value_layout[self.loss_value]
        want = self._loss_layout()
        if want != lay:
            logits = self.redist(logits, lay, want, logits.dtype if logits is not None else self.cfg.compute_dtype,
                                 self.cfg.device)
        c = want.coord(self.rank)
        if c is None or logits is None:
            return None
        y = self.local_labels(labels)
        if c.rep == 0 and c.b == 0:
            mbuf = self.metrics_buf
        else:
            mbuf = torch.zeros(N_SLOTS, device=self.cfg.device)  # replicas do not double count
        g = self.loss(logits, y, mbuf)
        if want.b_deg > 1:
            g = g / want.b_deg
        if want != lay:
            g = self.redist(g, want.dual(), lay.dual(), g.dtype, self.cfg.device)
        return g

    def backward(self, dlogits: Optional[torch.Tensor], zero_grads: bool = True, accumulate: bool = False,
                 sync: bool = True):
        """Reverse pass.  Micro-batching (``train_step_pipelined``) calls it
        once per micro-batch: ``zero_grads`` only for the first, ``accumulate``
        (every dW adds, beta = 1) for the rest, ``sync`` (bucketed gradient
        all-reduces overlapped with this pass) only for the last."""
        grads: Dict[Value, torch.Tensor] = {}
        if dlogits is not None:
            grads[self.loss_value] = dlogits
        self._sync_row_tracking()
        ov = getattr(self, "_overlap_lr", None)
        self._ov_flats = set()
        if ov is not None and sync and not accumulate:
            for f in self._overlap_flats():
                f["opt"].begin_step()
                self._ov_flats.add(id(f))
        for f in self.flats:
            if zero_grads:
                self._zero_flat(f)
            for b in f["buckets"]:
                b["pending"] = sum(1 for p in b["params"] if p.trainable)
        self._works = []
        prof = self.cfg.profiling
        wg_on = self._wg_enabled()
        n = len(self.steps)
        if getattr(self, "_step_index", None) is None or len(self._step_index) != n:
            self._step_index = {id(st): k for k, st in enumerate(self.steps)}
            self._flag_ctxs = [st.ctx.extra["dact_src"].ctx for st in self.steps
                               if st.ctx is not None and "dact_src" in st.ctx.extra]
            self._flag_ctxs += [st.ctx.extra["dbias_src"][0].ctx for st in self.steps
                                if st.ctx is not None and "dbias_src" in st.ctx.extra]
        for c in self._flag_ctxs:   # run-time hand-off flags never outlive a backward pass
            c.extra.pop("grad_is_preact", None)
            c.extra.pop("db_done", None)
        for i in range(n - 1, -1, -1):
            s = self.steps[i]
            if s is self.softmax_fused_step and self.loss is not None and self.loss.fuses_softmax:
                continue
            if s.kind == "comm":
                g = grads.pop(s.outputs[0], None)
                if not self.requires_grad.get(s.inputs[0], False):
                    continue
                if g is None and s.dst.coord(self.rank) is not None:
                    g = torch.zeros(s.dst.piece_shape, dtype=self.cfg.compute_dtype, device=self.cfg.device)
                t0 = self.tracer.begin(f"{s.name}:bwd", "comm", self.step_num) if prof else None
                gi = self.redist(g, s.dst.dual(), s.src.dual(), g.dtype if g is not None else self.cfg.compute_dtype,
                                 self.cfg.device)
                self.tracer.end(t0)
                self._acc(grads, s.inputs[0], gi)
                continue
            saved = self._saved.pop(i, None)
            if s.active:
                gouts = [grads.pop(o, None) for o in s.outputs]
                for o, g in zip(s.outputs, gouts):
                    if g is not None and o in self.retain:
                        self.retained_grads[o] = g.detach().clone()
                need = [self.requires_grad.get(v, False) for v in s.inputs]
                if any(g is not None for g in gouts) and (any(need) or any(p.trainable for p in s.weights)):
                    gouts = [g if g is not None else None for g in gouts]
                    if gouts[0] is None:
                        gouts[0] = torch.zeros(s.ctx.output_shapes[0], dtype=self.cfg.compute_dtype,
                                               device=self.cfg.device)
                    wgs = [p.grad if p.trainable else None for p in s.weights]
                    # sole-consumer weights may be overwritten (beta = 0) by their dW GEMM;
                    # shared ones accumulate.  Existing input grads are offered for in-place
                    # accumulation (ops return the same tensor when they used it).
                    s.ctx.extra["wgrad_beta"] = [0.0 if (p.n_consumers == 1 and not accumulate) else 1.0
                                                 for p in s.weights]
                    # an input gradient still read by a pending side-stream dW GEMM
                    # (or aliasing this op's output gradient, which its own dW GEMM
                    # reads) is not offered for in-place accumulation: the op
                    # returns a fresh tensor and _acc adds
                    side = wg_on and s.op_type in ("LINEAR", "MULTIHEAD_ATTENTION")
                    busy = {g.untyped_storage().data_ptr() for g in gouts if g is not None} if side else set()
                    s.ctx.extra["grad_acc"] = [
                        a if (nd and a is not None and not self._wg_reads(a)
                              and a.untyped_storage().data_ptr() not in busy) else None
                        for a, nd in ((grads.get(v), nd) for v, nd in zip(s.inputs, need))]
                    if side:
                        s.ctx.extra["wgrad_stream"] = self._wg
                    else:
                        s.ctx.extra.pop("wgrad_stream", None)
                    bsrc = s.ctx.extra.get("dbias_src")
                    s.ctx.extra.pop("dsum_target", None)
                    if bsrc is not None:
                        bw = bsrc[0].weights[bsrc[1]]
                        if bw is not None and bw.trainable:
                            s.ctx.extra["dsum_target"] = (bw.grad, bsrc[0].ctx)
                    src = s.ctx.extra.get("dact_src")
                    s.ctx.extra.pop("dact", None)
                    if src is not None and need[0] and s.inputs[0] not in self.retain:
                        # (activation, pre-activation, producer's fp32 bias grad, producer ctx)
                        ps = self._saved.get(self._step_index[id(src)])
                        if ps is not None and ps[1] is not None:
                            bw = src.weights[1] if len(src.weights) > 1 else None
                            db = bw.grad if (bw is not None and bw.trainable) else None
                            s.ctx.extra["dact"] = (src.ctx.a("activation"), ps[1], db, src.ctx)
                    impl = opbase.get_impl(s.op_type)
                    t0 = self.tracer.begin(f"{s.name}:bwd", "compute", self.step_num) if prof else None
                    gins = impl.backward(s.ctx, saved, gouts, wgs, need)
                    # hand-offs of this backward only: left in ctx.extra they would
                    # keep every step's input gradients / pre-activations alive
                    # into the next forward (3.2 GB on BERT-large, tools/mem_audit.py)
                    for k in ("grad_acc", "dact", "dsum_target"):
                        s.ctx.extra.pop(k, None)
                    self.tracer.end(t0)
                    if self.cfg.sync_debug:
                        self._debug_sync(s, "backward")
                    for v, g, nd in zip(s.inputs, gins, need):
                        if g is not None and nd:
                            self._acc(grads, v, g)
            if sync:
                for p in s.weights:
                    if p.final_step == i and p.trainable:
                        if p.regularizer is not None:
                            self._add_regularizer_grad(p)
                        self._param_done(p)
        self._saved = {}
        self._env = {}
        self._wg_join()
        if sync:
            self._finish_grad_sync()
        if self._ov_flats:
            # buckets whose params never finalised (untrainable) update now, then join
            for f in self.flats:
                if id(f) in self._ov_flats:
                    for b in f["buckets"]:
                        if not b.get("updated"):
                            self._update_bucket(f, b)
            torch.cuda.current_stream(self.cfg.device).wait_stream(self._upd_stream)

    def _sync_row_tracking(self):
        """Embedding backward records touched rows only for tables whose flat
        is on the sparse path (the flag may be cleared after compile)."""
        for f in self.flats:
            for p in f["params"]:
                if 0 <= p.final_step < len(self.steps):
                    ex = self.steps[p.final_step].ctx.extra
                    ex["track_rows"] = bool(f["sparse"] and p.sparse)
                    if not ex["track_rows"]:
                        ex.pop("touched_rows", None)

    def _zero_flat(self, f):
        """Reset a flat's gradients.  Sparse flats only hold non-zero rows the
        last backward touched and no update consumed: clear just those."""
        if not f["sparse"]:
            if f["grad"].is_cuda and K.available():
                K.zero_(f["grad"])
            else:
                f["grad"].zero_()
            return
        for p in f["params"]:
            if not (0 <= p.final_step < len(self.steps)):
                continue
            rows = self.steps[p.final_step].ctx.extra.pop("touched_rows", None)
            if rows:
                n = p.grad.shape[0]
                idx = torch.cat([r.to(torch.long) for r in rows]).clamp_(0, n - 1)
                p.grad.view(n, -1).index_fill_(0, idx, 0)

    def zero_gradients(self):
        """FFModel.zero_gradients: every gradient buffer back to zero."""
        self._sync_row_tracking()
        for f in self.flats:
            self._zero_flat(f)

    def _acc(self, grads, v, g):
        if g is None:
            return
        if v in grads and grads[v] is g:
            return  # accumulated in place by the op
        if v in grads:
            grads[v] = grads[v] + g
        else:
            grads[v] = g

    def _param_done(self, p: ParamPiece):
        fb = self._param_bucket.get(id(p))
        if fb is None:
            return
        f, b = fb
        b["pending"] -= 1
        if b["pending"] == 0 and id(f) in self._ov_flats:
            self._wg_join()
            self._update_bucket(f, b)
        elif b["pending"] == 0 and self.cfg.overlap_grad_sync:
            if self.dist.syncs(f["group"]):
                self._wg_join()
            self._launch_bucket(f, b)

    def _add_regularizer_grad(self, p: ParamPiece):
        """Kernel regularizer (reference Linear backward, linear_kernels.cu:258):
        dW += lambda * W (L2) or lambda * sign(W) (L1).  Added once per step
        to the summed gradient: each of the |group| replicas adds 1/|group| of
        it before the all-reduce sums them."""
        kind, lam = p.regularizer
        lam = lam / max(1, len(p.group))
        # the compute copy is whole on every replica (bf16: all-gathered after
        # each sharded update; fp32: it IS the master, all-gathered likewise);
        # under ZeRO a bf16 run keeps only this rank's shard of the master current
        w = p.compute.view(p.grad.shape)
        if kind == "l2":
            p.grad.add_(w.to(p.grad.dtype), alpha=lam)
        else:
            p.grad.add_(torch.sign(w).to(p.grad.dtype), alpha=lam)

    def _debug_sync(self, s, phase: str):
        """sync_debug: wait for the operator's kernels; a fault surfaces here,
        attributed to the operator."""
        if self.cfg.device.type != "cuda" or torch.cuda.is_current_stream_capturing():
            return
        try:
            torch.cuda.synchronize(self.cfg.device)
        except RuntimeError as e:
            raise RuntimeError(f"device error after {phase} of operator {s.name} ({s.op_type}): {e}") from e

    # ---- weight-gradient side stream
    def _wg_enabled(self) -> bool:
        """Side-stream dW GEMMs: CUDA only, from the second step on (the
        first step's GEMMs are autotuned alone on the compute stream)."""
        if not (self.cfg.wgrad_stream and self.cfg.device.type == "cuda" and self.step_num >= 1):
            return False
        if getattr(self, "_wg", None) is None:
            # (stream, tensors its queued GEMMs read, their storage pointers)
            self._wg = (torch.cuda.Stream(device=self.cfg.device), [], set())
        return True

    def _wg_reads(self, t: Optional[torch.Tensor]) -> bool:
        wg = getattr(self, "_wg", None)
        return bool(t is not None and wg is not None and wg[2] and t.untyped_storage().data_ptr() in wg[2])

    def _wg_join(self):
        """The compute stream waits for every queued dW GEMM; the tensors
        they read may be freed / overwritten from here on."""
        wg = getattr(self, "_wg", None)
        if wg is None or not wg[1]:
            return
        torch.cuda.current_stream(self.cfg.device).wait_stream(wg[0])
        wg[1].clear()
        wg[2].clear()

    def _launch_bucket(self, f, b):
        if self.dist.syncs(f["group"]) and not b.get("launched"):
            if f["zero"]:
                # sharded optimizer: each rank only needs the sum of its shard
                w = self.dist.reduce_scatter_(f["grad"][b["lo"]:b["hi"]], f["group"], async_op=True)
            elif f["ps"]:
                # parameter server: only the group leader needs the summed gradient
                w = self.dist.reduce_(f["grad"][b["lo"]:b["hi"]], f["group"], min(f["group"]), async_op=True)
            else:
                w = self.dist.all_reduce_(f["grad"][b["lo"]:b["hi"]], f["group"], async_op=True)
            b["launched"] = True
            if w is not None:
                self._works.append(w)
                f.setdefault("works", []).append(w)

    def _gather_updated(self):
        """Sharded optimizer: all-gather every bucket's updated compute copy
        (the bf16 weights, or the fp32 master when computing in fp32)."""
        for f in self.flats:
            if not f["zero"] or not self.dist.distributed:
                continue
            tgt = f["compute"] if f["compute"] is not None else f["master"]
            for b in f["buckets"]:
                self.dist.all_gather_(tgt[b["lo"]:b["hi"]], f["group"])

    def _gather_masters(self):
        """Make the fp32 masters whole again (checkpoints, get_parameter)."""
        for f in self.flats:
            if not f["zero"] or not self.dist.distributed or f["compute"] is None:
                continue
            for b in f["buckets"]:
                self.dist.all_gather_(f["master"][b["lo"]:b["hi"]], f["group"])

    def _finish_grad_sync(self):
        for f in self.flats:
            for b in f["buckets"]:
                if not b.get("launched"):
                    self._launch_bucket(f, b)
        for f in self.flats:
            for b in f["buckets"]:
                b["launched"] = False
        if getattr(self, "_defer_grad_wait", False):
            # train_step: update() waits flat by flat, so the optimizer step of
            # a flat whose all-reduces finished (the bf16 GEMM weights) runs
            # while the last buckets (the fp32 embedding tables, finalised at
            # the very end of the backward pass) are still being reduced
            return
        self._wait_works()

    def _wait_works(self, f=None):
        """The compute stream waits for the pending gradient collectives of
        flat ``f`` (all flats when None)."""
        for ff in ([f] if f is not None else self.flats):
            for w in ff.pop("works", []):
                w.wait()
        if f is None:
            self._works = []

    def update(self, lr: Optional[float] = None):
        scale = 1.0
        if self.cfg.grad_clip > 0:
            self._wait_works()
            norm = self.grad_norm()
            if norm > self.cfg.grad_clip:
                scale = self.cfg.grad_clip / (norm + 1e-6)
        pre = getattr(self, "_ov_flats", set())
        for f in self.flats:
            if id(f) in pre:   # updated bucket by bucket during the backward pass
                for b in f["buckets"]:
                    b["updated"] = False
                continue
            if f.get("ps") and self.dist.distributed and self.rank != min(f["group"]):
                continue  # PS: only the leader updates (its optimizer state is the only one)
            self._wait_works(f)
            if f["sparse"]:
                self._sparse_sgd(f, lr, scale)
                continue
            f["opt"].step(lr=lr, grad_scale=scale)
        self._wait_works()   # flats that skipped their step: before the next backward zeroes their grads
        self._ov_flats = set()
        self._gather_updated()
        self._broadcast_ps()
        self.step_num += 1

    def _sparse_sgd(self, f, lr: Optional[float], scale: float):
        """w[r] -= lr * g[r]; g[r] = 0 for the rows the step touched (ids
        recorded by the embedding backward; duplicates write identical values,
        out-of-range ids clamp onto the last row, which then gets the same
        value the dense update gives it -- capture-safe, no boolean mask)."""
        lr = f["opt"].cfg.lr if lr is None else lr
        f["opt"].step_num += 1
        todo = []
        for p in f["params"]:
            if not p.trainable:
                continue
            rows = self.steps[p.final_step].ctx.extra.pop("touched_rows", None)
            if rows:
                todo.append((p, rows))
        from .. import kernels as K
        if todo and todo[0][0].master.is_cuda and K.available():
            # every table of the flat in one native launch pair (the framework
            # path below is ~11 kernels per table)
            tabs = []
            for p, rows in todo:
                n = p.grad.shape[0]
                idx = rows[0] if len(rows) == 1 else torch.cat([r.to(torch.long) for r in rows])
                c = None if p.compute is p.master else p.compute.view(n, -1)
                tabs.append((p.master.view(n, -1), p.grad.view(n, -1), c, idx.reshape(-1)))
            if K.sparse_sgd_rows(tabs, lr * scale):
                return
        for p, rows in todo:
            n = p.grad.shape[0]
            idx = torch.cat([r.to(torch.long) for r in rows]).clamp_(0, n - 1)
            m2, g2 = p.master.view(n, -1), p.grad.view(n, -1)
            vals = m2.index_select(0, idx) - (lr * scale) * g2.index_select(0, idx).float()
            m2.index_copy_(0, idx, vals)
            g2.index_fill_(0, idx, 0)
            if p.compute is not p.master:
                p.compute.view(n, -1).index_copy_(0, idx, vals.to(p.compute.dtype))

    def _broadcast_ps(self):
        """Parameter server: the leader's updated weights go back to the replicas."""
        for f in self.flats:
            if not f.get("ps") or not self.dist.distributed:
                continue
            leader = min(f["group"])
            self.dist.broadcast_(f["master"], f["group"], leader)
            if f["compute"] is not None:
                self.dist.broadcast_(f["compute"], f["group"], leader)

    def grad_norm(self) -> float:
        # every logical gradient element counted once: only the canonical
        # owner (copy 0, partial replica 0, implicit replica 0) of each shard
        tot = torch.zeros(1, device=self.cfg.device, dtype=torch.float64)
        for f in self.flats:
            if f["zero"]:
                # reduce-scattered: every rank of the group owns one shard of the sum
                c = f["params"][0].layout.coord(self.rank)
                if c is not None and c.a == 0 and c.rep == 0:
                    for b in f["buckets"]:
                        s0, s1 = b["shard"]
                        tot += f["grad"][s0:s1].double().pow(2).sum()
        for p in self.params:
            if not p.group or p.grad is None or self.flats[p.flat_id]["zero"]:
                continue
            c = p.layout.coord(self.rank)
            if c is not None and c.b == 0 and c.a == 0 and c.rep == 0:
                tot += p.grad.double().pow(2).sum()
        if self.dist.distributed:
            import torch.distributed as dist
            dist.all_reduce(tot)
        return float(tot.sqrt().item())

    def enable_arena(self, nbytes: int):
        """Run the step's allocations out of one device region of ``nbytes``
        (runtime/arena.py, csrc/runtime/arena.cpp), sized by the caller from
        the liveness memory plan.  Eager steps allocate inside it until a
        graph is captured; captures use it as their pool."""
        from .arena import Arena
        self.arena = Arena(self.cfg.device, int(nbytes))
        # torch's block cache files a freed block under the stream that
        # allocated it and reuses it only on that stream: eager steps, the
        # capture warm-up and the capture itself all run on this one stream,
        # so the capture reuses the blocks the eager steps left in the pool
        self._arena_stream = torch.cuda.Stream(device=self.cfg.device)
        return self.arena

    @contextlib.contextmanager
    def _arena_ctx(self):
        a = getattr(self, "arena", None)
        if a is None or getattr(self, "_graph", None) is not None or torch.cuda.is_current_stream_capturing():
            # after a capture the pool's free blocks belong to the graph
            yield
            return
        s, cur = self._arena_stream, torch.cuda.current_stream(self.cfg.device)
        if s == cur:
            with a.use():
                yield
            return
        s.wait_stream(cur)
        with torch.cuda.stream(s), a.use():
            yield
        cur.wait_stream(s)

    def train_step(self, feeds: Dict[str, torch.Tensor], labels: torch.Tensor, lr: Optional[float] = None):
        with self._arena_ctx():
            self._train_step(feeds, labels, lr)

    def _train_step(self, feeds: Dict[str, torch.Tensor], labels: torch.Tensor, lr: Optional[float] = None):
        self.forward(feeds, training=True, free_env=True)
        prof = self.cfg.profiling
        t0 = self.tracer.begin("__loss__:fwd", "compute", self.step_num) if prof else None
        g = self.compute_loss(labels)
        self.tracer.end(t0)
        self._overlap_lr = (True, lr)
        self._defer_grad_wait = True
        try:
            self.backward(g)
        finally:
            self._overlap_lr = None
            self._defer_grad_wait = False
        t0 = self.tracer.begin("__update__:fwd", "compute", self.step_num) if prof else None
        self.update(lr)
        self.tracer.end(t0)
        self._after_first_update()

    def _after_first_update(self):
        """Once per executor, after the first update (plain or pipelined
        step), outside graph capture:
          * distributed: the first step tuned every GEMM signature on each rank
            on its own, so agree on one kernel per signature before later steps
            / the capture (partial-sum replicas' bias gradients would drift
            apart otherwise);
          * the autotuner's candidates left split-K slabs of every split degree
            they tried in the workspace cache (15.5 GB on GPT-3 medium,
            tools/mem_audit.py): drop them, the chosen kernels re-create theirs."""
        if self.cfg.device.type != "cuda" or torch.cuda.is_current_stream_capturing():
            return
        if self.dist.distributed and not getattr(self, "_choices_synced", False):
            from ..ops.gemm import sync_choices
            sync_choices()
            self._choices_synced = True
        if not getattr(self, "_ws_trimmed", False) and getattr(self, "_graph", None) is None:
            torch.cuda.synchronize(self.cfg.device)
            K.trim_workspaces()
            self._ws_trimmed = True

    def _overlap_flats(self) -> List[dict]:
        """Flats whose buckets may be updated during the backward pass: one
        device, no gradient collective, no global gradient norm, dense."""
        if not self.cfg.overlap_update or self.cfg.grad_clip > 0 or self.cfg.device.type != "cuda":
            return []
        out = []
        for f in self.flats:
            if f["zero"] or f["ps"] or f["sparse"] or (self.dist.syncs(f["group"])):
                continue
            if isinstance(f["opt"], FlatOptimizer) and f["opt"].range_capable():
                out.append(f)
        return out

    def _update_bucket(self, f, b):
        """Run bucket ``b``'s optimizer update on the side stream once the
        compute stream has produced its last gradient (event fork); the main
        stream joins before the next step reads the weights."""
        if self._upd_stream is None:
            self._upd_stream = torch.cuda.Stream(device=self.cfg.device)
        cur = torch.cuda.current_stream(self.cfg.device)
        ev = torch.cuda.Event()
        ev.record(cur)
        self._upd_stream.wait_event(ev)
        with torch.cuda.stream(self._upd_stream):
            f["opt"].step_range(b["lo"], b["hi"], lr=self._overlap_lr[1])
        b["updated"] = True

    def pipeline_stages(self) -> int:
        """Distinct device blocks the strategy places operators on (1 when
        every operator spans the whole world)."""
        blocks = {tuple(v) for v in self.views.values()} if self.views else set()
        return max(1, len(blocks))

    def train_step_pipelined(self, feeds_list: Sequence[Dict[str, torch.Tensor]], labels_list: Sequence[torch.Tensor],
                             lr: Optional[float] = None, schedule: str = "1f1b"):
        with self._arena_ctx():
            self._train_step_pipelined(feeds_list, labels_list, lr, schedule)

    def _train_step_pipelined(self, feeds_list, labels_list, lr=None, schedule: str = "1f1b"):
        """One optimizer step over ``len(feeds_list)`` micro-batches (each of
        the compiled batch shape): gradients accumulated over the
        micro-batches, one synchronisation + update.

        With a strategy that places consecutive layers on disjoint device
        blocks (machine views = pipeline stages), every rank walks the same
        step list, so stage s runs micro-batch i+1's forward while stage s+1
        runs micro-batch i's (the stage-boundary transfers, all-to-alls on
        the two stages' ranks only, are the only rendezvous).  ``schedule``:

          * ``"gpipe"`` -- every forward, then every backward in reverse: m
            micro-batches of activations live at the peak;
          * ``"1f1b"`` -- S (= pipeline stages) warm-up forwards, then one
            backward per forward (B0 F_S B1 F_S+1 ...), then the drain: at
            most S micro-batches live, the same bubble.

        With one stage it is plain gradient accumulation.  The loss gradient
        of each micro-batch is scaled by 1/m, so the update equals the one of
        a single batch m times larger."""
        m = len(feeds_list)
        if m == 0 or m != len(labels_list):
            raise ValueError("train_step_pipelined: need one label tensor per micro-batch")
        if schedule not in ("gpipe", "1f1b"):
            raise ValueError(f"train_step_pipelined: unknown schedule {schedule!r}")
        if schedule == "gpipe":
            order = [("F", i) for i in range(m)] + [("B", i) for i in range(m - 1, -1, -1)]
        else:
            w = min(m, self.pipeline_stages())
            order = [("F", i) for i in range(w)]
            for i in range(m):
                order.append(("B", i))
                if i + w < m:
                    order.append(("F", i + w))
        stash: Dict[int, tuple] = {}
        n_back = 0
        self.peak_live_micro_batches = 0
        for kind, i in order:
            if kind == "F":
                self.forward(feeds_list[i], training=True, free_env=True)
                g = self.compute_loss(labels_list[i])
                if g is not None and m > 1:
                    g = g / m
                stash[i] = (self._saved, self._env, g)
                self.peak_live_micro_batches = max(self.peak_live_micro_batches, len(stash))
            else:
                self._saved, self._env, g = stash.pop(i)
                self.backward(g, zero_grads=(n_back == 0), accumulate=(n_back > 0), sync=(n_back == m - 1))
                n_back += 1
        self.update(lr)
        self._after_first_update()

    def make_graphed_train_step(self, feeds, labels, warmup: int = 2, schedule: str = "1f1b"):
        """Capture one whole training iteration (forward, loss, backward with
        the bucketed RCCL gradient all-reduces, fused optimizer update) into a
        hipGraph and return ``step(feeds=None, labels=None)`` that replays it.

        Inputs/labels live in static device buffers (pass new batches to
        ``step`` to copy them in).  Adam's learning rate and step counter are
        kept on the device, so replays are exact; the GEMM autotuner settles
        during ``warmup`` (eager) before capture.  This replaces the
        reference's Legion tracing (begin_trace/end_trace around the loop).

        ``feeds`` / ``labels`` as LISTS (one entry per micro-batch) capture the
        pipelined step instead (``train_step_pipelined`` with ``schedule``):
        every micro-batch's forward / backward, the stage-boundary transfers
        (graph segments cut at each), one synchronisation + update."""
        if self.cfg.device.type != "cuda":
            raise RuntimeError("graph capture needs a GPU")
        if self.cfg.grad_clip > 0:
            raise RuntimeError("gradient clipping syncs with the host; disable it for graph capture")
        micro = isinstance(feeds, (list, tuple))

        def static_piece_feeds(fd):
            out = {}
            for k, v in fd.items():
                piece = self._local_piece(k, v)
                if piece is not None:
                    out[k] = piece.clone()
            return out

        def static_piece_labels(lb):
            y = self.local_labels(lb)
            return y.clone() if y is not None else None

        if micro:
            if len(feeds) != len(labels) or not feeds:
                raise ValueError("make_graphed_train_step: one label tensor per micro-batch")
            static_feeds = [static_piece_feeds(fd) for fd in feeds]
            static_labels = [static_piece_labels(lb) for lb in labels]

            def run():
                self.train_step_pipelined(static_feeds, static_labels, schedule=schedule)
        else:
            static_feeds = static_piece_feeds(feeds)
            static_labels = static_piece_labels(labels)

            def run():
                self.train_step(static_feeds, static_labels)
        for f in self.flats:
            f["opt"].enable_device_hparams()
        arena = getattr(self, "arena", None)
        side = self._arena_stream if arena is not None else torch.cuda.Stream(device=self.cfg.device)
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(warmup):
                run()
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize(self.cfg.device)
        # no garbage collection inside the capture: a collected cycle that owns
        # a HIP event / stream would call its destroy API mid-capture (abort)
        gc_was_on = gc.isenabled()
        gc.disable()
        K.note_graph_capture()
        try:
            if self.dist.distributed:
                # across ranks: one graph segment between consecutive collectives
                # (runtime/graphs.py); the RCCL calls are re-issued at replay
                graph = self._capture_segments(side, run)
                replay = graph.replay
            else:
                graph = torch.cuda.CUDAGraph()
                with torch.cuda.graph(graph, pool=arena.pool_id if arena is not None else None,
                                      stream=side if arena is not None else None,
                                      capture_error_mode="thread_local"):
                    run()
                replay = graph.replay
                # one device: the step is one graph, launched by the same
                # native replayer (csrc/runtime/replay.cpp) as the segmented
                # multi-rank chain
                R = _native_replay_module()
                if R is not None:
                    rp = R.Replayer()
                    rp.add_graph(graph)
                    self._native_replayer = rp
                    replay = rp.replay
                    self.native_replay = True
        finally:
            if gc_was_on:
                gc.enable()
        self._graph = graph

        def copy_in(dst_feeds, dst_labels, new_feeds, new_labels):
            if new_feeds:
                for k, v in new_feeds.items():
                    if k in dst_feeds:
                        dst_feeds[k].copy_(self._local_piece(k, v), non_blocking=True)
            if new_labels is not None and dst_labels is not None:
                dst_labels.copy_(self.local_labels(new_labels), non_blocking=True)

        def step(new_feeds=None, new_labels=None):
            if micro:
                for i in range(len(static_feeds)):
                    copy_in(static_feeds[i], static_labels[i], new_feeds[i] if new_feeds else None,
                            new_labels[i] if new_labels is not None else None)
            else:
                copy_in(static_feeds, static_labels, new_feeds, new_labels)
            replay()
            self.step_num += 1
            for f in self.flats:
                f["opt"].step_num += 1

        return step

    def _capture_segments(self, side, run):
        """Capture one training step as hipGraph segments cut at every
        collective (runtime/graphs.SegmentRecorder).  Raises NotCapturable
        (after leaving capture mode cleanly) when the step reaches a
        collective that cannot be re-issued from a recorded closure."""
        arena = getattr(self, "arena", None)
        rec = SegmentRecorder(pool=arena.pool_id if arena is not None else None)
        torch.cuda.synchronize(self.cfg.device)
        if arena is None:
            # the eager steps' cached blocks go back to the device first, so the
            # segments' private pool reuses that memory (torch.cuda.graph does
            # the same for a one-graph capture): without it a BERT-large rank
            # reserved 93 GB for a 35 GB step
            torch.cuda.empty_cache()
        self.dist.recorder = rec
        try:
            with torch.cuda.stream(side):
                rec.begin()
                run()
                rec.end()
        except BaseException:
            rec.abort()
            self._works = []
            for f in self.flats:
                f.pop("works", None)
                for b in f["buckets"]:
                    b["launched"] = False
            raise
        finally:
            self.dist.recorder = None
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize(self.cfg.device)
        self.graph_segments = (rec.n_graphs(), rec.n_collectives())
        # the chain replays from C++ (csrc/runtime/replay.cpp) when every
        # collective carries a descriptor and _ffreplay is built
        self.native_replay = rec.build_native()
        return rec

    def zero_metrics(self):
        self.metrics_buf.zero_()
        self.metrics_start = time.time()

    def perf_metrics(self) -> PerfMetrics:
        buf = self.metrics_buf.clone()
        if self.dist.distributed:
            import torch.distributed as dist
            dist.all_reduce(buf)
        out_dim = self.value_layout[self.loss_value].sizes[-1]
        return PerfMetrics.from_buffer(buf, self.metrics_names, self.loss.loss_type if self.loss else "",
                                       self.metrics_start, out_dim)

    # --------------------------------------------------------------- profiling
    def profile_report(self) -> Dict[str, float]:
        """Milliseconds per ``op:fwd`` / ``op:bwd`` / redistribution since the
        last ``tracer.clear()`` (needs ExecConfig.profiling)."""
        return self.tracer.report()

    def export_chrome_trace(self, path: str) -> str:
        return self.tracer.export_chrome_trace(path, {"world": self.world, "rank": self.rank})

    # ------------------------------------------------------------ checkpoint
    def state_dict(self) -> Dict[str, Any]:
        """Local (this rank's) shards + optimizer state + shard metadata."""
        self._gather_masters()
        st = {"step": self.step_num, "rank": self.rank, "world": self.world, "params": {}, "optimizer": []}
        for p in self.params:
            if p.group:
                c = p.layout.coord(self.rank)
                st["params"][p.name] = {"tensor": self._to_logical(p, p.master).detach().cpu().clone(),
                                        "box": p.layout.box(c.shard), "logical_shape": p.logical_shape}
        for f in self.flats:
            st["optimizer"].append({"step": f["opt"].step_num,
                                    **{k: t.detach().cpu().clone() for k, t in f["opt"].state_tensors().items()}})
        return st

    def load_state_dict(self, st: Dict[str, Any]):
        for p in self.params:
            if p.group and p.name in st["params"]:
                p.master.copy_(self._to_physical(p, st["params"][p.name]["tensor"].to(p.master.device)))
                if p.compute is not p.master:
                    p.compute.copy_(p.master)
        for f, o in zip(self.flats, st.get("optimizer", [])):
            f["opt"].step_num = int(o["step"])
            for k, t in f["opt"].state_tensors().items():
                if k in o:
                    t.copy_(o[k].to(t.device))
        self.step_num = int(st.get("step", 0))
