"""Operator implementation interface and registry.

Every PCG compute operator maps to an ``OpImpl`` that runs on the *local
piece* of its parallel tensors (the executor hands it this rank's shards):

* ``forward(ctx, inputs, weights) -> (outputs, saved)``
* ``backward(ctx, saved, grad_outputs, weight_grads) -> input_grads``
  weight gradients are ACCUMULATED into the fp32 buffers in ``weight_grads``
  (views of the flat gradient buffer, ``None`` when not needed).

Parity: lib/local-execution/src/ops/*.cc (init/forward/backward task impls
per op) + lib/kernels/include/kernels/*_kernels.h.  Instead of task
signatures / slot bindings (op_task_signature.cc, op_task_invocation.cc) an
op receives plain tensors: on MI355X the executor is a single process per GPU
issuing HIP launches on one stream, so no Legion-style privilege plumbing is
needed.
"""
from __future__ import annotations

import dataclasses
from typing import Any, Callable, Dict, List, Optional, Sequence

import torch

_REGISTRY: Dict[str, "OpImpl"] = {}


@dataclasses.dataclass
class OpContext:
    op_type: str
    attrs: Dict[str, Any]
    name: str
    # position of this rank in the op's task space
    sum_index: int = 0          # partial-sum replica index of the output
    sum_degree: int = 1
    copy_index: int = 0
    input_copy_degree: int = 1  # e.g. attention head parallel degree
    input_sum_degree: int = 1
    training: bool = True
    compute_dtype: torch.dtype = torch.float32
    device: torch.device = torch.device("cpu")
    seed: int = 0
    step: int = 0
    output_shapes: Optional[List[Sequence[int]]] = None
    extra: Dict[str, Any] = dataclasses.field(default_factory=dict)

    def a(self, key, default=None):
        return self.attrs.get(key, default)


class OpImpl:
    """Base class; subclasses register with @register("OP_TYPE", ...)."""

    def forward(self, ctx: OpContext, inputs: List[torch.Tensor], weights: List[torch.Tensor]):
        raise NotImplementedError

    def backward(self, ctx: OpContext, saved, grad_outputs: List[Optional[torch.Tensor]],
                 weight_grads: List[Optional[torch.Tensor]], need_input_grad: List[bool]):
        raise NotImplementedError

    # Weight initialisation hook (op-aware fan computation); default None ->
    # generic initializer on the logical shape.
    def init_weight(self, ctx: OpContext, index: int, logical_shape, initializer: dict, gen: torch.Generator):
        return None

    # Counter-based (sharded) initialisation: (kind, a, b, c, d) for
    # runtime.initializers.counter_init_piece, or None for the generic mapping.
    def init_spec(self, ctx: OpContext, index: int, logical_shape, initializer: dict):
        return None

    # Physical storage of a weight piece.  Ops whose kernels want a fused /
    # permuted layout (attention: one [E, 3*Hl*k] QKV operand) override these;
    # the executor stores physical pieces and converts at every logical
    # boundary (set/get_parameter, checkpoints), so a logical element keeps
    # its meaning under any sharding.
    def to_physical(self, attrs: dict, index: int, piece: torch.Tensor) -> torch.Tensor:
        return piece

    def to_logical(self, attrs: dict, index: int, piece: torch.Tensor) -> torch.Tensor:
        return piece


def register(*op_types: str) -> Callable:
    def deco(cls):
        inst = cls()
        for t in op_types:
            _REGISTRY[t] = inst
        return cls

    return deco


def get_impl(op_type: str) -> OpImpl:
    if op_type not in _REGISTRY:
        raise NotImplementedError(f"no runtime implementation for operator {op_type}")
    return _REGISTRY[op_type]


def registered_ops() -> List[str]:
    return sorted(_REGISTRY)


def acc_grad(buf: Optional[torch.Tensor], value: torch.Tensor):
    """Accumulate ``value`` into the fp32 weight-gradient view ``buf``."""
    if buf is None:
        return
    buf.add_(value.reshape(buf.shape).to(buf.dtype))
