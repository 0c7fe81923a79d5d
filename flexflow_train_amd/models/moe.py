"""Mixture-of-experts classifier (examples/cpp/mixture_of_experts/moe.cc:
input -> gate (Dense + softmax + top-k) -> experts -> aggregate -> softmax).

The reference's ``ff.moe`` relies on GROUP_BY / AGGREGATE operators that do
not exist in its operator vocabulary.  Here ``FFModel.moe``
builds the softmax gate and top-k selection from ordinary operators and
routes tokens through the EXPERTS operator (ops/moe.py), which the search can
shard expert-parallel (replicated tokens + partial sums, or all-to-all
dispatch).  ``build_moe_dense_gating`` keeps the original formulation in
which every expert is its own Dense branch (expert parallelism by placement).
"""
from __future__ import annotations

import dataclasses

import numpy as np

from ..core import ActiMode, DataType, FFModel


@dataclasses.dataclass
class MoEConfig:
    batch_size: int = 64
    input_dim: int = 784
    num_experts: int = 8
    num_select: int = 2
    expert_hidden: int = 512
    num_classes: int = 10
    expert_parallel_mode: str = "replicated"


def build_moe(model: FFModel, cfg: MoEConfig):
    x = model.create_tensor([cfg.batch_size, cfg.input_dim], DataType.DT_FLOAT, name="input")
    h = model.moe(x, cfg.num_experts, cfg.num_select, cfg.expert_hidden, out_dim=cfg.num_classes,
                  expert_parallel_mode=cfg.expert_parallel_mode, name="moe")
    return {"input": x}, model.softmax(h, name="softmax")


def build_moe_dense_gating(model: FFModel, cfg: MoEConfig):
    x = model.create_tensor([cfg.batch_size, cfg.input_dim], DataType.DT_FLOAT, name="input")
    gate = model.softmax(model.dense(x, cfg.num_experts, name="gate"), name="gate_softmax")
    vals, _ = model.top_k(gate, cfg.num_select, True, name="gate_topk")
    kth = model.split(vals, [cfg.num_select - 1, 1], 1, name="kth_split")[1] if cfg.num_select > 1 else vals
    # weights = gate * [gate >= kth], built from supported elementwise ops
    margin = model.subtract(gate, kth, name="gate_margin")                 # >= 0 for selected experts
    sel = model.relu(model.scalar_add(model.scalar_multiply(margin, 1e6, name="gate_sharpen"), 1.0,
                                      name="gate_shift"), name="gate_sel")  # >0 iff selected
    sel = model.min(sel, model.scalar_add(model.scalar_multiply(sel, 0.0, name="zeros"), 1.0, name="ones"),
                    name="gate_clip")                                        # in {0,1} (up to ties)
    weights = model.multiply(gate, sel, name="gate_weights")
    experts = model.split(weights, [1] * cfg.num_experts, 1, name="gate_split")
    out = None
    for e in range(cfg.num_experts):
        h = model.dense(x, cfg.expert_hidden, ActiMode.AC_MODE_RELU, name=f"expert{e}.fc1")
        h = model.dense(h, cfg.num_classes, name=f"expert{e}.fc2")
        h = model.multiply(h, experts[e], name=f"expert{e}.scale")
        out = h if out is None else model.add(out, h, name=f"expert_sum{e}")
    return {"input": x}, model.softmax(out, name="softmax")


def moe_synthetic(cfg: MoEConfig, rng: np.random.Generator):
    return ({"input": rng.standard_normal((cfg.batch_size, cfg.input_dim), dtype=np.float32)},
            rng.integers(0, cfg.num_classes, (cfg.batch_size, 1), dtype=np.int32))
