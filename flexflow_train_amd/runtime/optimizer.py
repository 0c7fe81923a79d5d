"""Optimizers over flat parameter buffers.

Parity: SGD (lr, momentum, nesterov, weight_decay) and Adam (alpha, beta1,
beta2, weight_decay, epsilon; alpha_t bias correction) from
lib/pcg/include/pcg/optimizer_attrs (sgd/adam_optimizer_attrs.struct.toml),
lib/runtime/src/optimizer.cc:101-230 and lib/kernels/src/cuda/
optimizer_kernel.cu.  The reference's new local executor leaves update()
unimplemented (local_training_backing.cc:148-150); here every parameter of a
rank lives in one flat fp32 buffer per gradient-sync group, so one fused HIP
launch updates the whole model and refreshes the bf16 compute copy.
"""
from __future__ import annotations

import dataclasses
from typing import Optional

import torch

from .. import kernels as K


@dataclasses.dataclass
class SGDConfig:
    lr: float = 0.01
    momentum: float = 0.0
    nesterov: bool = False
    weight_decay: float = 0.0


@dataclasses.dataclass
class AdamConfig:
    lr: float = 0.001           # "alpha" in the reference
    beta1: float = 0.9
    beta2: float = 0.999
    weight_decay: float = 0.0
    epsilon: float = 1e-8
    decoupled: bool = False     # AdamW (decoupled) vs Adam (L2 folded into the gradient, the reference)


class FlatOptimizer:
    """Optimizer state for one flat buffer (master fp32 + optional bf16 copy)."""

    def __init__(self, cfg, master: torch.Tensor, grad: torch.Tensor, bf16_copy: Optional[torch.Tensor]):
        self.cfg = cfg
        self.master = master
        self.grad = grad
        self.bf16 = bf16_copy
        self.step_num = 0
        self.hp: Optional[torch.Tensor] = None   # device {lr, step} for hipGraph replay (Adam)
        self.m = self.v = self.mom = None
        if isinstance(cfg, AdamConfig):
            self.m = torch.zeros_like(master)
            self.v = torch.zeros_like(master)
        elif cfg.momentum:
            self.mom = torch.zeros_like(master)

    def state_tensors(self):
        return {k: t for k, t in (("m", self.m), ("v", self.v), ("mom", self.mom)) if t is not None}

    def enable_device_hparams(self):
        """Keep {lr, step} in device memory so a captured hipGraph of the
        training step replays with the current learning rate / bias correction."""
        if isinstance(self.cfg, AdamConfig) and self.master.is_cuda and self.hp is None:
            self.hp = torch.tensor([float(self.cfg.lr), float(self.step_num)], device=self.master.device)

    def set_lr(self, lr: float):
        self.cfg.lr = lr
        if self.hp is not None:
            self.hp[0].fill_(float(lr))

    # ---- bucket-wise update (executor: overlapped with the backward pass)
    def range_capable(self) -> bool:
        return self.master.is_cuda and K.available() and self.master.numel() % 8 == 0

    def begin_step(self):
        """Advance the step counters once; ``step_range`` then updates slices."""
        self.step_num += 1
        if self.hp is not None:
            self.hp[1:].add_(1.0)

    def step_range(self, lo: int, hi: int, lr: Optional[float] = None, grad_scale: float = 1.0):
        """Update elements [lo, hi) with the counters of the current step
        (after ``begin_step``); HIP path only (``range_capable``)."""
        c = self.cfg
        lr = c.lr if lr is None else lr
        sl = slice(lo, hi)
        bf = self.bf16[sl] if self.bf16 is not None else None
        if isinstance(c, AdamConfig):
            K.adam_step(self.master[sl], self.grad[sl], self.m[sl], self.v[sl], bf, lr, c.beta1, c.beta2, c.epsilon,
                        c.weight_decay, self.step_num, grad_scale, c.decoupled, hp=self.hp)
        else:
            K.sgd_step(self.master[sl], self.grad[sl], self.mom[sl] if self.mom is not None else None, bf, lr,
                       c.momentum, c.weight_decay, c.nesterov, grad_scale)

    def step(self, lr: Optional[float] = None, grad_scale: float = 1.0):
        self.step_num += 1
        c = self.cfg
        lr = c.lr if lr is None else lr
        if self.master.numel() == 0:
            return
        use_hip = self.master.is_cuda and K.available() and self.master.numel() % 4 == 0
        if isinstance(c, AdamConfig):
            if use_hip:
                if self.hp is not None:
                    self.hp[1:].add_(1.0)   # device-side step counter (captured with the graph)
                K.adam_step(self.master, self.grad, self.m, self.v, self.bf16, lr, c.beta1, c.beta2, c.epsilon,
                            c.weight_decay, self.step_num, grad_scale, c.decoupled, hp=self.hp)
                return
            g = self.grad * grad_scale
            if not c.decoupled and c.weight_decay:
                g = g + c.weight_decay * self.master
            self.m.mul_(c.beta1).add_(g, alpha=1 - c.beta1)
            self.v.mul_(c.beta2).addcmul_(g, g, value=1 - c.beta2)
            bc1 = 1 - c.beta1 ** self.step_num
            bc2 = 1 - c.beta2 ** self.step_num
            upd = (self.m / bc1) / ((self.v / bc2).sqrt() + c.epsilon)
            if c.decoupled and c.weight_decay:
                upd = upd + c.weight_decay * self.master
            self.master.add_(upd, alpha=-lr)
        else:
            if use_hip:
                K.sgd_step(self.master, self.grad, self.mom, self.bf16, lr, c.momentum, c.weight_decay,
                           c.nesterov, grad_scale)
                return
            g = self.grad * grad_scale
            if c.weight_decay:
                g = g + c.weight_decay * self.master
            if self.mom is not None:
                self.mom.mul_(c.momentum).add_(g)
                g = g + c.momentum * self.mom if c.nesterov else self.mom
            self.master.add_(g, alpha=-lr)
        if self.bf16 is not None:
            self.bf16.copy_(self.master)


class ShardedOptimizer:
    """ZeRO-style sharded optimizer over one flat buffer: this rank updates
    (and keeps optimizer state for) only its shard of every gradient bucket;
    the executor reduce-scatters gradients into those shards and all-gathers
    the updated weights.  Optimizer memory and update traffic drop by the
    data-parallel degree; the collective volume equals one all-reduce.
    (The reference has no sharded optimizer)"""

    def __init__(self, cfg, master: torch.Tensor, grad: torch.Tensor, bf16_copy: Optional[torch.Tensor],
                 shards):
        self.cfg = cfg
        self.master = master
        self.shards = list(shards)
        self.parts = [FlatOptimizer(cfg, master[a:b], grad[a:b], bf16_copy[a:b] if bf16_copy is not None else None)
                      for a, b in self.shards]

    @property
    def step_num(self) -> int:
        return self.parts[0].step_num if self.parts else 0

    @step_num.setter
    def step_num(self, v: int):
        for p in self.parts:
            p.step_num = v

    @property
    def hp(self):
        return self.parts[0].hp if self.parts else None

    def state_tensors(self):
        out = {}
        for i, p in enumerate(self.parts):
            for k, t in p.state_tensors().items():
                out[f"{k}.{i}"] = t
        return out

    def enable_device_hparams(self):
        for p in self.parts:
            p.enable_device_hparams()

    def set_lr(self, lr: float):
        self.cfg.lr = lr
        for p in self.parts:
            p.set_lr(lr)

    def step(self, lr: Optional[float] = None, grad_scale: float = 1.0):
        for p in self.parts:
            p.step(lr=lr, grad_scale=grad_scale)
