"""Dynamic recompilation (re-parallelisation mid-training).

Parity: lib/runtime/src/recompile.h:26-41 / recompile_state.cc:21-37 and
``FFModel::recompile_on_condition`` (model.h:107): a ``trigger`` predicate
is checked every call; when it fires, ``alter`` mutates the model / config
(only on the first recompilation, as in the reference) and the model is
recompiled.  Here recompilation re-runs the strategy search (or imports /
data-parallel, per the possibly altered FFConfig), rebuilds the per-rank
executor and carries the full logical weights, the optimizer moments and
the step counters over to the new parallelisation, so training continues
seamlessly under the new strategy (the MoE example's use, moe.cc:204).
"""
from __future__ import annotations

from typing import Callable


class RecompileState:
    def __init__(self, trigger_func: Callable, alter_func: Callable, ffmodel=None):
        self.trigger_func = trigger_func
        self.alter_func = alter_func
        self.ff = ffmodel
        self.recompilations = 0

    def trigger(self) -> bool:
        return bool(self.trigger_func(self.ff))

    def alter(self):
        if self.recompilations == 0:
            self.alter_func(self.ff)
        self.recompilations += 1
