"""Checkpoint / resume.

Reference: the legacy runtime has no real checkpointing (SURVEY §5.4 —
only Tensor.get_tensor/set_tensor round-trips and the strategy file); this
module provides sharded checkpoints for the per-rank executor:

* ``save_checkpoint(model, dir)``: every rank writes ``rank<r>.pt`` holding
  its LOGICAL weight pieces (with their boxes in the full tensor) and its
  flat optimizer state; rank 0 writes ``meta.json`` (world, step, strategy
  fingerprint, parameter shapes).  Files are written with ``torch.save`` of
  plain tensors/dicts and read back with ``weights_only=True``.
* ``load_checkpoint(model, dir)``: same world + same strategy -> exact resume
  (weights + optimizer state + step).  Different world or strategy -> the
  full logical weights are reassembled from every rank's boxes and
  re-sliced for the new layout (optimizer state restarts).
"""
from __future__ import annotations

import json
import os
import re
import shutil
from typing import Dict, Optional

import torch


def _fingerprint(ex) -> str:
    return str(ex.pcg.structural_hash()) + "@" + str(ex.world) + ":" + json.dumps(
        sorted((int(k), list(v)) for k, v in ex.views.items()))


def save_checkpoint(model, path: str, progress: Optional[dict] = None):
    """Every rank writes its shard; rank 0 writes meta.json only after every
    rank's file is complete (barrier), so a directory WITH meta.json is a
    complete checkpoint.  ``progress``: training-loop position (fit resume)."""
    ex = model.executor if hasattr(model, "executor") else model
    os.makedirs(path, exist_ok=True)
    if ex.rank == 0:
        # rewriting an existing directory: it stops counting as complete
        # before any shard is replaced, so a crash mid-save cannot leave old
        # meta.json beside a mix of old and new shards
        try:
            os.remove(os.path.join(path, "meta.json"))
        except FileNotFoundError:
            pass
    ex.dist.barrier()
    st = ex.state_dict()
    tmp = os.path.join(path, f"rank{ex.rank}.pt.tmp")
    torch.save(st, tmp)
    os.replace(tmp, os.path.join(path, f"rank{ex.rank}.pt"))
    ex.dist.barrier()
    if ex.rank == 0:
        meta = {"format": "ffmi355x.checkpoint.v1", "world": ex.world, "step": ex.step_num,
                "fingerprint": _fingerprint(ex),
                "params": {p.name: list(p.logical_shape) for p in ex.params}}
        if progress is not None:
            meta["progress"] = progress
        with open(os.path.join(path, "meta.json.tmp"), "w") as f:
            json.dump(meta, f, indent=1)
        os.replace(os.path.join(path, "meta.json.tmp"), os.path.join(path, "meta.json"))
    ex.dist.barrier()


_STEP_DIR = re.compile(r"^step-(\d+)$")


def latest_checkpoint(root: str) -> Optional[str]:
    """Newest COMPLETE step checkpoint under ``root`` (a ``step-N`` directory
    holding meta.json), or None."""
    if not root or not os.path.isdir(root):
        return None
    best = None
    for d in os.listdir(root):
        m = _STEP_DIR.match(d)
        if m and os.path.exists(os.path.join(root, d, "meta.json")):
            if best is None or int(m.group(1)) > best[0]:
                best = (int(m.group(1)), d)
    return os.path.join(root, best[1]) if best else None


def save_step_checkpoint(model, root: str, progress: dict, keep: int = 2) -> str:
    """``root/step-<N>`` for the executor's step N; older complete step
    checkpoints beyond the newest ``keep`` are removed (rank 0)."""
    ex = model.executor if hasattr(model, "executor") else model
    path = os.path.join(root, f"step-{ex.step_num}")
    save_checkpoint(model, path, progress)
    if ex.rank == 0 and keep > 0:
        # only COMPLETE checkpoints (meta.json written) count towards `keep`;
        # a directory without meta.json is the leftover of a crashed save
        # (every rank writes the same step and meets at the barrier below, so
        # none is in progress here) and is removed on its own
        done, stale = [], []
        for d in os.listdir(root):
            m = _STEP_DIR.match(d)
            if m:
                (done if os.path.exists(os.path.join(root, d, "meta.json")) else stale).append((int(m.group(1)), d))
        done.sort()
        for _n, d in done[:-keep] + stale:
            shutil.rmtree(os.path.join(root, d), ignore_errors=True)
    ex.dist.barrier()
    return path


def _assemble_full(path: str, world: int) -> Dict[str, torch.Tensor]:
    full: Dict[str, torch.Tensor] = {}
    for r in range(world):
        f = os.path.join(path, f"rank{r}.pt")
        if not os.path.exists(f):
            continue
        st = torch.load(f, map_location="cpu", weights_only=True)
        for name, rec in st["params"].items():
            t = full.get(name)
            if t is None:
                t = full[name] = torch.zeros(tuple(rec["logical_shape"]), dtype=torch.float32)
            box = tuple(slice(lo, hi) for lo, hi in rec["box"])
            t[box] = rec["tensor"].reshape(t[box].shape)
    return full


def read_checkpoint_meta(path: str) -> dict:
    with open(os.path.join(path, "meta.json")) as f:
        return json.load(f)


def load_checkpoint(model, path: str, strict: bool = True):
    ex = model.executor if hasattr(model, "executor") else model
    meta = read_checkpoint_meta(path)
    if meta.get("format") != "ffmi355x.checkpoint.v1":
        raise ValueError(f"{path}: not a checkpoint")
    same = meta["world"] == ex.world and meta["fingerprint"] == _fingerprint(ex)
    if same and os.path.exists(os.path.join(path, f"rank{ex.rank}.pt")):
        st = torch.load(os.path.join(path, f"rank{ex.rank}.pt"), map_location="cpu", weights_only=True)
        ex.load_state_dict(st)
    else:
        full = _assemble_full(path, meta["world"])
        names = set(ex.parameter_names())
        missing = names - set(full)
        if strict and missing:
            raise KeyError(f"checkpoint lacks parameters: {sorted(missing)}")
        for n in names & set(full):
            ex.set_parameter(n, full[n])
        for p in ex.params:
            if p.group and p.compute is not p.master:
                p.compute.copy_(p.master)
        ex.step_num = int(meta.get("step", 0))
    ex.dist.barrier()
    return meta
