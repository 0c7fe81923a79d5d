"""Checkpoint / resume.

Reference: the legacy runtime has no real checkpointing (SURVEY §5.4 —
only Tensor.get_tensor/set_tensor round-trips and the strategy file, and the
new FFI's CG (de)serialisation, lib/pcg/ffi/include/flexflow/pcg.h:45-54);
this module provides sharded checkpoints for the per-rank executor.  A
checkpoint directory holds:

* ``rank<r>.pt`` (every rank): its LOGICAL weight pieces with their boxes in
  the full tensor, the same pieces of its optimizer state (Adam m / v,
  momentum), the flat optimizer state as stored (for an exact same-layout
  resume), the per-flat step counters and the torch CPU / GPU RNG states.
  Written with ``torch.save`` of plain tensors / dicts, read back with
  ``weights_only=True``.
* ``meta.json`` (rank 0, written last: a directory with it is complete):
  world, step, strategy fingerprint, parameter shapes, progress.
* ``model.json`` — the computation graph in the CG JSON v1 format
  (``ComputationGraph.to_json``), when the FFModel is known.
* ``strategy.json`` — the parallel strategy (PCG + placements) in the
  ``--import-strategy`` format, so ``FFConfig.import_strategy_file`` can
  rebuild the exact layout the checkpoint was written under.

``load_checkpoint(model, dir)``: same world + same strategy -> exact resume
(weights + optimizer state + step + RNG).  Different world or strategy ->
the full logical weights AND optimizer state are reassembled from every
rank's boxes and re-sliced for the new layout, the step counters carried
over.  Only the ZeRO-sharded optimizer (``shard_optimizer``) keeps its state
rank-local and restarts it on a layout change (meta records
``optimizer_resharded: false``).
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
    st["opt_pieces"] = _optimizer_pieces(ex)
    st["rng"] = {"cpu": torch.get_rng_state()}
    if torch.cuda.is_available() and ex.cfg.device.type == "cuda":
        st["rng"]["cuda"] = torch.cuda.get_rng_state(ex.cfg.device)
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
        meta["optimizer"] = {"keys": ex._opt_state_keys(), "sharded": bool(ex.cfg.shard_optimizer)}
        cg = getattr(model, "cg", None)
        if cg is not None:
            with open(os.path.join(path, "model.json.tmp"), "w") as f:
                f.write(cg.to_json())
            os.replace(os.path.join(path, "model.json.tmp"), os.path.join(path, "model.json"))
            meta["model"] = "model.json"
        from ..search.strategy import export_strategy
        export_strategy(os.path.join(path, "strategy.json"), ex.pcg, ex.views,
                        {"world": ex.world, "source": "checkpoint"})
        meta["strategy"] = "strategy.json"
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


def _rank_files(path: str, world: int):
    for r in range(world):
        f = os.path.join(path, f"rank{r}.pt")
        if os.path.exists(f):
            yield r, f


def _add_params(full: Dict[str, torch.Tensor], st: dict):
    for name, rec in st["params"].items():
        t = full.get(name)
        if t is None:
            t = full[name] = torch.zeros(tuple(rec["logical_shape"]), dtype=torch.float32)
        box = tuple(slice(lo, hi) for lo, hi in rec["box"])
        t[box] = rec["tensor"].reshape(t[box].shape)


def _optimizer_pieces(ex) -> Dict[str, dict]:
    """This rank's LOGICAL pieces of every weight's optimizer state (the
    canonical owner of each shard only), boxed like the weights."""
    keys = ex._opt_state_keys()
    out: Dict[str, dict] = {}
    if not keys or ex.cfg.shard_optimizer:
        return out
    for p in ex.params:
        if not p.group:
            continue
        c = p.layout.coord(ex.rank)
        if c is None or c.b != 0 or c.rep != 0 or c.a != 0:
            continue
        opt = ex.flats[p.flat_id]["opt"]
        rec = {"box": p.layout.box(c.shard), "logical_shape": p.logical_shape}
        for k in keys:
            flat = getattr(opt, k, None)
            if flat is None:
                continue
            piece = flat[p.offset:p.offset + p.numel].view(p.layout.piece_shape)
            rec[k] = ex._to_logical(p, piece).detach().float().cpu().clone()
        out[p.name] = rec
    return out


def _add_opt_pieces(full: Dict[str, Dict[str, torch.Tensor]], st: dict):
    for name, rec in st.get("opt_pieces", {}).items():
        box = tuple(slice(lo, hi) for lo, hi in rec["box"])
        for k, t in rec.items():
            if k in ("box", "logical_shape"):
                continue
            dst = full.setdefault(name, {}).get(k)
            if dst is None:
                dst = full[name][k] = torch.zeros(tuple(rec["logical_shape"]), dtype=torch.float32)
            dst[box] = t.reshape(dst[box].shape)


def _assemble_once(path: str, world: int, rng_rank: int):
    """One pass over the saved rank files (each loaded once, then dropped):
    the logical weights, the logical optimizer state, the optimizer step
    counter and the RNG state of ``rng_rank``'s file."""
    full: Dict[str, torch.Tensor] = {}
    ofull: Dict[str, Dict[str, torch.Tensor]] = {}
    steps, rng = None, None
    for r, f in _rank_files(path, world):
        st = torch.load(f, map_location="cpu", weights_only=True)
        _add_params(full, st)
        _add_opt_pieces(ofull, st)
        opts = st.get("optimizer") or []
        if steps is None and opts:
            steps = int(opts[0]["step"])
        if r == rng_rank:
            rng = {"rng": st.get("rng")}
        del st
    return full, ofull, steps, rng


def _restore_rng(st: dict, ex):
    rng = st.get("rng") or {}
    if "cpu" in rng:
        torch.set_rng_state(rng["cpu"])
    if "cuda" in rng and torch.cuda.is_available() and ex.cfg.device.type == "cuda":
        torch.cuda.set_rng_state(rng["cuda"], ex.cfg.device)


def read_checkpoint_meta(path: str) -> dict:
    with open(os.path.join(path, "meta.json")) as f:
        return json.load(f)


def load_checkpoint(model, path: str, strict: bool = True):
    ex = model.executor if hasattr(model, "executor") else model
    meta = read_checkpoint_meta(path)
    if meta.get("format") != "ffmi355x.checkpoint.v1":
        raise ValueError(f"{path}: not a checkpoint")
    same = meta["world"] == ex.world and meta["fingerprint"] == _fingerprint(ex)
    mine = os.path.join(path, f"rank{ex.rank}.pt")
    if same and os.path.exists(mine):
        st = torch.load(mine, map_location="cpu", weights_only=True)
        ex.load_state_dict(st)
        _restore_rng(st, ex)
        meta["resharded"] = False
    else:
        rng_rank = ex.rank if ex.rank < meta["world"] else 0
        full, ofull, steps, rng = _assemble_once(path, meta["world"], rng_rank)
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
        # optimizer state: reassembled per weight and re-sliced like the weights
        opt_ok = not ex.cfg.shard_optimizer and not meta.get("optimizer", {}).get("sharded", False)
        if opt_ok:
            for n in names & set(ofull):
                ex.set_optimizer_state(n, ofull[n])
            for f in ex.flats:
                f["opt"].step_num = steps if steps is not None else ex.step_num
        if rng is not None:
            _restore_rng(rng, ex)
        meta["resharded"] = True
        meta["optimizer_resharded"] = opt_ok
    ex.dist.barrier()
    return meta
