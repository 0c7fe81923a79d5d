"""The reference's legacy protobuf strategy files (``--import-strategy`` /
``--export-strategy`` with a ``.pb`` file).

Format (``FFProtoBuf::Strategy``, written by examples/cpp/DLRM/strategies/
dlrm_strategy.cc and shipped as dlrm_strategy_*embs_*gpus.pb; the .proto
itself is not in the reference tree, the field numbers below are read off
those files' wire encoding):

    message Strategy { repeated Op ops = 1; }
    message Op {
      string name = 1;
      DeviceType device_type = 2;        // GPU = 0, CPU = 1
      repeated int32 dims = 3;           // parallel degree per tensor dim, innermost dim FIRST
      repeated int32 device_ids = 4;     // one device per part
      repeated MemoryType memory_types = 5;  // FBM = 0 (framebuffer), ZCM = 1 (zero-copy host)
    }

A record's ``dims`` are the legacy ParallelConfig: reversed tensor order, so
the LAST entry is the sample (batch) degree and, for a Linear / Embedding,
the first is the output-channel degree (``add_linear_config(...,
num_parts_channel, num_parts_sample, ...)``).  Records are keyed by op name;
the DLRM files use generic names ("embedding3", "linear", "concat"), so a
record applies to

  1. the layer with exactly that name, else
  2. ``<type><i>``: the i-th layer of that operator type, else
  3. ``<type>``: every layer of that type without a more specific record;

layers without any record run data parallel (the legacy default).  The
device list becomes a machine view (first device, block size): a table on
GPU 3 is the view (3, 1).  Memory types are parsed and reported but all
tensors live in HBM (288 GB per MI355X makes the zero-copy placement of
the 16 GB-class GPUs unnecessary).
"""
from __future__ import annotations

import json
from typing import Dict, List, Optional, Tuple

from .. import _ffcore as C

_TYPE_NAMES = {
    "embedding": "EMBEDDING", "linear": "LINEAR", "dense": "LINEAR", "concat": "CONCAT",
    "batch_matmul": "BATCHMATMUL", "batchmatmul": "BATCHMATMUL", "transpose": "TRANSPOSE", "conv2d": "CONV2D",
    "conv": "CONV2D", "pool2d": "POOL2D", "pool": "POOL2D", "softmax": "SOFTMAX", "attention": "MULTIHEAD_ATTENTION",
    "multihead_attention": "MULTIHEAD_ATTENTION", "layer_norm": "LAYERNORM", "layernorm": "LAYERNORM",
    "batch_norm": "BATCHNORM", "flat": "FLAT", "reshape": "RESHAPE", "dropout": "DROPOUT",
}
_LOSS_NAMES = ("mse_loss", "loss", "cross_entropy", "sparse_cross_entropy")
_DEVICE = {0: "GPU", 1: "CPU"}
_MEMORY = {0: "FBM", 1: "ZCM"}


# ------------------------------------------------------------------ wire codec
def _varint(b: bytes, i: int) -> Tuple[int, int]:
    r = s = 0
    while True:
        if i >= len(b):
            raise ValueError("truncated varint")
        c = b[i]
        i += 1
        r |= (c & 0x7F) << s
        s += 7
        if c < 0x80:
            return r, i


def _fields(b: bytes):
    i = 0
    while i < len(b):
        key, i = _varint(b, i)
        f, w = key >> 3, key & 7
        if w == 0:
            v, i = _varint(b, i)
        elif w == 2:
            n, i = _varint(b, i)
            v = b[i:i + n]
            i += n
        elif w == 5:
            v = b[i:i + 4]
            i += 4
        elif w == 1:
            v = b[i:i + 8]
            i += 8
        else:
            raise ValueError(f"unsupported wire type {w}")
        yield f, w, v


def _ints(w: int, v) -> List[int]:
    if w == 0:
        return [v]
    out, i = [], 0                      # packed repeated field
    while i < len(v):
        x, i = _varint(v, i)
        out.append(x)
    return out


def decode(data: bytes) -> List[dict]:
    ops = []
    for f, w, v in _fields(data):
        if f != 1 or w != 2:
            continue
        op = {"name": "", "device_type": "GPU", "dims": [], "device_ids": [], "memory_types": []}
        for g, gw, gv in _fields(v):
            if g == 1 and gw == 2:
                op["name"] = gv.decode()
            elif g == 2:
                op["device_type"] = _DEVICE.get(_ints(gw, gv)[0], "GPU")
            elif g == 3:
                op["dims"] += _ints(gw, gv)
            elif g == 4:
                op["device_ids"] += _ints(gw, gv)
            elif g == 5:
                op["memory_types"] += [_MEMORY.get(x, str(x)) for x in _ints(gw, gv)]
        ops.append(op)
    return ops


def _enc_varint(x: int) -> bytes:
    out = bytearray()
    while True:
        c = x & 0x7F
        x >>= 7
        if x:
            out.append(c | 0x80)
        else:
            out.append(c)
            return bytes(out)


def _enc_field(f: int, w: int, payload: bytes) -> bytes:
    return _enc_varint((f << 3) | w) + payload


def encode(ops: List[dict]) -> bytes:
    """Same (unpacked) encoding protobuf-cpp's SerializeToOstream wrote for
    the reference's files."""
    dev = {v: k for k, v in _DEVICE.items()}
    mem = {v: k for k, v in _MEMORY.items()}
    out = bytearray()
    for op in ops:
        body = bytearray()
        name = op["name"].encode()
        body += _enc_field(1, 2, _enc_varint(len(name)) + name)
        body += _enc_field(2, 0, _enc_varint(dev.get(op.get("device_type", "GPU"), 0)))
        for d in op.get("dims", []):
            body += _enc_field(3, 0, _enc_varint(int(d)))
        for d in op.get("device_ids", []):
            body += _enc_field(4, 0, _enc_varint(int(d)))
        for m in op.get("memory_types", []):
            body += _enc_field(5, 0, _enc_varint(mem.get(m, 0)))
        out += _enc_field(1, 2, _enc_varint(len(body)) + bytes(body))
    return bytes(out)


def is_legacy_file(path: str) -> bool:
    if path.endswith(".pb"):
        return True
    with open(path, "rb") as f:
        head = f.read(64).lstrip()
    return not head.startswith(b"{")


# -------------------------------------------------------------- to a strategy
def _records_for_layers(cg, ops: List[dict]) -> Dict[int, dict]:
    layers = [n for n in cg.topo_order() if cg.layer_op(n).op_type not in ("INPUT", "WEIGHT")]
    by_name = {cg.layer_name(n): n for n in layers if cg.layer_name(n)}
    by_type: Dict[str, List[int]] = {}
    for n in layers:
        by_type.setdefault(cg.layer_op(n).op_type, []).append(n)
    exact, indexed, generic = {}, {}, {}
    for op in ops:
        nm = op["name"]
        if nm in _LOSS_NAMES:
            continue
        if nm in by_name:
            exact[by_name[nm]] = op
            continue
        base = nm.rstrip("0123456789")
        t = _TYPE_NAMES.get(base.lower().rstrip("_"))
        if t is None:
            raise ValueError(f"strategy record '{nm}' matches no layer and no operator type")
        cands = by_type.get(t, [])
        if base != nm:
            i = int(nm[len(base):])
            if i >= len(cands):
                raise ValueError(f"strategy record '{nm}': the model has only {len(cands)} {t} layers")
            indexed[cands[i]] = op
        else:
            for n in cands:
                generic[n] = op
    out = dict(generic)
    out.update(indexed)
    out.update(exact)
    return out


def _view(op: dict, world: int, name: str) -> Optional[Tuple[int, ...]]:
    """The record's device ids as a placement (partition order = the task
    order: the innermost dim varies fastest in both); None = every rank."""
    ids = [int(d) for d in op.get("device_ids", ())]
    if not ids:
        return None
    if max(ids) >= world or min(ids) < 0:
        raise ValueError(f"strategy record '{name}' uses device {max(ids)} but only {world} ranks run")
    if len(set(ids)) != len(ids):
        raise ValueError(f"strategy record '{name}': devices {ids} repeat")
    if ids == list(range(world)):
        return None
    return tuple(ids)


def task_devices(view, total: int) -> List[int]:
    """``total`` device ids of a placement in task order (one per partition;
    implicit replicas dropped), every rank's first ``total`` when None."""
    if view is None:
        return list(range(total))
    devs = list(view)
    reps = max(1, len(devs) // max(1, total))
    return devs[::reps][:total]


def to_pcg(cg, ops: List[dict], world: int):
    """Lower a legacy strategy onto ``cg`` for ``world`` ranks: (pcg, views, report)."""
    strat = json.loads(C.data_parallel_strategy(cg, world))
    recs = _records_for_layers(cg, ops)
    name_of = {n: cg.layer_name(n) for n in cg.topo_order()}
    key_of = {}
    for n in recs:
        key = name_of[n] if name_of[n] in strat else str(n)
        if key not in strat:
            raise ValueError(f"layer {name_of[n]!r} has no strategy entry")
        key_of[n] = key
    views_cg: Dict[int, Tuple[int, ...]] = {}
    for n, op in recs.items():
        dims = [int(d) for d in op.get("dims", ())] or [1]
        sample = dims[-1]
        channel = dims[0] if len(dims) >= 2 else 1
        total = 1
        for d in dims:
            total *= d
        if op.get("device_ids") and len(op["device_ids"]) != total:
            raise ValueError(f"strategy record '{op['name']}': {len(op['device_ids'])} devices for degrees {dims}")
        t = cg.layer_op(n).op_type
        cfg = {"batch": sample, "seq": 1, "model": 1, "kind": "none"}
        if channel > 1:
            if t not in ("LINEAR", "EMBEDDING", "CONV2D"):
                raise ValueError(f"strategy record '{op['name']}': channel degree {channel} on a {t} layer")
            cfg.update(model=channel, kind="column")
        strat[key_of[n]] = cfg
        v = _view(op, world, op["name"])
        if v is not None:
            views_cg[n] = v
    pcg, cg_to_pcg, _ = C.lower_strategy(cg, json.dumps(strat), world)
    views = {int(cg_to_pcg[n]): v for n, v in views_cg.items() if n in cg_to_pcg}
    report = {"source": "import:legacy-pb", "records": len(ops), "matched_layers": len(recs),
              "zero_copy_records": sum(1 for o in ops if "ZCM" in o.get("memory_types", ()))}
    return pcg, views, report


def from_pcg(pcg, views: Dict[int, Tuple[int, ...]]) -> List[dict]:
    """Per-op legacy records of a lowered strategy (dims innermost-first)."""
    ops = []
    for n in pcg.topo_order():
        op = pcg.layer_op(n)
        if op.op_type in ("INPUT", "WEIGHT") or pcg.is_weight_path(n) or C.is_parallel_op(op.type):
            continue
        ps = pcg.shape(C.ValueRef(n, 0))
        deg = list(ps.shard_degrees())
        total = ps.total_parallel_degree()
        ops.append({"name": pcg.layer_name(n) or f"{op.op_type.lower()}{n}", "device_type": "GPU",
                    "dims": list(reversed(deg)), "device_ids": task_devices(views.get(n), total),
                    "memory_types": []})
    return ops
