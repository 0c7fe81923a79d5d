"""Distributed context and the layout-redistribution engine (RCCL over xGMI).

One process per GPU (torchrun-style env: RANK / WORLD_SIZE / LOCAL_RANK /
MASTER_ADDR / MASTER_PORT); torch.distributed's "nccl" backend is RCCL on
ROCm; "gloo" serves the CPU tests.

``redistribute(x, src, dst)`` moves a tensor between two layouts of the same
logical shape.  Every rank computes the same global plan (deterministic), so
sub-communicators can be created collectively up front.  The plan is lowered
to the cheapest primitive that implements it:

  * local slice / copy (no communication) — Replicate after a Reduction,
    Repartition of a replicated tensor, matching views;
  * all_reduce over a group — Reduction (sum of partials), the backward of
    Replicate (sum of copy gradients);
  * all_gather over a group — Combine;
  * one all_to_all_single with per-rank split sizes — any other view change
    (resharding to a different dim, DLRM table-sharded -> batch-sharded
    embeddings, different machine views); each (receiver, sender) pair moves
    at most one box, zero-size splits for pairs that exchange nothing;
  * matched send / recv pairs — a pipeline-stage boundary (each receiver
    fed by one rank of the previous stage, no rank on both sides);
  * batched point-to-point (isend/irecv of the intersecting boxes) — the
    fallback (``FF_REDIST_P2P=1``).

Parity: replaces Legion region copies + the NCCL weight-sync-only path of the
reference (lib/runtime/src/legion_backing.cc:173-257, optimizer_kernel.cu:83);
SURVEY §2.8 "MI355X-native equivalent".
"""
from __future__ import annotations

import dataclasses
import math
import os
from typing import Any, Dict, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

from ..runtime.graphs import check_capturable
from .layout import Box, Layout, intersect, rel_slices


class DistContext:
    """Process-group bookkeeping for one rank."""

    def __init__(self, rank: int = 0, world: int = 1, device: Optional[torch.device] = None,
                 force_collectives: bool = False):
        self.rank = rank
        self.world = world
        self.device = device or torch.device("cpu")
        # FF_DIST_WORLD1=1: a one-rank process group whose collectives are
        # still issued (single-member groups included), so the whole RCCL
        # path -- communicator creation, bucketed gradient all-reduce /
        # reduce-scatter / all-gather, all-to-all redistribution and the
        # graph segments cut at every collective -- runs on a single GPU
        self.force_collectives = force_collectives
        self._groups: Dict[Tuple[int, ...], object] = {}
        self.stats = {"all_reduce": 0, "all_gather": 0, "all_to_all": 0, "p2p": 0, "local": 0, "bytes": 0}
        self.msg_sizes: Dict[str, set] = {}
        # runtime/graphs.SegmentRecorder while a distributed step is being
        # captured: in-place collectives become segment boundaries
        self.recorder = None

    def _issue(self, fn, async_op: bool, desc=None):
        if self.recorder is not None:
            return self.recorder.collective(fn, async_op, desc)
        return fn()

    @staticmethod
    def _pg(grp):
        """The c10d ProcessGroup object behind ``grp`` (None = the default group)."""
        if grp is not None:
            return grp
        from torch.distributed import distributed_c10d
        return distributed_c10d._get_default_group()

    @staticmethod
    def _group_rank(grp, rank: int) -> int:
        return rank if grp is None else dist.get_group_rank(grp, rank)

    @classmethod
    def from_env(cls, device: Optional[torch.device] = None, backend: Optional[str] = None) -> "DistContext":
        world = int(os.environ.get("WORLD_SIZE", "1"))
        rank = int(os.environ.get("RANK", "0"))
        force = os.environ.get("FF_DIST_WORLD1", "0") == "1"
        if (world > 1 or force) and not dist.is_initialized():
            if world == 1:
                os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
                os.environ.setdefault("MASTER_PORT", str(_free_port()))
                os.environ.setdefault("RANK", "0")
                os.environ.setdefault("WORLD_SIZE", "1")
            backend = backend or os.environ.get("FF_DIST_BACKEND") or None
            if backend is None:
                backend = "nccl" if (device is not None and device.type == "cuda") else "gloo"
            kw = {}
            if backend == "nccl" and device is not None:
                kw["device_id"] = device
            # a hung collective (a failed / stalled rank) fails after this many
            # seconds instead of blocking forever, so an elastic launcher
            # (torchrun --max-restarts) can restart the job from its last
            # checkpoint (FFConfig.checkpoint_dir)
            tmo = os.environ.get("FF_DIST_TIMEOUT_S")
            if tmo:
                import datetime
                kw["timeout"] = datetime.timedelta(seconds=float(tmo))
            dist.init_process_group(backend=backend, **kw)
        if dist.is_initialized():
            rank, world = dist.get_rank(), dist.get_world_size()
        return cls(rank, world, device, force_collectives=force and dist.is_initialized())

    @property
    def distributed(self) -> bool:
        return (self.world > 1 or self.force_collectives) and dist.is_initialized()

    @property
    def backend(self) -> str:
        return str(dist.get_backend()) if dist.is_initialized() else "none"

    def syncs(self, ranks: Sequence[int]) -> bool:
        """True when a collective over ``ranks`` is actually issued."""
        return self.distributed and (len(ranks) > 1 or (self.force_collectives and len(ranks) == 1))

    def group(self, ranks: Sequence[int]):
        """Sub-communicator for ``ranks``; MUST be called in the same order on
        every rank (plans are built identically everywhere)."""
        key = tuple(sorted(ranks))
        if len(key) == self.world:
            return None  # default group
        if key not in self._groups:
            self._groups[key] = dist.new_group(list(key))
        return self._groups[key]

    def barrier(self):
        if self.distributed:
            dist.barrier()

    def all_reduce_(self, t: torch.Tensor, ranks: Sequence[int], async_op: bool = False):
        if not self.syncs(ranks):
            return None
        self.note_size("all_reduce", t.numel() * t.element_size())
        self.stats["all_reduce"] += 1
        self.stats["bytes"] += t.numel() * t.element_size()
        grp = self.group(ranks)
        return self._issue(lambda: dist.all_reduce(t, group=grp, async_op=async_op), async_op,
                           ("all_reduce", t, None, self._pg(grp), 0))

    def reduce_scatter_(self, t: torch.Tensor, ranks: Sequence[int], async_op: bool = False):
        """In-place reduce-scatter of the 1-D ``t``: afterwards chunk i (of
        len(ranks) equal chunks) on the i-th rank of sorted(ranks) holds the
        sum.  RCCL runs it in place (output = input + rank * chunk); gloo has
        no reduce-scatter, so the CPU path all-reduces (a superset)."""
        if not self.syncs(ranks):
            return None
        self.stats["reduce_scatter"] = self.stats.get("reduce_scatter", 0) + 1
        self.stats["bytes"] += t.numel() * t.element_size()
        if t.is_cuda:
            n = len(ranks)
            i = sorted(ranks).index(self.rank)
            chunk = t.numel() // n
            grp = self.group(ranks)
            out = t[i * chunk:(i + 1) * chunk]
            return self._issue(lambda: dist.reduce_scatter_tensor(out, t, group=grp, async_op=async_op), async_op,
                               ("reduce_scatter", t, out, self._pg(grp), 0))
        return dist.all_reduce(t, group=self.group(ranks), async_op=async_op)

    def reduce_(self, t: torch.Tensor, ranks: Sequence[int], dst: int, async_op: bool = False):
        """Sum ``t`` over ``ranks`` into rank ``dst`` (parameter-server gradient
        gather, the reference's ParamSync::PS, optimizer_kernel.cu:43-70)."""
        if not self.syncs(ranks):
            return None
        self.stats["reduce"] = self.stats.get("reduce", 0) + 1
        self.stats["bytes"] += t.numel() * t.element_size()
        grp = self.group(ranks)
        return self._issue(lambda: dist.reduce(t, dst=dst, group=grp, async_op=async_op), async_op,
                           ("reduce", t, None, self._pg(grp), self._group_rank(grp, dst)))

    def broadcast_(self, t: torch.Tensor, ranks: Sequence[int], src: int, async_op: bool = False):
        if not self.syncs(ranks):
            return None
        self.stats["broadcast"] = self.stats.get("broadcast", 0) + 1
        self.stats["bytes"] += t.numel() * t.element_size()
        grp = self.group(ranks)
        return self._issue(lambda: dist.broadcast(t, src=src, group=grp, async_op=async_op), async_op,
                           ("broadcast", t, None, self._pg(grp), self._group_rank(grp, src)))

    def all_gather_(self, t: torch.Tensor, ranks: Sequence[int]):
        """In-place all-gather of the equal chunks of the 1-D ``t`` (chunk i
        comes from the i-th rank of sorted(ranks))."""
        if not self.syncs(ranks):
            return
        n = len(ranks)
        i = sorted(ranks).index(self.rank)
        chunk = t.numel() // n
        self.stats["all_gather"] += 1
        self.stats["bytes"] += t.numel() * t.element_size()
        if t.is_cuda:
            grp = self.group(ranks)
            piece = t[i * chunk:(i + 1) * chunk]
            self._issue(lambda: dist.all_gather_into_tensor(t, piece, group=grp), False,
                        ("all_gather", piece, t, self._pg(grp), 0))
        else:
            dist.all_gather(list(t.split(chunk)), t[i * chunk:(i + 1) * chunk].clone(), group=self.group(ranks))

    def note_size(self, kind: str, nbytes: int):
        """Message sizes the step issues, per collective kind (the collective
        cost model is calibrated at these sizes: parallel/calibrate.py)."""
        s = self.msg_sizes.setdefault(kind, set())
        if len(s) < 64:
            s.add(int(nbytes))

    def max_scalar(self, v: float) -> float:
        if not self.distributed:
            return v
        check_capturable("max_scalar")
        t = torch.tensor([v], dtype=torch.float64, device=self.device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())


def _free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


# ---------------------------------------------------------------------------
@dataclasses.dataclass
class Contribution:
    src_rank: int
    src_box: Box      # box of the source piece
    part: Box         # intersection (global coordinates)


@dataclasses.dataclass
class Plan:
    kind: str                                   # local | all_reduce | all_gather | all_to_all | p2p
    contributions: Dict[int, List[Contribution]]
    dst_boxes: Dict[int, Optional[Box]]
    src_boxes: Dict[int, Optional[Box]]
    groups: List[Tuple[int, ...]]
    gather_dim: int = -1
    # per-device index tensors of deduplicated all_gather pieces, built once
    # (an upload per step would be a pageable copy inside graph capture)
    index_cache: Dict[Any, torch.Tensor] = dataclasses.field(default_factory=dict, compare=False, repr=False)


def _summed_sources(src: Layout, dst: Layout, s_d: int) -> List[int]:
    Ss, Sd = src.sum_degree, dst.sum_degree
    if Ss == Sd:
        return [s_d]
    if Ss % Sd == 0:
        k = Ss // Sd
        return [s_d * k + j for j in range(k)]
    if Sd % Ss == 0:
        k = Sd // Ss
        return [s_d // k] if s_d % k == 0 else []
    raise ValueError(f"incompatible summed degrees {Ss} -> {Sd}")


def make_plan(src: Layout, dst: Layout, world: int) -> Plan:
    if src.sizes != dst.sizes:
        raise ValueError(f"redistribute: logical shapes differ {src.sizes} vs {dst.sizes}")
    contributions: Dict[int, List[Contribution]] = {}
    dst_boxes: Dict[int, Optional[Box]] = {}
    src_boxes: Dict[int, Optional[Box]] = {}
    for r in range(world):
        cs = src.coord(r)
        src_boxes[r] = src.box(cs.shard) if cs is not None else None
        cd = dst.coord(r)
        if cd is None:
            dst_boxes[r] = None
            continue
        bd = dst.box(cd.shard)
        dst_boxes[r] = bd
        contribs = []
        for s_s in _summed_sources(src, dst, dst.summed_index(cd)):
            for shard in src.shards():
                bs = src.box(shard)
                part = intersect(bs, bd)
                if part is None:
                    continue
                holders = src.holders(shard, s_s)
                if r in holders:
                    choice = r
                else:
                    # spread readers over holders deterministically
                    choice = holders[(r + cd.rep) % len(holders)]
                contribs.append(Contribution(choice, bs, part))
        contributions[r] = contribs

    # ---- classify
    all_local = all(all(c.src_rank == r for c in cl) and len(cl) <= 1 for r, cl in contributions.items())
    if all_local:
        return Plan("local", contributions, dst_boxes, src_boxes, [])
    # all_reduce: each rank's contributions are full-box copies from a group containing itself
    groups = []
    ok = True
    for r, cl in contributions.items():
        g = tuple(sorted(c.src_rank for c in cl))
        if r not in g or len(set(g)) != len(g):
            ok = False
            break
        if any(c.part != dst_boxes[r] or c.src_box != dst_boxes[r] for c in cl):
            ok = False
            break
        for m in g:
            cm = contributions.get(m)
            if cm is None or tuple(sorted(c.src_rank for c in cm)) != g or dst_boxes[m] != dst_boxes[r]:
                ok = False
                break
        if not ok:
            break
        if g not in groups:
            groups.append(g)
    if ok and src.sum_degree > dst.sum_degree:
        return Plan("all_reduce", contributions, dst_boxes, src_boxes, groups)
    # reduce_scatter: the partial-sum replicas of one box, each member keeping
    # an equal slice of the sum along one dim (a row-parallel output going to a
    # sharded consumer): one reduce_scatter_tensor over the group instead of an
    # all_to_all of the partial slices plus a local sum
    if src.sum_degree > dst.sum_degree:
        rs = _reduce_scatter_groups(contributions, dst_boxes)
        if rs is not None:
            return Plan("reduce_scatter", contributions, dst_boxes, src_boxes, rs[0], gather_dim=rs[1])
    # all_gather: each rank assembles its dst box from its group's own pieces
    groups = []
    ok = src.sum_degree == dst.sum_degree
    gdim = -1
    if ok:
        for r, cl in contributions.items():
            g = tuple(sorted(c.src_rank for c in cl))
            if r not in g or len(set(g)) != len(g) or len(g) < 2:
                ok = False
                break
            for c in cl:
                if c.part != c.src_box or c.src_box != src_boxes[c.src_rank]:
                    ok = False
                    break
                diff = [i for i, ((l1, h1), (l2, h2)) in enumerate(zip(c.src_box, dst_boxes[r])) if (l1, h1) != (l2, h2)]
                if len(diff) != 1 or (gdim != -1 and diff[0] != gdim):
                    ok = False
                    break
                gdim = diff[0]
            if not ok:
                break
            for m in g:
                cm = contributions.get(m)
                if cm is None or tuple(sorted(c.src_rank for c in cm)) != g or dst_boxes[m] != dst_boxes[r]:
                    ok = False
                    break
            if not ok:
                break
            if g not in groups:
                groups.append(g)
    if ok and gdim >= 0:
        return Plan("all_gather", contributions, dst_boxes, src_boxes, groups, gather_dim=gdim)
    # general resharding (e.g. DLRM's table-sharded embeddings -> batch-sharded
    # MLP input): every (receiver, sender) pair moves at most one box, so the
    # whole exchange is ONE all_to_all with per-rank split sizes (RCCL spreads
    # it over all xGMI links at once) instead of a batch of point-to-point ops
    pairs = [(r, c.src_rank) for r, cl in contributions.items() for c in cl]
    # only the ranks that send or receive take part (a pipeline-stage boundary
    # involves the two stages' ranks, not the world)
    involved = tuple(sorted({r for r, _ in pairs if any(c.src_rank != r for c in contributions[r])} |
                            {m for r, m in pairs if m != r}))
    sub = [involved] if 1 < len(involved) < world else []
    # a pipeline-stage boundary: every receiver takes its box from at most one
    # other rank, every sender feeds at most one, and no rank does both ->
    # matched send / recv pairs (one xGMI link each), not an all_to_all that
    # rendezvouses both stages' ranks
    remote = [(r, m) for r, m in pairs if r != m]
    senders = [m for _, m in remote]
    receivers = [r for r, _ in remote]
    if (remote and len(set(senders)) == len(senders) and len(set(receivers)) == len(receivers)
            and not set(senders) & set(receivers) and os.environ.get("FF_REDIST_SENDRECV", "1") == "1"
            and os.environ.get("FF_REDIST_P2P", "0") != "1"):
        # (the sub-group serves the all_to_all form of the same exchange: gloo
        # moves device tensors only through collectives)
        return Plan("send_recv", contributions, dst_boxes, src_boxes, sub)
    if len(pairs) == len(set(pairs)) and os.environ.get("FF_REDIST_P2P", "0") != "1":
        return Plan("all_to_all", contributions, dst_boxes, src_boxes, sub)
    return Plan("p2p", contributions, dst_boxes, src_boxes, [])


def _reduce_scatter_groups(contributions, dst_boxes):
    """(groups, dim) when every rank's destination box is its equal slice,
    along one dim, of one source box whose partial sums its group's members
    hold (the members being exactly the ranks that receive the slices), with
    the slices in the members' rank order; else None."""
    groups: List[Tuple[int, ...]] = []
    rdim = -1
    for r, cl in contributions.items():
        if not cl:
            return None
        g = tuple(sorted(c.src_rank for c in cl))
        b0 = cl[0].src_box
        if r not in g or len(set(g)) != len(g) or len(g) < 2:
            return None
        if any(c.src_box != b0 or c.part != dst_boxes[r] for c in cl):
            return None
        boxes = []
        for m in g:
            cm = contributions.get(m)
            if (cm is None or dst_boxes.get(m) is None or tuple(sorted(c.src_rank for c in cm)) != g
                    or any(c.src_box != b0 for c in cm)):
                return None
            boxes.append(dst_boxes[m])
        diffs = {i for b in boxes for i, (x, y) in enumerate(zip(b, b0)) if x != y}
        if len(diffs) != 1:
            return None
        d = diffs.pop()
        if rdim not in (-1, d):
            return None
        rdim = d
        starts = [b[d][0] for b in boxes]
        sizes = [b[d][1] - b[d][0] for b in boxes]
        # equal slices, tiling the source box in the members' (sorted) order
        if len(set(sizes)) != 1 or starts != sorted(starts) or starts[0] != b0[d][0] \
                or starts[-1] + sizes[-1] != b0[d][1] or len(set(starts)) != len(starts):
            return None
        if g not in groups:
            groups.append(g)
    return (groups, rdim) if rdim >= 0 else None


def execute_plan(plan: Plan, x: Optional[torch.Tensor], ctx: DistContext, dst_shape: Sequence[int],
                 dtype: torch.dtype, device: torch.device) -> Optional[torch.Tensor]:
    me = ctx.rank
    my_dst = plan.dst_boxes.get(me)
    my_src = plan.src_boxes.get(me)
    if plan.kind == "local":
        ctx.stats["local"] += 1
        if my_dst is None:
            return None
        cl = plan.contributions[me]
        if not cl:
            return torch.zeros(dst_shape, dtype=dtype, device=device)
        c = cl[0]
        if c.part == my_src:
            return x
        return x[rel_slices(c.part, my_src)].contiguous()
    if plan.kind in ("all_reduce", "reduce_scatter", "all_gather") and not any(me in g for g in plan.groups):
        return None   # these plans' groups are exactly the receivers: nothing to send or receive here
    if plan.kind == "all_reduce":
        y = x.clone()
        g = next(g for g in plan.groups if me in g)
        ctx.all_reduce_(y, g)
        return y
    if plan.kind == "reduce_scatter":
        g = next(g for g in plan.groups if me in g)
        ctx.stats["reduce_scatter"] = ctx.stats.get("reduce_scatter", 0) + 1
        d = plan.gather_dim
        n = len(g)
        # chunk i of the flat input = member g[i]'s slice (g is sorted and the
        # slices follow it along d): contiguous as it stands when d is the
        # outermost dim with a non-trivial extent, one packing copy otherwise
        xs = x.contiguous()
        if all(xs.shape[i] == 1 for i in range(d)):
            inp = xs.reshape(-1)
        else:
            inp = torch.stack(xs.chunk(n, dim=d)).reshape(-1)
        out = torch.empty(dst_shape, dtype=xs.dtype, device=xs.device)
        grp = ctx.group(g)
        ctx.note_size("reduce_scatter", inp.numel() * inp.element_size())
        ctx._issue(lambda: dist.reduce_scatter_tensor(out.view(-1), inp, group=grp), False,
                   ("reduce_scatter", inp, out.view(-1), ctx._pg(grp), 0))
        return out.to(dtype)
    if plan.kind == "all_gather":
        g = next(g for g in plan.groups if me in g)
        ctx.stats["all_gather"] += 1
        xs = x.contiguous()
        n = len(g)
        grp = ctx.group(g)
        # one all_gather_into_tensor into [n, *piece] (member order = sorted
        # ranks), then the members' pieces in box order along the gather dim:
        # a view when the pieces already follow that order on the outermost
        # dim, one copy (movedim + reshape) otherwise -- no list + cat
        flat = torch.empty((n,) + tuple(xs.shape), dtype=xs.dtype, device=xs.device)
        ctx.note_size("all_gather", flat.numel() * flat.element_size())
        ctx._issue(lambda: dist.all_gather_into_tensor(flat.view(-1), xs.view(-1), group=grp), False,
                   ("all_gather", xs.view(-1), flat.view(-1), ctx._pg(grp), 0))
        order = sorted(range(n), key=lambda i: plan.src_boxes[g[i]][plan.gather_dim][0])
        # members holding identical boxes (implicit replicas) appear once
        seen, keep = set(), []
        for i in order:
            b = plan.src_boxes[g[i]]
            if b in seen:
                continue
            seen.add(b)
            keep.append(i)
        d = plan.gather_dim
        if keep == list(range(n)):
            sel = flat
        elif keep == list(range(keep[0], keep[0] + len(keep))):
            sel = flat.narrow(0, keep[0], len(keep))
        else:
            key = (str(flat.device), tuple(keep))
            idx = plan.index_cache.get(key)
            if idx is None:
                idx = plan.index_cache[key] = torch.tensor(keep, device=flat.device)
            sel = flat[idx]
        if all(xs.shape[i] == 1 for i in range(d)):
            return sel.reshape(tuple(xs.shape[:d]) + (len(keep) * xs.shape[d],) + tuple(xs.shape[d + 1:]))
        return sel.movedim(0, d).reshape(tuple(xs.shape[:d]) + (len(keep) * xs.shape[d],) + tuple(xs.shape[d + 1:]))
    if plan.kind == "all_to_all":
        return _exchange_all_to_all(plan, x, ctx, dst_shape, dtype, device)
    if plan.kind == "send_recv":
        return _exchange_send_recv(plan, x, ctx, dst_shape, dtype, device)
    # ---- generic point-to-point
    ctx.stats["p2p"] += 1
    ops = []
    recv_bufs = []
    for r, cl in plan.contributions.items():
        for c in cl:
            if c.src_rank == me and r != me:
                piece = x[rel_slices(c.part, my_src)].contiguous()
                ops.append(dist.P2POp(dist.isend, piece, r))
    result = None
    if my_dst is not None:
        result = torch.zeros(dst_shape, dtype=dtype, device=device)
        for c in plan.contributions[me]:
            if c.src_rank == me:
                result[rel_slices(c.part, my_dst)] += x[rel_slices(c.part, my_src)]
            else:
                buf = torch.empty([h - l for l, h in c.part], dtype=dtype, device=device)
                ops.append(dist.P2POp(dist.irecv, buf, c.src_rank))
                recv_bufs.append((c, buf))
    if ops:
        def _p2p():
            for w in dist.batch_isend_irecv(ops):
                w.wait()
        ctx._issue(_p2p, False)
    for c, buf in recv_bufs:
        result[rel_slices(c.part, my_dst)] += buf
    return result


def _exchange_all_to_all(plan: Plan, x: Optional[torch.Tensor], ctx: DistContext, dst_shape: Sequence[int],
                         dtype: torch.dtype, device: torch.device) -> Optional[torch.Tensor]:
    me, world = ctx.rank, ctx.world
    my_dst, my_src = plan.dst_boxes.get(me), plan.src_boxes.get(me)
    ctx.stats["all_to_all"] += 1
    send = [None] * world
    for r in range(world):
        for c in plan.contributions.get(r) or ():
            if c.src_rank == me:
                send[r] = x[rel_slices(c.part, my_src)].reshape(-1)
    recv_c = [None] * world
    if my_dst is not None:
        for c in plan.contributions[me]:
            recv_c[c.src_rank] = c
    in_sizes = [0 if p is None else p.numel() for p in send]
    out_sizes = [0 if c is None else math.prod(h - l for l, h in c.part) for c in recv_c]
    parts = [p for p in send if p is not None and p.numel()]
    sendbuf = torch.cat(parts) if parts else torch.empty(0, dtype=dtype, device=device)
    recvbuf = torch.empty(sum(out_sizes), dtype=sendbuf.dtype, device=device)
    sendbuf = sendbuf.to(device)
    if plan.groups:
        # a sub-group exchange (pipeline-stage boundary): ranks outside it take
        # no part; members address each other by group rank (sorted order)
        g = plan.groups[0]
        if me not in g:
            # outside the exchange: any destination box this rank has is served
            # entirely from its own source piece (a rank that received from
            # another would be a member)
            if my_dst is None:
                return None
            result = torch.zeros(dst_shape, dtype=dtype, device=device)
            for c in plan.contributions[me]:
                assert c.src_rank == me, "non-member of a sub-group all_to_all receives from another rank"
                result[rel_slices(c.part, my_dst)] += x[rel_slices(c.part, my_src)].to(dtype)
            return result
        grp = ctx.group(g)
        gi = [in_sizes[m] for m in g]
        go = [out_sizes[m] for m in g]
        ctx.stats["all_to_all_subgroup"] = ctx.stats.get("all_to_all_subgroup", 0) + 1
        ctx.note_size("all_to_all", sendbuf.numel() * sendbuf.element_size())
        ctx._issue(lambda: dist.all_to_all_single(recvbuf, sendbuf, output_split_sizes=go, input_split_sizes=gi,
                                                  group=grp), False,
                   ("all_to_all", sendbuf, recvbuf, ctx._pg(grp), 0, list(go), list(gi)))
    else:
        ctx.note_size("all_to_all", sendbuf.numel() * sendbuf.element_size())
        ctx._issue(lambda: dist.all_to_all_single(recvbuf, sendbuf, output_split_sizes=out_sizes,
                                                  input_split_sizes=in_sizes), False,
                   ("all_to_all", sendbuf, recvbuf, ctx._pg(None), 0, list(out_sizes), list(in_sizes)))
    if my_dst is None:
        return None
    result = torch.zeros(dst_shape, dtype=dtype, device=device)
    off = 0
    for m in range(world):
        c = recv_c[m]
        if c is None:
            continue
        n = out_sizes[m]
        result[rel_slices(c.part, my_dst)] += recvbuf[off:off + n].view([h - l for l, h in c.part]).to(dtype)
        off += n
    return result


def _exchange_send_recv(plan: Plan, x: Optional[torch.Tensor], ctx: DistContext, dst_shape: Sequence[int],
                        dtype: torch.dtype, device: torch.device) -> Optional[torch.Tensor]:
    """Matched point-to-point pairs (a pipeline-stage boundary): each sender
    isends its one piece, each receiver irecvs its one piece, batched into one
    coalesced group; ranks outside the pairs only copy their own pieces."""
    if device.type == "cuda" and ctx.backend != "nccl":
        # gloo point-to-point takes host tensors only: the same boxes through
        # the (sub-group) all_to_all
        return _exchange_all_to_all(plan, x, ctx, dst_shape, dtype, device)
    me = ctx.rank
    my_dst, my_src = plan.dst_boxes.get(me), plan.src_boxes.get(me)
    ctx.stats["send_recv"] = ctx.stats.get("send_recv", 0) + 1
    sends, recvs = [], []
    for r, cl in plan.contributions.items():
        for c in cl:
            if c.src_rank == me and r != me:
                sends.append((r, x[rel_slices(c.part, my_src)].contiguous()))
    result = None
    if my_dst is not None:
        result = torch.zeros(dst_shape, dtype=dtype, device=device)
        for c in plan.contributions[me]:
            if c.src_rank == me:
                result[rel_slices(c.part, my_dst)] += x[rel_slices(c.part, my_src)].to(dtype)
            else:
                buf = torch.empty([h - l for l, h in c.part], dtype=dtype, device=device)
                recvs.append((c.src_rank, buf, c))
    if sends or recvs:
        for _, t in sends:
            ctx.note_size("send_recv", t.numel() * t.element_size())
        ops = [dist.P2POp(dist.isend, t, peer) for peer, t in sends] + \
              [dist.P2POp(dist.irecv, b, peer) for peer, b, _ in recvs]

        def _pairs():
            for w in dist.batch_isend_irecv(ops):
                w.wait()
        ctx._issue(_pairs, False, ("send_recv", [(p, t) for p, t in sends], [(p, b) for p, b, _ in recvs],
                                    ctx._pg(None), 0))
    for _, buf, c in recvs:
        result[rel_slices(c.part, my_dst)] += buf
    return result


class Redistributor:
    """Caches plans and creates every sub-communicator they need up front."""

    def __init__(self, ctx: DistContext):
        self.ctx = ctx
        self._plans: Dict[Tuple[Layout, Layout], Plan] = {}

    def plan(self, src: Layout, dst: Layout) -> Plan:
        key = (src, dst)
        if key not in self._plans:
            p = make_plan(src, dst, self.ctx.world)
            for g in p.groups:
                if self.ctx.distributed:
                    self.ctx.group(g)
            self._plans[key] = p
        return self._plans[key]

    def __call__(self, x: Optional[torch.Tensor], src: Layout, dst: Layout, dtype: torch.dtype,
                 device: torch.device) -> Optional[torch.Tensor]:
        p = self.plan(src, dst)
        if p.kind != "local" and not self.ctx.distributed:
            raise RuntimeError(f"redistribution {p.kind} needs torch.distributed (world={self.ctx.world})")
        return execute_plan(p, x, self.ctx, dst.piece_shape, dtype, device)
