"""Parallel tensor layouts over the world of ranks (one process per GPU).

A ``Layout`` places the pieces of a ParallelTensorShape on ranks:

* shard degrees per dim (``degrees``) — each piece is a box of the tensor;
* axis ``a`` = the forward partial-sum axis (sum_degree), axis ``b`` = the
  forward discard-copy axis (discard_copy_degree);
* ``reps`` = implicit redundant replicas when the total degree T is smaller
  than the device block (the same piece computed redundantly).

Placement (the MachineView of the op that produces the tensor): a device
list (``devices``; the contiguous block ``[start, start + block)`` when it is
None); entry ``lin*reps + rep`` of it holds task coordinate
``unravel(lin, degrees + [a, b])`` (row-major, copy axis innermost, implicit
replicas innermost of all).  Device lists come from the machine-mapping DP's
MachineViews (strided views included: ``get_device_ids`` lists a view's
devices in exactly this task order).  With this canonical
placement the Unity/Megatron patterns line up without data movement:
DP x TP puts TP groups on consecutive ranks, Replicate after Reduction is a
no-op, a column-parallel Linear's output shard lives where its input copy
lives.  (Reference counterpart: MachineView + get_machine_space_coordinate,
lib/pcg/src/pcg/machine_view.cc:45-113, and FFMapper::slice_task,
lib/runtime/src/mapper.cc:335-430.)

``summed`` selects which of a / b is summed: forward layouts sum axis a
(partials) and treat b as identical copies; gradients flow on the DUAL
layout (a identical, b summed), because d/d(partial) of a sum is the same
for every partial, while gradients of identical copies add up.
"""
from __future__ import annotations

import dataclasses
import math
from typing import List, Optional, Sequence, Tuple

Box = Tuple[Tuple[int, int], ...]


@dataclasses.dataclass(frozen=True)
class Coord:
    shard: Tuple[int, ...]
    a: int
    b: int
    rep: int


@dataclasses.dataclass(frozen=True)
class Layout:
    sizes: Tuple[int, ...]
    degrees: Tuple[int, ...]
    a_deg: int = 1
    b_deg: int = 1
    block: int = 1          # number of ranks in the device block
    start: int = 0          # first rank of the block
    summed: str = "a"       # which of a / b is summed ("a": forward, "b": gradient)
    # Parameters place their copy axis OUTERMOST: a weight's copies follow
    # the consumer's outer (batch / sequence) task dims while its shards
    # follow the consumer's inner copy / last-dim axes, so DP x TP puts a
    # TP group's weight shards on consecutive ranks, exactly where the
    # matching activation pieces live.
    copy_outer: bool = False
    # explicit placement (device per entry); None: [start, start + block)
    devices: Optional[Tuple[int, ...]] = None

    def __post_init__(self):
        if self.devices is not None:
            devs = tuple(int(d) for d in self.devices)
            object.__setattr__(self, "devices", devs)
            object.__setattr__(self, "block", len(devs))
            object.__setattr__(self, "start", devs[0] if devs else 0)
            if len(set(devs)) != len(devs):
                raise ValueError(f"layout: placement repeats a device {devs}")
        if len(self.sizes) != len(self.degrees):
            raise ValueError("layout: rank mismatch")
        for s, d in zip(self.sizes, self.degrees):
            if d < 1 or s % d:
                raise ValueError(f"layout: size {s} not divisible by degree {d}")
        if self.block % self.total:
            raise ValueError(f"layout: total degree {self.total} does not divide device block {self.block}")

    # ---- basic properties
    @property
    def total(self) -> int:
        return math.prod(self.degrees) * self.a_deg * self.b_deg

    @property
    def reps(self) -> int:
        return self.block // self.total

    @property
    def piece_shape(self) -> Tuple[int, ...]:
        return tuple(s // d for s, d in zip(self.sizes, self.degrees))

    @property
    def sum_degree(self) -> int:
        return self.a_deg if self.summed == "a" else self.b_deg

    @property
    def same_degree(self) -> int:
        return self.b_deg if self.summed == "a" else self.a_deg

    def dual(self) -> "Layout":
        return dataclasses.replace(self, summed="b" if self.summed == "a" else "a")

    def with_block(self, block: int, start: int = 0) -> "Layout":
        return dataclasses.replace(self, block=block, start=start, devices=None)

    def with_devices(self, devices: Sequence[int]) -> "Layout":
        return dataclasses.replace(self, devices=tuple(devices))

    # ---- placement
    def _index(self, rank: int) -> int:
        if self.devices is None:
            return rank - self.start
        try:
            return self.devices.index(rank)
        except ValueError:
            return -1

    def coord(self, rank: int) -> Optional[Coord]:
        idx = self._index(rank)
        if idx < 0 or idx >= self.block:
            return None
        lin, rep = divmod(idx, self.reps)
        dims = self._dims()
        c = []
        for d in reversed(dims):
            lin, r = divmod(lin, d)
            c.append(r)
        c.reverse()
        if self.copy_outer:
            return Coord(tuple(c[1:-1]), c[-1], c[0], rep)
        return Coord(tuple(c[:-2]), c[-2], c[-1], rep)

    def _dims(self) -> List[int]:
        if self.copy_outer:
            return [self.b_deg] + list(self.degrees) + [self.a_deg]
        return list(self.degrees) + [self.a_deg, self.b_deg]

    def rank_of(self, coord: Coord) -> int:
        dims = self._dims()
        if self.copy_outer:
            vals = [coord.b] + list(coord.shard) + [coord.a]
        else:
            vals = list(coord.shard) + [coord.a, coord.b]
        lin = 0
        for d, v in zip(dims, vals):
            lin = lin * d + v
        idx = lin * self.reps + coord.rep
        return self.start + idx if self.devices is None else self.devices[idx]

    def ranks(self) -> List[int]:
        if self.devices is not None:
            return list(self.devices)
        return list(range(self.start, self.start + self.block))

    def summed_index(self, c: Coord) -> int:
        return c.a if self.summed == "a" else c.b

    def same_index(self, c: Coord) -> int:
        return c.b if self.summed == "a" else c.a

    def box(self, shard: Sequence[int]) -> Box:
        ps = self.piece_shape
        return tuple((i * p, (i + 1) * p) for i, p in zip(shard, ps))

    def holders(self, shard: Tuple[int, ...], summed_idx: int) -> List[int]:
        """All ranks holding the piece (shard, summed index): every identical
        copy and every implicit replica."""
        out = []
        for s in range(self.same_degree):
            for rep in range(self.reps):
                a, b = (summed_idx, s) if self.summed == "a" else (s, summed_idx)
                out.append(self.rank_of(Coord(tuple(shard), a, b, rep)))
        return out

    def shards(self):
        def rec(i, acc):
            if i == len(self.degrees):
                yield tuple(acc)
                return
            for j in range(self.degrees[i]):
                yield from rec(i + 1, acc + [j])

        yield from rec(0, [])


def layout_from_pshape(pshape, block: int = 0, start: int = 0, devices: Optional[Sequence[int]] = None) -> Layout:
    """Layout of a C++ ParallelTensorShape (flexflow_train_amd._ffcore) on the
    block [start, start + block) or on an explicit device list."""
    sizes = tuple(int(d.size) for d in pshape.shard_dims)
    degs = tuple(int(d.degree) for d in pshape.shard_dims)
    if devices is not None:
        devices = tuple(int(d) for d in devices)
        if devices == tuple(range(devices[0], devices[0] + len(devices))):
            return Layout(sizes, degs, int(pshape.sum_degree), int(pshape.discard_copy_degree), len(devices),
                          devices[0])
        return Layout(sizes, degs, int(pshape.sum_degree), int(pshape.discard_copy_degree), len(devices),
                      devices[0], devices=devices)
    return Layout(sizes, degs, int(pshape.sum_degree), int(pshape.discard_copy_degree), block, start)


def placement(view, world: int) -> Tuple[int, ...]:
    """Normalise a machine view to a device tuple: a device list / tuple as
    is, a ``{"start": s, "block": b}`` dict (or ``("block", s, b)``) as the
    block, None as the whole world."""
    if view is None:
        return tuple(range(world))
    if isinstance(view, dict):
        if "devices" in view:
            return tuple(int(d) for d in view["devices"])
        return tuple(range(int(view["start"]), int(view["start"]) + int(view["block"])))
    if len(view) == 3 and view[0] == "block":
        return tuple(range(int(view[1]), int(view[1]) + int(view[2])))
    return tuple(int(d) for d in view)


def block(start: int, size: int) -> Tuple[int, ...]:
    """The contiguous device block [start, start + size) as a placement."""
    return tuple(range(start, start + size))


def intersect(b1: Box, b2: Box) -> Optional[Box]:
    out = []
    for (l1, h1), (l2, h2) in zip(b1, b2):
        lo, hi = max(l1, l2), min(h1, h2)
        if lo >= hi:
            return None
        out.append((lo, hi))
    return tuple(out)


def rel_slices(inner: Box, outer: Box):
    return tuple(slice(l - ol, h - ol) for (l, h), (ol, _) in zip(inner, outer))
