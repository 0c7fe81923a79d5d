"""Attribute (spatial) parallelism: halo exchange for window operators
(CONV2D / POOL2D) whose input is sharded along H.

The reference exposes attribute parallelism only as a flag
(bin/arg_parser/arg_parser.cc:60 ``--enable-attribute-parallel``) and its
op-attrs rejects H / W degrees (conv_2d.cc:82-83); here an NCHW activation
may be split into ``d`` equal row bands (op_attrs.cc ``spatial_split_ok``).

Shard ``j`` owns input rows ``[j Hl, (j+1) Hl)`` and computes output rows
``[j OHl, (j+1) OHl)``, which read input rows ``[lo_j, hi_j)`` with
``lo_j = j OHl s - p`` and ``hi_j = ((j+1) OHl - 1) s - p + k``.  Before the
op, each shard receives the rows it lacks from its two neighbours (point to
point, one ``batch_isend_irecv``: on MI355X one xGMI hop each way) and pads
the global border explicitly, so the op itself runs unpadded in H.  The
backward pass returns the halo rows' gradients to the shards that own them
(the transpose of the exchange) and adds them there.
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

import torch
import torch.distributed as dist


def conv_out(n: int, k: int, s: int, p: int) -> int:
    return (n + 2 * p - k) // s + 1


class HaloPlan:
    """Per-shard row bookkeeping (identical on every rank)."""

    def __init__(self, H: int, k: int, s: int, p: int, d: int):
        OH = conv_out(H, k, s, p)
        if H % d or OH % d:
            raise ValueError(f"halo: H={H} / OH={OH} not divisible by {d}")
        self.H, self.k, self.s, self.p, self.d = H, k, s, p, d
        self.Hl, self.OHl = H // d, OH // d
        self.rows: List[Tuple[int, int, int, int, int, int]] = []
        for j in range(d):
            lo = j * self.OHl * s - p
            hi = ((j + 1) * self.OHl - 1) * s - p + k
            top = max(0, j * self.Hl - max(lo, 0))                  # rows from shard j-1
            bot = max(0, min(hi, H) - (j + 1) * self.Hl)            # rows from shard j+1
            skip_top = max(0, max(lo, 0) - j * self.Hl)             # own rows nobody here reads
            skip_bot = max(0, (j + 1) * self.Hl - min(hi, H))
            pad_top, pad_bot = max(0, -lo), max(0, hi - H)
            if top > self.Hl or bot > self.Hl or (j == 0 and top) or (j == d - 1 and bot):
                raise ValueError("halo: wider than one neighbour")
            self.rows.append((top, bot, skip_top, skip_bot, pad_top, pad_bot))


class HaloGroup:
    """The ranks holding the H bands of one (batch, channel) slice, ordered
    by band index; ``index`` is this rank's band."""

    def __init__(self, dist_ctx, ranks: Sequence[int], index: int, plan: HaloPlan, pad_value: float = 0.0):
        self.dist_ctx = dist_ctx
        self.ranks = list(ranks)
        self.index = index
        self.plan = plan
        self.pad_value = pad_value

    # ------------------------------------------------------------- exchange
    def _p2p(self, sends, recvs):
        ops = [dist.P2POp(dist.isend, t.contiguous(), r) for r, t in sends if t.numel()]
        ops += [dist.P2POp(dist.irecv, t, r) for r, t in recvs if t.numel()]
        if not ops:
            return
        self.dist_ctx.stats["p2p"] += 1
        self.dist_ctx.stats["halo"] = self.dist_ctx.stats.get("halo", 0) + 1
        self.dist_ctx.stats["bytes"] += sum(t.numel() * t.element_size() for _, t in sends)

        def run():
            for w in dist.batch_isend_irecv(ops):
                w.wait()
        self.dist_ctx._issue(run, False)

    def extend(self, x: torch.Tensor) -> torch.Tensor:
        """x: this band [N, C, Hl, W] -> the rows its outputs read, halos
        and border padding included."""
        P, j = self.plan, self.index
        top, bot, skip_top, skip_bot, pad_top, pad_bot = P.rows[j]
        N, C, Hl, W = x.shape
        sends, recvs = [], []
        if j > 0 and P.rows[j - 1][1]:                  # the previous band needs my first rows
            sends.append((self.ranks[j - 1], x[:, :, :P.rows[j - 1][1]]))
        if j < P.d - 1 and P.rows[j + 1][0]:            # the next band needs my last rows
            sends.append((self.ranks[j + 1], x[:, :, Hl - P.rows[j + 1][0]:]))
        r_top = torch.empty((N, C, top, W), dtype=x.dtype, device=x.device)
        r_bot = torch.empty((N, C, bot, W), dtype=x.dtype, device=x.device)
        if top:
            recvs.append((self.ranks[j - 1], r_top))
        if bot:
            recvs.append((self.ranks[j + 1], r_bot))
        self._p2p(sends, recvs)
        parts = []
        if pad_top:
            parts.append(torch.full((N, C, pad_top, W), self.pad_value, dtype=x.dtype, device=x.device))
        parts += [r_top, x[:, :, skip_top:Hl - skip_bot], r_bot]
        if pad_bot:
            parts.append(torch.full((N, C, pad_bot, W), self.pad_value, dtype=x.dtype, device=x.device))
        y = torch.cat(parts, dim=2)
        if x.is_cuda:
            y = y.contiguous(memory_format=torch.channels_last)
        return y

    def fold(self, dx: torch.Tensor) -> torch.Tensor:
        """Gradient of ``extend``: dx [N, C, rows read, W] -> this band's
        [N, C, Hl, W], halo gradients returned to (and added by) their owners."""
        P, j = self.plan, self.index
        top, bot, skip_top, skip_bot, pad_top, pad_bot = P.rows[j]
        N, C, _, W = dx.shape
        Hl = P.Hl
        g_top = dx[:, :, pad_top:pad_top + top]
        mid0 = pad_top + top
        g_mid = dx[:, :, mid0:mid0 + Hl - skip_top - skip_bot]
        g_bot = dx[:, :, mid0 + Hl - skip_top - skip_bot:mid0 + Hl - skip_top - skip_bot + bot]
        sends, recvs = [], []
        if top:
            sends.append((self.ranks[j - 1], g_top))
        if bot:
            sends.append((self.ranks[j + 1], g_bot))
        n_first = P.rows[j - 1][1] if j > 0 else 0       # my first rows, read by band j-1
        n_last = P.rows[j + 1][0] if j < P.d - 1 else 0  # my last rows, read by band j+1
        r_first = torch.empty((N, C, n_first, W), dtype=dx.dtype, device=dx.device)
        r_last = torch.empty((N, C, n_last, W), dtype=dx.dtype, device=dx.device)
        if n_first:
            recvs.append((self.ranks[j - 1], r_first))
        if n_last:
            recvs.append((self.ranks[j + 1], r_last))
        self._p2p(sends, recvs)
        out = torch.zeros((N, C, Hl, W), dtype=dx.dtype, device=dx.device)
        if dx.is_cuda:
            out = out.contiguous(memory_format=torch.channels_last)
        out[:, :, skip_top:Hl - skip_bot] = g_mid
        if n_first:
            out[:, :, :n_first] += r_first
        if n_last:
            out[:, :, Hl - n_last:] += r_last
        return out
