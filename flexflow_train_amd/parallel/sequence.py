"""Sequence (context) parallel attention over a group of ranks.

The reference has no way to scale sequence length across devices: its MHA
rejects a sharded sequence dim (lib/op-attrs/src/op-attrs/ops/attention/
multihead_attention_parallel_inputs.cc:46-66) and runs monolithic cuDNN
attention (lib/kernels/src/cuda/ops/attention_kernels.cu:255).  SURVEY §5.7
asks for both standard lowerings of a seq-sharded attention; our IR allows a
sequence degree on q/k/v (csrc/ffcore/src/op_attrs.cc mha_spec) and the
runtime lowers it here:

* **Ulysses** (head <-> sequence all-to-all): every rank projects its own
  sequence chunk, one ``all_to_all`` turns [B, S/s, H, d] into
  [B, S, H/s, d], the flash kernel runs on full sequences for H/s heads, and
  a second all-to-all returns the output to sequence shards.  Four
  all-to-alls forward (q, k, v, o) and four backward; every transfer is one
  RCCL all-to-all, which on the fully connected xGMI mesh uses all 7 links
  at once.  Needs H_local % s == 0.
* **Ring attention**: K/V blocks travel around the ring of ranks with
  batched isend/irecv while each rank computes blockwise attention of its
  queries against the block it holds, merging partial results through the
  log-sum-exp (the flash kernel emits log2-domain LSE).  Backward circulates
  (K, V, dK, dV) the same way using the *global* LSE and output, which makes
  every block's contribution exact; one extra hop returns dK/dV home.
  Causal masking skips blocks above the diagonal; with a causal mask the
  zig-zag layout (rank i holds chunks i and 2s-1-i of 2s) balances the work
  over the ranks.  Works for any head count; the next block's transfer
  (forward and backward) and the dK/dV accumulator hop overlap the current
  block's compute, and every transfer is capturable in a segmented hipGraph.
"""
from __future__ import annotations

import math
from typing import List, Optional, Sequence

import torch
import torch.distributed as dist

from .. import kernels as K

LOG2E = 1.4426950408889634


class SeqGroup:
    """The ranks sharing one sequence (ordered by sequence-chunk index)."""

    def __init__(self, dist_ctx, ranks: Sequence[int], index: int):
        self.dist_ctx = dist_ctx
        self.ranks = list(ranks)
        self.index = index
        self.size = len(self.ranks)

    @property
    def pg(self):
        return self.dist_ctx.group(self.ranks)

    def next_rank(self) -> int:
        return self.ranks[(self.index + 1) % self.size]

    def prev_rank(self) -> int:
        return self.ranks[(self.index - 1) % self.size]


# ----------------------------------------------------------------- kernels
def _flash_ok(q) -> bool:
    return q.is_cuda and q.dtype == torch.bfloat16 and q.shape[-1] in (64, 128) and K.available()


def block_attention(q, k, v, causal: bool, scale: float):
    """(o [B,Sq,H,d] in q.dtype, lse [B,H,Sq] fp32 log2 domain)."""
    if _flash_ok(q):
        return K.attention_fwd(q, k, v, causal=causal, scale=scale)
    qt, kt, vt = (t.transpose(1, 2).float() for t in (q, k, v))
    s = torch.matmul(qt, kt.transpose(-1, -2)) * (scale * LOG2E)
    if causal:
        Sq, Sk = s.shape[-2:]
        s = s.masked_fill(torch.ones(Sq, Sk, dtype=torch.bool, device=s.device).triu(1), float("-inf"))
    lse = torch.logsumexp(s / LOG2E, -1) * LOG2E
    p = torch.exp2(s - lse.unsqueeze(-1))
    o = torch.matmul(p, vt).transpose(1, 2).to(q.dtype).contiguous()
    return o, lse.contiguous()


def block_attention_bwd(q, k, v, o, lse, do, causal: bool, scale: float):
    """Gradients of one (q-block, kv-block) pair given the GLOBAL lse / o."""
    if _flash_ok(q):
        dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
        K.attention_bwd(q, k, v, o, lse, do, dq, dk, dv, causal=causal, scale=scale)
        return dq, dk, dv
    qt, kt, vt, ot, dot = (t.transpose(1, 2).float() for t in (q, k, v, o, do))
    s = torch.matmul(qt, kt.transpose(-1, -2)) * (scale * LOG2E)
    if causal:
        Sq, Sk = s.shape[-2:]
        s = s.masked_fill(torch.ones(Sq, Sk, dtype=torch.bool, device=s.device).triu(1), float("-inf"))
    p = torch.exp2(s - lse.unsqueeze(-1))
    dp = torch.matmul(dot, vt.transpose(-1, -2))
    delta = (dot * ot).sum(-1, keepdim=True)
    ds = p * (dp - delta) * scale
    dq = torch.matmul(ds, kt).transpose(1, 2)
    dk = torch.matmul(ds.transpose(-1, -2), qt).transpose(1, 2)
    dv = torch.matmul(p.transpose(-1, -2), dot).transpose(1, 2)
    return dq.to(q.dtype), dk.to(k.dtype), dv.to(v.dtype)


def merge(o, lse, o_j, lse_j):
    """Online-softmax merge of two partial results (log2-domain LSE)."""
    if o is None:
        return o_j.float(), lse_j
    new = torch.maximum(lse, lse_j)
    safe = torch.where(torch.isinf(new), torch.zeros_like(new), new)
    new = safe + torch.log2(torch.exp2(lse - safe) + torch.exp2(lse_j - safe))
    w = torch.exp2(lse - new).transpose(1, 2).unsqueeze(-1)       # [B,S,H,1]
    wj = torch.exp2(lse_j - new).transpose(1, 2).unsqueeze(-1)
    return o * w + o_j.float() * wj, new


# ------------------------------------------------------------------ Ulysses
def _a2a(x: torch.Tensor, grp: SeqGroup) -> torch.Tensor:
    out = torch.empty_like(x)
    pg = grp.pg
    grp.dist_ctx._issue(lambda: dist.all_to_all_single(out, x, group=pg), False)
    grp.dist_ctx.stats["sp_all_to_all"] = grp.dist_ctx.stats.get("sp_all_to_all", 0) + 1
    return out


def seq_to_heads(x: torch.Tensor, grp: SeqGroup) -> torch.Tensor:
    """[B, S/s, H, d] (sequence shard) -> [B, S, H/s, d] (head shard)."""
    B, Sl, H, d = x.shape
    s = grp.size
    send = x.reshape(B, Sl, s, H // s, d).permute(2, 0, 1, 3, 4).contiguous()
    recv = _a2a(send, grp)                                    # [s(seq chunk), B, Sl, H/s, d]
    return recv.permute(1, 0, 2, 3, 4).reshape(B, s * Sl, H // s, d)


def heads_to_seq(x: torch.Tensor, grp: SeqGroup) -> torch.Tensor:
    """[B, S, H/s, d] (head shard) -> [B, S/s, H, d] (sequence shard)."""
    B, S, Hs, d = x.shape
    s = grp.size
    send = x.reshape(B, s, S // s, Hs, d).permute(1, 0, 2, 3, 4).contiguous()
    recv = _a2a(send, grp)                                    # [s(head chunk), B, Sl, H/s, d]
    return recv.permute(1, 2, 0, 3, 4).reshape(B, S // s, s * Hs, d)


def ulysses_fwd(q, k, v, causal, scale, grp: SeqGroup):
    qh, kh, vh = (seq_to_heads(t.contiguous(), grp) for t in (q, k, v))
    oh, lse = block_attention(qh, kh, vh, causal, scale)
    return heads_to_seq(oh, grp).contiguous(), (qh, kh, vh, oh, lse)


def ulysses_bwd(do, saved, causal, scale, grp: SeqGroup):
    qh, kh, vh, oh, lse = saved
    doh = seq_to_heads(do.contiguous(), grp)
    dqh, dkh, dvh = block_attention_bwd(qh, kh, vh, oh, lse, doh, causal, scale)
    return tuple(heads_to_seq(t.contiguous(), grp) for t in (dqh, dkh, dvh))


# --------------------------------------------------------------------- ring
class _Reqs:
    """The requests of one batched isend/irecv as a single waitable work."""

    def __init__(self, reqs):
        self.reqs = list(reqs or [])

    def wait(self):
        for r in self.reqs:
            r.wait()
        return True


def _exchange(tensors: List[torch.Tensor], grp: SeqGroup):
    """Send ``tensors`` to the next rank and receive the previous rank's,
    asynchronously: returns (work, received buffers).  The receive buffers
    are allocated before the transfer is issued and the transfer goes through
    DistContext._issue, so inside a segmented hipGraph capture it becomes a
    segment boundary re-issued at replay (runtime/graphs.py) and the compute
    between issue and ``work.wait()`` runs while the blocks move."""
    send = [t.contiguous() for t in tensors]
    recv = [torch.empty_like(t) for t in send]
    nxt, prv, pg = grp.next_rank(), grp.prev_rank(), grp.pg

    def fn():
        ops = [dist.P2POp(dist.isend, t, nxt, group=pg) for t in send]
        ops += [dist.P2POp(dist.irecv, r, prv, group=pg) for r in recv]
        return _Reqs(dist.batch_isend_irecv(ops))

    work = grp.dist_ctx._issue(fn, True)
    grp.dist_ctx.stats["ring_p2p"] = grp.dist_ctx.stats.get("ring_p2p", 0) + len(send)
    return work, recv


def ring_fwd(q, k, v, causal, scale, grp: SeqGroup):
    s, i = grp.size, grp.index
    q, k, v = q.contiguous(), k.contiguous(), v.contiguous()
    o = lse = None
    cur = [k, v]
    for t in range(s):
        j = (i - t) % s                       # owner of the block we hold
        pending = None
        if t < s - 1:
            pending = _exchange(cur, grp)     # overlap the next block's transfer
        if not (causal and j > i):
            o_j, lse_j = block_attention(q, cur[0], cur[1], causal and j == i, scale)
            o, lse = merge(o, lse, o_j, lse_j)
        if pending is not None:
            pending[0].wait()
            cur = pending[1]
    o = o.to(q.dtype)
    return o, (q, k, v, o, lse.contiguous())


def _ring_bwd_loop(q, k, v, grp: SeqGroup, block_grads):
    """The backward ring shared by the contiguous and zig-zag layouts.

    K/V blocks circulate forward with the next hop issued BEFORE the block's
    compute; the dK/dV accumulator of the block a rank holds travels one step
    behind: the accumulator received from the previous rank is waited for
    only after this rank's own contribution to that block is computed, so
    both transfers overlap compute.  ``block_grads(j, k_j, v_j)`` returns
    (dq contribution, dk_j, dv_j) for the block owned by rank j (None where
    the causal mask skips it).  After s steps the last accumulator hop lands
    on the block's owner."""
    s, i = grp.size, grp.index
    dq = torch.zeros(q.shape, dtype=torch.float32, device=q.device)
    kv = [k, v]
    acc_pending = None
    for t in range(s):
        j = (i - t) % s
        kv_pending = _exchange(kv, grp) if t < s - 1 else None
        g = block_grads(j, kv[0], kv[1])
        if g is not None:
            dq_j, dk_j, dv_j = g
            dq += dq_j
        else:
            dk_j = torch.zeros(k.shape, dtype=torch.float32, device=k.device)
            dv_j = torch.zeros(v.shape, dtype=torch.float32, device=v.device)
        if acc_pending is not None:
            acc_pending[0].wait()
            dk_j = dk_j + acc_pending[1][0]
            dv_j = dv_j + acc_pending[1][1]
        acc_pending = _exchange([dk_j, dv_j], grp) if s > 1 else (None, [dk_j, dv_j])
        if kv_pending is not None:
            kv_pending[0].wait()
            kv = kv_pending[1]
    if acc_pending[0] is not None:
        acc_pending[0].wait()
    dk, dv = acc_pending[1]
    return dq.to(q.dtype), dk.to(k.dtype), dv.to(v.dtype)


def ring_bwd(do, saved, causal, scale, grp: SeqGroup):
    q, k, v, o, lse = saved
    i = grp.index
    do = do.contiguous()

    def block_grads(j, k_j, v_j):
        if causal and j > i:
            return None
        dq_j, dk_j, dv_j = block_attention_bwd(q, k_j, v_j, o, lse, do, causal and j == i, scale)
        return dq_j.float(), dk_j.float(), dv_j.float()

    return _ring_bwd_loop(q, k, v, grp, block_grads)


# ---------------------------------------------------------- zig-zag ring
# Causal ring attention over contiguous sequence shards is unbalanced: rank i
# attends to i + 1 blocks, so the last rank does s blocks of work while the
# first does one.  The zig-zag layout cuts the sequence into 2s chunks and
# gives rank i chunks i and 2s-1-i (one early, one late): every ring step then
# costs every rank half a block (the diagonal step a causal block), whatever
# i and j.  The rest of the model keeps contiguous shards; q/k/v are moved
# into the zig-zag layout by one all-to-all (stacked) and the output back by
# another (two each way in the backward).

def _contig(c: int, s: int):
    return c // 2, c % 2                      # chunk -> (owner, slot)


def _zigzag(c: int, s: int):
    return (c, 0) if c < s else (2 * s - 1 - c, 1)


def _relayout(x: torch.Tensor, grp: SeqGroup, before, after) -> torch.Tensor:
    """Move the two sequence chunks of ``x`` [B, S_local, ...] (dim 1 split
    in halves = chunk slots) from layout ``before`` to layout ``after``
    (chunk c -> (owner, slot)) with one variable-split all-to-all."""
    s, i = grp.size, grp.index
    B, Sl = x.shape[0], x.shape[1]
    if Sl % 2:
        raise ValueError(f"zig-zag ring attention needs an even local sequence length, got {Sl}")
    parts = x.reshape(B, 2, Sl // 2, *x.shape[2:])
    chunks = range(2 * s)
    out_c = sorted((c for c in chunks if before(c, s)[0] == i), key=lambda c: after(c, s))
    in_c = sorted((c for c in chunks if after(c, s)[0] == i), key=lambda c: (before(c, s)[0], after(c, s)[1]))
    send = torch.stack([parts[:, before(c, s)[1]] for c in out_c], 0).reshape(len(out_c), -1).contiguous()
    recv = torch.empty_like(send)
    in_splits = [sum(1 for c in out_c if after(c, s)[0] == r) for r in range(s)]
    out_splits = [sum(1 for c in in_c if before(c, s)[0] == r) for r in range(s)]
    pg = grp.pg
    grp.dist_ctx._issue(lambda: dist.all_to_all_single(recv, send, out_splits, in_splits, group=pg), False)
    grp.dist_ctx.stats["sp_all_to_all"] = grp.dist_ctx.stats.get("sp_all_to_all", 0) + 1
    out = torch.empty_like(parts)
    shp = parts.shape[:1] + parts.shape[2:]
    for n, c in enumerate(in_c):
        out[:, after(c, s)[1]] = recv[n].view(shp)
    return out.reshape(x.shape)


def _to_zigzag(ts: Sequence[torch.Tensor], grp: SeqGroup) -> List[torch.Tensor]:
    st = torch.stack([t.contiguous() for t in ts], 2)          # [B, Sl, n, ...]: one all-to-all for all
    z = _relayout(st, grp, _contig, _zigzag)
    return [z[:, :, n].contiguous() for n in range(len(ts))]


def _from_zigzag(ts: Sequence[torch.Tensor], grp: SeqGroup) -> List[torch.Tensor]:
    st = torch.stack([t.contiguous() for t in ts], 2)
    c = _relayout(st, grp, _zigzag, _contig)
    return [c[:, :, n].contiguous() for n in range(len(ts))]


def ring_zigzag_fwd(q, k, v, causal, scale, grp: SeqGroup):
    """Causal ring attention over zig-zag chunks (see above)."""
    s, i = grp.size, grp.index
    grp.dist_ctx.stats["ring_zigzag"] = grp.dist_ctx.stats.get("ring_zigzag", 0) + 1
    qz, kz, vz = _to_zigzag([q, k, v], grp)
    h = qz.shape[1] // 2
    o = lse = None
    cur = [kz, vz]
    for t in range(s):
        j = (i - t) % s
        pending = _exchange(cur, grp) if t < s - 1 else None
        if j == i:                      # own chunks: causal over [chunk i, chunk 2s-1-i]
            o, lse = merge(None, None, *block_attention(qz, cur[0], cur[1], True, scale))
        elif j < i:                     # both query chunks see the early key chunk j only
            o_j, lse_j = block_attention(qz, cur[0][:, :h], cur[1][:, :h], False, scale)
            o, lse = merge(o, lse, o_j, lse_j)
        else:                           # the late query chunk sees both of rank j's chunks
            o_j, lse_j = block_attention(qz[:, h:], cur[0], cur[1], False, scale)
            o_hi, lse_hi = merge(o[:, h:], lse[:, :, h:], o_j, lse_j)
            o = torch.cat([o[:, :h], o_hi], 1)
            lse = torch.cat([lse[:, :, :h], lse_hi], 2)
        if pending is not None:
            pending[0].wait()
            cur = pending[1]
    oz = o.to(q.dtype)
    (out,) = _from_zigzag([oz], grp)
    return out, (qz, kz, vz, oz, lse.contiguous())


def ring_zigzag_bwd(do, saved, causal, scale, grp: SeqGroup):
    qz, kz, vz, oz, lse = saved
    i = grp.index
    (doz,) = _to_zigzag([do], grp)
    h = qz.shape[1] // 2
    q_hi, o_hi, do_hi = qz[:, h:].contiguous(), oz[:, h:].contiguous(), doz[:, h:].contiguous()
    lse_hi = lse[:, :, h:].contiguous()

    def block_grads(j, k_j, v_j):
        if j == i:
            dq, dk, dv = block_attention_bwd(qz, k_j, v_j, oz, lse, doz, True, scale)
            return dq.float(), dk.float(), dv.float()
        dk = torch.zeros(k_j.shape, dtype=torch.float32, device=k_j.device)
        dv = torch.zeros(v_j.shape, dtype=torch.float32, device=v_j.device)
        if j < i:
            dq, dk_lo, dv_lo = block_attention_bwd(qz, k_j[:, :h].contiguous(), v_j[:, :h].contiguous(), oz, lse,
                                                   doz, False, scale)
            dk[:, :h] = dk_lo.float()
            dv[:, :h] = dv_lo.float()
            return dq.float(), dk, dv
        dq_hi, dk_f, dv_f = block_attention_bwd(q_hi, k_j, v_j, o_hi, lse_hi, do_hi, False, scale)
        dq = torch.zeros(qz.shape, dtype=torch.float32, device=qz.device)
        dq[:, h:] = dq_hi.float()
        return dq, dk_f.float(), dv_f.float()

    dqz, dkz, dvz = _ring_bwd_loop(qz, kz, vz, grp, block_grads)
    return tuple(_from_zigzag([dqz, dkz, dvz], grp))


def choose_mode(attrs: dict, heads_local: int, grp: SeqGroup) -> str:
    """auto: Ulysses when the local heads split over the group, else ring
    (zig-zag when causal); "ring" with a causal mask also runs zig-zag unless
    "ring_contiguous" is asked for."""
    mode = str(attrs.get("seq_parallel_mode", "auto"))
    causal = bool(attrs.get("causal", False))
    if mode == "auto":
        mode = "ulysses" if heads_local % grp.size == 0 else "ring"
    if mode == "ring" and causal:
        mode = "ring_zigzag"
    if mode == "ring_contiguous":
        mode = "ring"
    if mode == "ulysses" and heads_local % grp.size:
        raise ValueError(f"ulysses sequence parallelism needs heads ({heads_local}) divisible by {grp.size}")
    return mode


def sp_attention_fwd(q, k, v, causal, scale, grp: SeqGroup, mode: str):
    if mode == "ulysses":
        o, saved = ulysses_fwd(q, k, v, causal, scale, grp)
    elif mode == "ring_zigzag" and causal:
        o, saved = ring_zigzag_fwd(q, k, v, causal, scale, grp)
    else:
        mode = "ring"
        o, saved = ring_fwd(q, k, v, causal, scale, grp)
    return o, (mode, saved)


def sp_attention_bwd(do, saved, causal, scale, grp: SeqGroup):
    mode, inner = saved
    if mode == "ulysses":
        return ulysses_bwd(do, inner, causal, scale, grp)
    if mode == "ring_zigzag":
        return ring_zigzag_bwd(do, inner, causal, scale, grp)
    return ring_bwd(do, inner, causal, scale, grp)
