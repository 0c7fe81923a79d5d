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
  Causal masking skips blocks above the diagonal.  Works for any head
  count; transfer of the next block overlaps the current block's compute.
"""
from __future__ import annotations

import math
from typing import List, Optional, Sequence

import torch
import torch.distributed as dist

from ..runtime.graphs import check_capturable

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
def _exchange(tensors: List[torch.Tensor], grp: SeqGroup) -> List[torch.Tensor]:
    """Send ``tensors`` to the next rank, receive the previous rank's."""
    check_capturable("ring attention exchange")
    recv = [torch.empty_like(t) for t in tensors]
    ops = []
    for t in tensors:
        ops.append(dist.P2POp(dist.isend, t.contiguous(), grp.next_rank(), group=grp.pg))
    for r in recv:
        ops.append(dist.P2POp(dist.irecv, r, grp.prev_rank(), group=grp.pg))
    reqs = dist.batch_isend_irecv(ops)
    grp.dist_ctx.stats["ring_p2p"] = grp.dist_ctx.stats.get("ring_p2p", 0) + len(tensors)
    return reqs, recv


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
            for r in pending[0]:
                r.wait()
            cur = pending[1]
    o = o.to(q.dtype)
    return o, (q, k, v, o, lse.contiguous())


def ring_bwd(do, saved, causal, scale, grp: SeqGroup):
    q, k, v, o, lse = saved
    s, i = grp.size, grp.index
    do = do.contiguous()
    dq = torch.zeros(q.shape, dtype=torch.float32, device=q.device)
    cur = [k, v, torch.zeros(k.shape, dtype=torch.float32, device=k.device),
           torch.zeros(v.shape, dtype=torch.float32, device=v.device)]
    for t in range(s):
        j = (i - t) % s
        if not (causal and j > i):
            dq_j, dk_j, dv_j = block_attention_bwd(q, cur[0], cur[1], o, lse, do, causal and j == i, scale)
            dq += dq_j.float()
            cur[2] = cur[2] + dk_j.float()
            cur[3] = cur[3] + dv_j.float()
        if t < s - 1:
            reqs, cur = _exchange(cur, grp)
            for r in reqs:
                r.wait()
    # the block we hold belongs to rank i+1: one more hop returns dK/dV home
    if s > 1:
        reqs, back = _exchange(cur[2:], grp)
        for r in reqs:
            r.wait()
        dk, dv = back
    else:
        dk, dv = cur[2], cur[3]
    return dq.to(q.dtype), dk.to(k.dtype), dv.to(v.dtype)


def choose_mode(attrs: dict, heads_local: int, grp: SeqGroup) -> str:
    mode = str(attrs.get("seq_parallel_mode", "auto"))
    if mode == "auto":
        mode = "ulysses" if heads_local % grp.size == 0 else "ring"
    if mode == "ulysses" and heads_local % grp.size:
        raise ValueError(f"ulysses sequence parallelism needs heads ({heads_local}) divisible by {grp.size}")
    return mode


def sp_attention_fwd(q, k, v, causal, scale, grp: SeqGroup, mode: str):
    if mode == "ulysses":
        o, saved = ulysses_fwd(q, k, v, causal, scale, grp)
    else:
        o, saved = ring_fwd(q, k, v, causal, scale, grp)
    return o, (mode, saved)


def sp_attention_bwd(do, saved, causal, scale, grp: SeqGroup):
    mode, inner = saved
    if mode == "ulysses":
        return ulysses_bwd(do, inner, causal, scale, grp)
    return ring_bwd(do, inner, causal, scale, grp)
