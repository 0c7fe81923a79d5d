"""EXPERTS: mixture-of-experts FFN with top-k routing and expert parallelism.

Parity: the reference's MoE example (examples/cpp/mixture_of_experts/
moe.cc:159-164, ``ff.moe(input, num_exp, num_select, ...)``) composes top-k
gating, GROUP_BY, per-expert Dense layers and AGGREGATE; those operators are
missing from its vocabulary ("Example only").  Here the routed
expert block is one operator (IR: csrc/ffcore/src/op_attrs.cc experts_spec):

    out[b] = sum_j gate[b, j] * (W2[e] act(W1[e] x[b] + b1[e]) + b2[e]),  e = ids[b, j]

Dropless routing: the (token, slot) pairs are sorted by expert, every expert
runs two GEMMs over its contiguous row block (the MFMA / hipBLASLt GEMM
dispatch of ops/gemm.py with the bias + activation epilogue), results are
scaled by the gate and scatter-added back to their tokens.

Expert parallelism (weights sharded on the expert dim):
  * replicated tokens (discard copy c): rank with copy index i owns experts
    [i*E/c, (i+1)*E/c) and produces a partial sum; the PCG Reduction
    all-reduces it.
  * all-to-all (``expert_parallel_mode="alltoall"``): tokens stay batch
    sharded; pairs are dispatched to the rank owning their expert with one
    RCCL all-to-all (uneven splits, counts exchanged first), computed there,
    and returned with a second all-to-all; backward runs the transposes.
"""
from __future__ import annotations

from typing import List, Optional, Sequence

import torch
import torch.distributed as dist

from ..runtime.graphs import check_capturable

from .base import OpImpl, acc_grad, register
from .gemm import _blas


def matmul(a, b, trans_a=False, trans_b=False, bias=None, act="none", out=None, beta=0.0, pre=None):
    # expert row counts change every step: library GEMM (no per-shape autotune)
    return _blas(a, b, trans_a, trans_b, bias, act, out, beta, pre)


_ACT = {"none": lambda t: t, "relu": torch.relu, "gelu": lambda t: torch.nn.functional.gelu(t, approximate="tanh"),
        "sigmoid": torch.sigmoid, "tanh": torch.tanh}


class ExpertGroup:
    """Ranks exchanging tokens in all-to-all expert parallelism (ordered by
    expert shard)."""

    def __init__(self, dist_ctx, ranks: Sequence[int], index: int):
        self.dist_ctx = dist_ctx
        self.ranks = list(ranks)
        self.index = index
        self.size = len(self.ranks)

    @property
    def pg(self):
        return self.dist_ctx.group(self.ranks)


def _a2a_rows(x: torch.Tensor, send_counts: List[int], recv_counts: List[int], grp: ExpertGroup) -> torch.Tensor:
    out = torch.empty((sum(recv_counts),) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
    dist.all_to_all_single(out, x.contiguous(), output_split_sizes=recv_counts, input_split_sizes=send_counts,
                           group=grp.pg)
    grp.dist_ctx.stats["ep_all_to_all"] = grp.dist_ctx.stats.get("ep_all_to_all", 0) + 1
    return out


def _gpu_bf16(t) -> bool:
    return t.is_cuda and t.dtype == torch.bfloat16


def _expert_mlp_fwd(xs, eid, w1, b1, w2, b2, act, El):
    """Rows ``xs`` sorted by local expert id ``eid``; returns (y, pre, h, bounds)."""
    counts = torch.bincount(eid, minlength=El).tolist()
    H, O = w1.shape[2], w2.shape[2]
    pre = torch.empty(xs.shape[0], H, dtype=xs.dtype, device=xs.device)
    h = torch.empty_like(pre)
    y = torch.empty(xs.shape[0], O, dtype=xs.dtype, device=xs.device)
    lo = 0
    bounds = []
    for e, n in enumerate(counts):
        hi = lo + n
        bounds.append((lo, hi))
        if n:
            xe = xs[lo:hi]
            if _gpu_bf16(xe):
                h[lo:hi] = matmul(xe, w1[e], bias=b1[e] if b1 is not None else None, act=act,
                                  pre=pre[lo:hi] if act != "none" else None)
                if act == "none":
                    pre[lo:hi] = h[lo:hi]
                y[lo:hi] = matmul(h[lo:hi], w2[e], bias=b2[e] if b2 is not None else None)
            else:
                u = xe @ w1[e].to(xe.dtype)
                if b1 is not None:
                    u = u + b1[e].to(u.dtype)
                pre[lo:hi] = u
                h[lo:hi] = _ACT[act](u)
                v = h[lo:hi] @ w2[e].to(xe.dtype)
                if b2 is not None:
                    v = v + b2[e].to(v.dtype)
                y[lo:hi] = v
        lo = hi
    return y, pre, h, bounds


def _expert_mlp_bwd(dy, xs, pre, h, bounds, w1, w2, act, grads, need_dx):
    dW1, db1, dW2, db2 = grads
    dxs = torch.zeros_like(xs) if need_dx else None
    for e, (lo, hi) in enumerate(bounds):
        if hi == lo:
            continue
        g = dy[lo:hi]
        he, xe, pe = h[lo:hi], xs[lo:hi], pre[lo:hi]
        if db2 is not None:
            acc_grad(db2[e], g.float().sum(0))
        if _gpu_bf16(g):
            if dW2 is not None:
                matmul(he, g, trans_a=True, out=dW2[e], beta=1.0)
            dh = matmul(g, w2[e], trans_b=True)
        else:
            if dW2 is not None:
                acc_grad(dW2[e], he.float().t() @ g.float())
            dh = g @ w2[e].to(g.dtype).t()
        if act != "none":
            p = pe.float().detach().requires_grad_(True)
            _ACT[act](p).backward(dh.float())
            du = p.grad.to(dh.dtype)
        else:
            du = dh
        if db1 is not None:
            acc_grad(db1[e], du.float().sum(0))
        if _gpu_bf16(du):
            if dW1 is not None:
                matmul(xe, du, trans_a=True, out=dW1[e], beta=1.0)
            if need_dx:
                dxs[lo:hi] = matmul(du, w1[e], trans_b=True)
        else:
            if dW1 is not None:
                acc_grad(dW1[e], xe.float().t() @ du.float())
            if need_dx:
                dxs[lo:hi] = (du @ w1[e].to(du.dtype).t()).to(dxs.dtype)
    return dxs


@register("EXPERTS")
class ExpertsOp(OpImpl):
    @staticmethod
    def _weights(ctx, weights):
        if ctx.a("use_bias", True):
            return weights[0], weights[1], weights[2], weights[3]
        return weights[0], None, weights[1], None

    def forward(self, ctx, inputs, weights):
        x, ids, gate = inputs
        w1, b1, w2, b2 = self._weights(ctx, weights)
        act = ctx.a("activation", "relu")
        El = int(w1.shape[0])
        grp: Optional[ExpertGroup] = ctx.extra.get("ep_group")
        B, k = ids.shape
        tok = torch.arange(B, device=x.device).repeat_interleave(k)
        eg = ids.reshape(-1).long()
        g = gate.reshape(-1)
        if grp is None:
            # replicated tokens: this rank's experts only (partial sum)
            e0 = ctx.sum_index * El
            sel = ((eg >= e0) & (eg < e0 + El)).nonzero().squeeze(1)
            le = eg[sel] - e0
            order = torch.argsort(le, stable=True)
            sel = sel[order]
            xs = x[tok[sel]]
            y, pre, h, bounds = _expert_mlp_fwd(xs, le[order], w1, b1, w2, b2, act, El)
            out = torch.zeros(B, y.shape[1], dtype=torch.float32, device=x.device)
            out.index_add_(0, tok[sel], y.float() * g[sel].float().unsqueeze(1))
            saved = ("rep", x, sel, tok, g, xs, pre, h, bounds, y, w1, w2, None)
            return [out.to(x.dtype)], saved
        # all-to-all dispatch to expert owners
        owner = eg // El
        order = torch.argsort(owner, stable=True)
        send_counts = torch.bincount(owner, minlength=grp.size)
        recv_counts = torch.empty_like(send_counts)
        check_capturable("MoE all-to-all dispatch (data-dependent split sizes)")
        dist.all_to_all_single(recv_counts, send_counts, group=grp.pg)
        sc, rc = send_counts.tolist(), recv_counts.tolist()
        xr = _a2a_rows(x[tok[order]], sc, rc, grp)
        er = _a2a_rows((eg[order] - owner[order] * El).to(torch.int32).unsqueeze(1), sc, rc, grp).squeeze(1).long()
        lorder = torch.argsort(er, stable=True)
        xs = xr[lorder]
        y_s, pre, h, bounds = _expert_mlp_fwd(xs, er[lorder], w1, b1, w2, b2, act, El)
        y_r = torch.empty_like(y_s)
        y_r[lorder] = y_s
        y_back = _a2a_rows(y_r, rc, sc, grp)                    # rows in `order`
        out = torch.zeros(B, y_back.shape[1], dtype=torch.float32, device=x.device)
        sel = order
        out.index_add_(0, tok[sel], y_back.float() * g[sel].float().unsqueeze(1))
        saved = ("a2a", x, sel, tok, g, xs, pre, h, bounds, y_back, w1, w2, (sc, rc, lorder))
        return [out.to(x.dtype)], saved

    def backward(self, ctx, saved, grad_outputs, weight_grads, need_input_grad):
        mode, x, sel, tok, g, xs, pre, h, bounds, y_sel, w1, w2, extra = saved
        act = ctx.a("activation", "relu")
        if ctx.a("use_bias", True):
            grads = weight_grads[0], weight_grads[1], weight_grads[2], weight_grads[3]
        else:
            grads = weight_grads[0], None, weight_grads[1], None
        dout = grad_outputs[0]
        B, k = x.shape[0], g.numel() // x.shape[0]
        d_rows = dout[tok[sel]]                                 # [n, O]
        # gate gradient: <dout[token], y_pair>
        dgate = torch.zeros(g.numel(), dtype=torch.float32, device=x.device)
        dgate[sel] = (d_rows.float() * y_sel.float()).sum(1)
        dy_sel = (d_rows.float() * g[sel].float().unsqueeze(1)).to(x.dtype)
        need_dx = need_input_grad[0]
        if mode == "rep":
            dxs = _expert_mlp_bwd(dy_sel, xs, pre, h, bounds, w1, w2, act, grads, need_dx)
        else:
            sc, rc, lorder = extra
            grp = ctx.extra["ep_group"]
            dy_r = _a2a_rows(dy_sel, sc, rc, grp)
            dxs_l = _expert_mlp_bwd(dy_r[lorder].contiguous(), xs, pre, h, bounds, w1, w2, act, grads, True)
            dxr = torch.empty_like(dxs_l)
            dxr[lorder] = dxs_l
            dxs = _a2a_rows(dxr, rc, sc, grp)
        dx = None
        if need_dx:
            dx = torch.zeros(x.shape, dtype=torch.float32, device=x.device)
            dx.index_add_(0, tok[sel], dxs.float())
            dx = dx.to(x.dtype)
        dg = dgate.view(B, k).to(g.dtype) if need_input_grad[2] else None
        return [dx, None, dg]
