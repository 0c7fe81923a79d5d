"""MULTIHEAD_ATTENTION operator (projections + flash attention + output proj).

Parity: lib/local-execution/src/ops/attention.cc and lib/kernels/src/cuda/ops/
attention_kernels.cu (cuDNN multi-head attention with fused projections;
weights laid out as [qSize*kdim + kSize*kdim + vSize*vdim + vdim*embed, heads],
op-attrs attention.cc:136-170).

Local-piece layout (head-parallel degree h -> this rank owns Hl = H/h heads):
the logical weight piece [P, Hl] is stored physically as
  self-attention (q/k/v feature sizes equal):
      Wqkv [E, 3, Hl, kdim] (row-major, = one [E, 3*Hl*kdim] GEMM operand)
      Wo   [Hl*vdim, E]
  otherwise: Wq [Eq, Hl*k] | Wk [Ek, Hl*k] | Wv [Ev, Hl*v] | Wo [Hl*v, E]
input bias piece [2k+v, Hl] -> physically [3, Hl, k] (added by the QKV GEMM
epilogue); output bias [E] is added on partial-sum replica 0 only.
The fused QKV output [B, S, 3, Hl, k] is consumed by the flash kernel in
place (strided views), and dQKV is produced in the same packed layout, so the
backward needs exactly one GEMM for dW_qkv and one for dX.
"""
from __future__ import annotations

import math
import os

import torch

from .. import kernels as K
from ..parallel import sequence as SP
from .base import OpContext, OpImpl, acc_grad, register
from .gemm import matmul, wgrad_matmul

# q/k/v projection-bias gradients from the attention backward kernels'
# epilogues instead of a separate column-sum pass over dQKV
# (FF_ATTN_FUSED_DBIAS=1).  Round 2 did this with one fp32 atomic per column
# per wave onto H*D addresses, which made dK/dV 117 -> 220 us and dQ 76 -> 150
# us (profiles/ab_attn_dbias_r2.txt).  Round 3: each wave stores its 32-row
# partial sums into a slab row (a reduce-scatter, no atomics) and one
# reduction adds the slab; measured even with the 25 us pass it replaces
# (BERT-large 723-727 vs 728 samples/s, profiles/ab_attn_dbias_slab_r3.txt),
# so the pass stays the default.
_FUSED_DBIAS = os.environ.get("FF_ATTN_FUSED_DBIAS", "0") == "1"


def _dims(ctx: OpContext, q, k, v, W):
    H_local = W.shape[-1] if W.dim() == 2 else None
    E = int(ctx.a("embed_dim"))
    H = int(ctx.a("num_heads"))
    kd = int(ctx.a("kdim") or 0) or E // H
    vd = int(ctx.a("vdim") or 0) or E // H
    Hl = H // max(1, ctx.input_copy_degree)
    if H_local is not None:
        Hl = H_local
    return E, Hl, kd, vd, q.shape[-1], k.shape[-1], v.shape[-1]


def _split_weights(W, E, Hl, kd, vd, Eq, Ek, Ev):
    flat = W.reshape(-1)
    if Eq == Ek == Ev and kd == vd:
        n_qkv = Eq * 3 * Hl * kd
        Wqkv = flat[:n_qkv].view(Eq, 3 * Hl * kd)
        Wo = flat[n_qkv:n_qkv + Hl * vd * E].view(Hl * vd, E)
        # per-projection strided views of the fused operand, for attention whose
        # q / k / v are different tensors of the same width (cross-attention)
        W3 = Wqkv.view(Eq, 3, Hl * kd)
        return {"qkv": Wqkv, "o": Wo, "q": W3[:, 0], "k": W3[:, 1], "v": W3[:, 2]}
    o0 = 0
    Wq = flat[o0:o0 + Eq * Hl * kd].view(Eq, Hl * kd)
    o0 += Eq * Hl * kd
    Wk = flat[o0:o0 + Ek * Hl * kd].view(Ek, Hl * kd)
    o0 += Ek * Hl * kd
    Wv = flat[o0:o0 + Ev * Hl * vd].view(Ev, Hl * vd)
    o0 += Ev * Hl * vd
    Wo = flat[o0:o0 + Hl * vd * E].view(Hl * vd, E)
    return {"q": Wq, "k": Wk, "v": Wv, "o": Wo}


def _torch_attention(q, k, v, causal, scale):
    # q,k,v: [B, S, H, D] -> [B, S, H, D]
    qt, kt, vt = (t.transpose(1, 2) for t in (q, k, v))
    s = torch.matmul(qt.float(), kt.float().transpose(-1, -2)) * scale
    if causal:
        Sq, Sk = s.shape[-2:]
        mask = torch.ones(Sq, Sk, dtype=torch.bool, device=s.device).triu(1)
        s = s.masked_fill(mask, float("-inf"))
    p = torch.softmax(s, -1)
    return torch.matmul(p, vt.float()).transpose(1, 2).to(q.dtype)


def _layout_dims(attrs: dict, Hl: int):
    E = int(attrs["embed_dim"])
    H = int(attrs["num_heads"])
    kd = int(attrs.get("kdim") or 0) or E // H
    vd = int(attrs.get("vdim") or 0) or E // H
    Eq, Ek, Ev = (attrs.get("_in_features") or [E, E, E])[:3]
    return E, kd, vd, int(Eq), int(Ek), int(Ev)


def _blocks(E, kd, vd, Eq, Ek, Ev):
    # per-head logical column: [Wq: Eq x k][Wk: Ek x k][Wv: Ev x v][Wo: v x E]
    return [(Eq, kd), (Ek, kd), (Ev, vd), (vd, E)]


@register("MULTIHEAD_ATTENTION")
class MultiHeadAttentionOp(OpImpl):
    def to_physical(self, attrs, index, piece):
        if index > 1:
            return piece
        Hl = piece.shape[-1]
        E, kd, vd, Eq, Ek, Ev = _layout_dims(attrs, Hl)
        if index == 1:  # [2k+v, Hl] -> q[Hl, k] | k[Hl, k] | v[Hl, v]
            return torch.cat([piece[:kd].t().reshape(-1), piece[kd:2 * kd].t().reshape(-1),
                              piece[2 * kd:].t().reshape(-1)])
        parts, o = [], 0
        mats = []
        for (r, c) in _blocks(E, kd, vd, Eq, Ek, Ev):
            mats.append(piece[o:o + r * c].view(r, c, Hl))
            o += r * c
        q, k, v, wo = mats
        if Eq == Ek == Ev and kd == vd:
            qkv = torch.stack([m.permute(0, 2, 1) for m in (q, k, v)], dim=1)  # [E, 3, Hl, k]
            parts.append(qkv.reshape(-1))
        else:
            for m in (q, k, v):
                parts.append(m.permute(0, 2, 1).reshape(-1))                   # [Ein, Hl, d]
        parts.append(wo.permute(2, 0, 1).reshape(-1))                           # [Hl, v, E]
        return torch.cat(parts)

    def to_logical(self, attrs, index, piece):
        if index > 1:
            return piece
        Hl = piece.shape[-1]
        E, kd, vd, Eq, Ek, Ev = _layout_dims(attrs, Hl)
        flat = piece.reshape(-1)
        if index == 1:
            q = flat[:Hl * kd].view(Hl, kd).t()
            k = flat[Hl * kd:2 * Hl * kd].view(Hl, kd).t()
            v = flat[2 * Hl * kd:].view(Hl, vd).t()
            return torch.cat([q, k, v], dim=0).contiguous()
        cols = []
        if Eq == Ek == Ev and kd == vd:
            n = Eq * 3 * Hl * kd
            qkv = flat[:n].view(Eq, 3, Hl, kd)
            for j in range(3):
                cols.append(qkv[:, j].permute(0, 2, 1).reshape(Eq * kd, Hl))
            o = n
        else:
            o = 0
            for (r, c) in _blocks(E, kd, vd, Eq, Ek, Ev)[:3]:
                cols.append(flat[o:o + r * Hl * c].view(r, Hl, c).permute(0, 2, 1).reshape(r * c, Hl))
                o += r * Hl * c
        wo = flat[o:o + Hl * vd * E].view(Hl, vd, E).permute(1, 2, 0).reshape(vd * E, Hl)
        cols.append(wo)
        return torch.cat(cols, dim=0).contiguous()

    def init_weight(self, ctx, index, logical_shape, initializer, gen):
        # glorot per projection block (fan_in=E, fan_out=H*kdim), not on the
        # flattened [P, H] tensor whose fans are meaningless.
        if index != 0 or initializer.get("type") not in ("glorot_uniform", "glorot_normal"):
            return None
        P, H = logical_shape
        E = int(ctx.a("embed_dim"))
        kd = int(ctx.a("kdim") or 0) or E // int(ctx.a("num_heads"))
        bound = math.sqrt(6.0 / (E + H * kd))
        if initializer["type"] == "glorot_uniform":
            return (torch.rand(P, H, generator=gen) * 2 - 1) * bound
        return torch.randn(P, H, generator=gen) * math.sqrt(2.0 / (E + H * kd))

    def init_spec(self, ctx, index, logical_shape, initializer):
        if index != 0 or initializer.get("type") not in ("glorot_uniform", "glorot_normal"):
            return None
        P, H = logical_shape
        E = int(ctx.a("embed_dim"))
        kd = int(ctx.a("kdim") or 0) or E // int(ctx.a("num_heads"))
        if initializer["type"] == "glorot_uniform":
            bound = math.sqrt(6.0 / (E + H * kd))
            return (0, -bound, bound, 0.0, 0.0)
        return (1, 0.0, math.sqrt(2.0 / (E + H * kd)), 0.0, 0.0)

    def forward(self, ctx: OpContext, inputs, weights):
        q_in, k_in, v_in = inputs
        W = weights[0]
        b_in = weights[1] if len(weights) > 1 else None
        b_out = weights[2] if len(weights) > 2 and ctx.sum_index == 0 else None
        E, Hl, kd, vd, Eq, Ek, Ev = _dims(ctx, q_in, k_in, v_in, W)
        ws = _split_weights(W, E, Hl, kd, vd, Eq, Ek, Ev)
        B, Sq = q_in.shape[0], q_in.shape[1]
        Sk = k_in.shape[1]
        causal = bool(ctx.a("causal", False))
        scale = 1.0 / math.sqrt(kd)
        self_attn = (q_in is k_in) and (k_in is v_in) and "qkv" in ws
        x2 = q_in.reshape(-1, Eq).contiguous()
        bias_qkv = b_in.reshape(-1) if b_in is not None else None  # [3, Hl, k] order
        if self_attn:
            qkv = matmul(x2, ws["qkv"], bias=bias_qkv)                  # [B*S, 3*Hl*k]
            qkv5 = qkv.view(B, Sq, 3, Hl, kd)
            q, k, v = qkv5[:, :, 0], qkv5[:, :, 1], qkv5[:, :, 2]
            proj = qkv
        else:
            bq = bk = bv = None
            if bias_qkv is not None:
                bq, bk, bv = bias_qkv[:Hl * kd], bias_qkv[Hl * kd:2 * Hl * kd], bias_qkv[2 * Hl * kd:]
            q = matmul(x2, ws["q"], bias=bq).view(B, Sq, Hl, kd)
            k = matmul(k_in.reshape(-1, Ek).contiguous(), ws["k"], bias=bk).view(B, Sk, Hl, kd)
            v = matmul(v_in.reshape(-1, Ev).contiguous(), ws["v"], bias=bv).view(B, Sk, Hl, vd)
            proj = (q, k, v)
        grp = ctx.extra.get("seq_group")
        use_flash = (q.is_cuda and q.dtype == torch.bfloat16 and kd == vd and kd in (64, 128) and K.available())
        if grp is not None and grp.size > 1:
            # sequence-sharded q/k/v: Ulysses all-to-all or ring attention
            o, lse = SP.sp_attention_fwd(q, k, v, causal, scale, grp, SP.choose_mode(ctx.attrs, Hl, grp))
            lse = ("sp", lse)
        elif use_flash:
            o, lse = K.attention_fwd(q, k, v, causal=causal, scale=scale)
        else:
            o, lse = _torch_attention(q, k, v, causal, scale), None
        o2 = o.reshape(B * Sq, Hl * vd)
        out = matmul(o2, ws["o"], bias=b_out)
        saved = (x2, k_in if not self_attn else None, v_in if not self_attn else None, proj, o, lse, ws,
                 self_attn, (B, Sq, Sk, Hl, kd, vd, Eq, Ek, Ev, E, causal, scale))
        return [out.view(B, Sq, E)], saved

    def backward(self, ctx, saved, grad_outputs, weight_grads, need_input_grad):
        x2, k_in, v_in, proj, o, lse, ws, self_attn, dims = saved
        B, Sq, Sk, Hl, kd, vd, Eq, Ek, Ev, E, causal, scale = dims
        dW = weight_grads[0]
        db_in = weight_grads[1] if len(weight_grads) > 1 else None
        db_out = weight_grads[2] if len(weight_grads) > 2 else None  # identical on every partial replica
        dout = grad_outputs[0].reshape(B * Sq, E).contiguous()
        o2 = o.reshape(B * Sq, Hl * vd)
        gpu = dout.is_cuda and dout.dtype == torch.bfloat16 and K.available()
        # ---- output projection
        dW_views = _split_weights(dW, E, Hl, kd, vd, Eq, Ek, Ev) if dW is not None else None
        if ctx.extra.pop("db_done", False):
            db_out = None   # accumulated by the consuming add+LayerNorm's backward (layernorm_bwd dsum)
        if db_out is not None:
            if gpu:
                K.colsum_act(dout, None, "none", db_out, write_dx=False)
            else:
                acc_grad(db_out, dout.float().sum(0))
        wbeta = ctx.extra.get("wgrad_beta", [1.0])[0]
        if dW_views is not None:
            if gpu:
                wgrad_matmul(ctx, o2, dout, dW_views["o"], wbeta)
            else:
                acc_grad(dW_views["o"], o2.float().t() @ dout.float())
        do = matmul(dout, ws["o"], trans_b=True) if gpu else dout @ ws["o"].to(dout.dtype).t()
        do4 = do.view(B, Sq, Hl, vd)
        # ---- attention core
        if self_attn:
            qkv = proj
            qkv5 = qkv.view(B, Sq, 3, Hl, kd)
            q, k, v = qkv5[:, :, 0], qkv5[:, :, 1], qkv5[:, :, 2]
        else:
            q, k, v = proj
        if isinstance(lse, tuple):
            dq_, dk_, dv_ = SP.sp_attention_bwd(do4, lse[1], causal, scale, ctx.extra["seq_group"])
            if self_attn:
                dproj = torch.stack([dq_, dk_, dv_], dim=2).reshape(B * Sq, 3 * Hl * kd)
            else:
                dq, dk, dv = dq_, dk_, dv_
        elif lse is not None:
            if self_attn:
                dproj = torch.empty_like(qkv)
                d5 = dproj.view(B, Sq, 3, Hl, kd)
                dq, dk, dv = d5[:, :, 0], d5[:, :, 1], d5[:, :, 2]
            else:
                dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
            fused_db = None
            if _FUSED_DBIAS and self_attn and db_in is not None and kd == vd \
                    and db_in.dtype == torch.float32 and db_in.is_contiguous():
                dbf = db_in.reshape(-1)
                n = Hl * kd
                fused_db = (dbf[:n], dbf[n:2 * n], dbf[2 * n:3 * n])
            K.attention_bwd(q, k, v, o, lse, do4, dq, dk, dv, causal=causal, scale=scale, dbias=fused_db)
            if fused_db is not None:
                db_in = None   # accumulated by the attention backward kernels
        else:
            qf, kf, vf = (t.detach().float().requires_grad_(True) for t in (q, k, v))
            ref = _torch_attention(qf, kf, vf, causal, scale)
            ref.float().backward(do4.float())
            dq, dk, dv = (t.grad.to(do.dtype) for t in (qf, kf, vf))
            if self_attn:
                dproj = torch.stack([dq, dk, dv], dim=2).reshape(B * Sq, 3 * Hl * kd)
        # ---- input projections
        dx_q = dx_k = dx_v = None
        if self_attn:
            d2 = dproj.view(B * Sq, 3 * Hl * kd)
            if db_in is not None:
                if gpu:
                    K.colsum_act(d2, None, "none", db_in.reshape(-1), write_dx=False)
                else:
                    acc_grad(db_in, d2.float().sum(0))
            if dW_views is not None:
                if gpu:
                    wgrad_matmul(ctx, x2, d2, dW_views["qkv"], wbeta)
                else:
                    acc_grad(dW_views["qkv"], x2.float().t() @ d2.float())
            if need_input_grad[0]:
                acc = ctx.extra.get("grad_acc", [None])[0]
                if gpu and acc is not None and acc.dtype == d2.dtype and acc.is_contiguous():
                    matmul(d2, ws["qkv"], trans_b=True, out=acc.view(B * Sq, Eq), beta=1.0)
                    return [acc, None, None]
                dx_q = (matmul(d2, ws["qkv"], trans_b=True) if gpu else d2 @ ws["qkv"].to(d2.dtype).t()).view(B, Sq, Eq)
            return [dx_q, None, None]
        srcs = ((x2, dq, "q", Eq, Sq, kd), (k_in.reshape(-1, Ek).contiguous(), dk, "k", Ek, Sk, kd),
                (v_in.reshape(-1, Ev).contiguous(), dv, "v", Ev, Sk, vd))
        outs = []
        for j, (xin, dp, key, Ein, S, dd) in enumerate(srcs):
            d2 = dp.reshape(B * S, Hl * dd).contiguous()
            if db_in is not None:
                seg = db_in.reshape(-1)[j * Hl * kd:(j * Hl * kd) + Hl * dd]
                acc_grad(seg, d2.float().sum(0))
            if dW_views is not None:
                if gpu:
                    wgrad_matmul(ctx, xin, d2, dW_views[key], wbeta)
                else:
                    acc_grad(dW_views[key], xin.float().t() @ d2.float())
            if need_input_grad[j]:
                dxx = matmul(d2, ws[key], trans_b=True) if gpu else d2 @ ws[key].to(d2.dtype).t()
                outs.append(dxx.view(B, S, Ein))
            else:
                outs.append(None)
        return outs
