"""Relative Frobenius errors of the non-GEMM bf16 kernels against fp64
references on the same bf16 inputs (attention fwd / bwd, LayerNorm fwd / bwd):
the numbers the GPU tests' bounds are set from."""
import json
import math

import torch

from flexflow_train_amd import kernels as K

DEV = "cuda"


def rel(a, b):
    a, b = a.double(), b.double()
    return ((a - b).norm() / b.norm().clamp_min(1e-300)).item()


def ref_attn(q, k, v, causal):
    qf, kf, vf = (t.double().transpose(1, 2) for t in (q, k, v))
    s = qf @ kf.transpose(-1, -2) / math.sqrt(q.shape[-1])
    if causal:
        Sq, Sk = s.shape[-2:]
        s = s.masked_fill(torch.ones(Sq, Sk, device=q.device, dtype=torch.bool).triu(1), float("-inf"))
    return (torch.softmax(s, -1) @ vf).transpose(1, 2)


def main():
    out = []
    for causal in (False, True):
        for D in (64, 128):
            for S in (512, 320):
                torch.manual_seed(6)
                B, H = 2, 4
                qkv = torch.randn(B, S, 3, H, D, device=DEV, dtype=torch.bfloat16)
                q, k, v = qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]
                o, lse = K.attention_fwd(q, k, v, causal=causal)
                qf, kf, vf = (t.double().requires_grad_(True) for t in (q, k, v))
                ref = ref_attn(qf, kf, vf, causal)
                do = torch.randn_like(o)
                ref.backward(do.double())
                dqkv = torch.empty_like(qkv)
                K.attention_bwd(q, k, v, o, lse, do, dqkv[:, :, 0], dqkv[:, :, 1], dqkv[:, :, 2], causal=causal)
                torch.cuda.synchronize()
                out.append({"op": "attention", "causal": causal, "D": D, "S": S, "o": rel(o, ref),
                            "dq": rel(dqkv[:, :, 0], qf.grad), "dk": rel(dqkv[:, :, 1], kf.grad),
                            "dv": rel(dqkv[:, :, 2], vf.grad),
                            "o_bf16_floor": rel(ref.to(torch.bfloat16), ref)})
    for N in (1024, 768, 4096, 1600):
        torch.manual_seed(0)
        M = 257
        x = torch.randn(M, N, device=DEV, dtype=torch.bfloat16)
        r = torch.randn(M, N, device=DEV, dtype=torch.bfloat16)
        g = (1 + 0.1 * torch.randn(N, device=DEV)).to(torch.bfloat16)
        b = (0.1 * torch.randn(N, device=DEV)).to(torch.bfloat16)
        y, s, mean, rstd = K.layernorm_fwd(x, g, b, 1e-5, residual=r)
        xs = (x.double() + r.double()).requires_grad_(True)
        ref = torch.nn.functional.layer_norm(xs, (N,), g.double(), b.double(), 1e-5)
        dy = torch.randn(M, N, device=DEV, dtype=torch.bfloat16)
        ss = s.double().requires_grad_(True)
        gg = g.double().requires_grad_(True)
        bb = b.double().requires_grad_(True)
        ref2 = torch.nn.functional.layer_norm(ss, (N,), gg, bb, 1e-5)
        ref2.backward(dy.double())
        dg = torch.zeros(N, device=DEV)
        db = torch.zeros(N, device=DEV)
        dx = K.layernorm_bwd(dy, s, mean, rstd, g, dg, db)
        torch.cuda.synchronize()
        out.append({"op": "layernorm", "N": N, "y": rel(y, ref), "dx_vs_stored_sum": rel(dx, ss.grad),
                    "dg": rel(dg, gg.grad), "db": rel(db, bb.grad), "sum": rel(s, x.double() + r.double())})
    for o in out:
        print(json.dumps(o))


if __name__ == "__main__":
    main()
