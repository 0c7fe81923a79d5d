"""Blockwise (ring-attention) math on the flash kernels: merging per-block
forward results through the LSE and summing per-block backward results
computed with the global LSE must reproduce whole-sequence attention.  The
communication itself is covered by the multi-process CPU tests
(test_distributed.py::test_attention_sequence_parallel*)."""
import math

import pytest
import torch

from flexflow_train_amd.parallel import sequence as SP


def _ref(q, k, v, causal, scale):
    qt, kt, vt = (t.transpose(1, 2).float() for t in (q, k, v))
    s = qt @ kt.transpose(-1, -2) * scale
    if causal:
        S = s.shape[-1]
        s = s.masked_fill(torch.ones(S, S, dtype=torch.bool, device=s.device).triu(1), float("-inf"))
    return (torch.softmax(s, -1) @ vt).transpose(1, 2)


def _blockwise(q, k, v, causal, scale, nb, dev):
    """Rank i's view of a ring over nb blocks, all ranks simulated here."""
    B, S, H, D = q.shape
    L = S // nb
    qs, ks, vs = (list(t.split(L, 1)) for t in (q, k, v))
    outs, lses = [], []
    for i in range(nb):
        o = lse = None
        for j in range(nb):
            if causal and j > i:
                continue
            oj, lj = SP.block_attention(qs[i].contiguous(), ks[j].contiguous(), vs[j].contiguous(),
                                        causal and i == j, scale)
            o, lse = SP.merge(o, lse, oj, lj)
        outs.append(o.to(q.dtype))
        lses.append(lse.contiguous())
    return outs, lses, (qs, ks, vs)


@pytest.mark.gpu
@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("nb,D", [(2, 64), (4, 128), (4, 64)])
def test_ring_blocks_match_full_attention(causal, nb, D):
    from flexflow_train_amd import kernels as K
    assert K.available()
    torch.manual_seed(0)
    B, S, H = 2, 512, 4
    scale = 1.0 / math.sqrt(D)
    q, k, v = (torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16) for _ in range(3))
    outs, lses, (qs, ks, vs) = _blockwise(q, k, v, causal, scale, nb, "cuda")
    o = torch.cat(outs, 1)
    qf, kf, vf = (t.float().requires_grad_(True) for t in (q, k, v))
    ref = _ref(qf, kf, vf, causal, scale)
    torch.testing.assert_close(o.float(), ref, rtol=2e-2, atol=2e-2)
    do = torch.randn_like(q)
    ref.backward(do.float())
    L = S // nb
    dos = do.split(L, 1)
    dq = [torch.zeros(B, L, H, D, device="cuda") for _ in range(nb)]
    dk = [torch.zeros(B, L, H, D, device="cuda") for _ in range(nb)]
    dv = [torch.zeros(B, L, H, D, device="cuda") for _ in range(nb)]
    for i in range(nb):
        for j in range(nb):
            if causal and j > i:
                continue
            a, b, c = SP.block_attention_bwd(qs[i].contiguous(), ks[j].contiguous(), vs[j].contiguous(),
                                             outs[i], lses[i], dos[i].contiguous(), causal and i == j, scale)
            dq[i] += a.float()
            dk[j] += b.float()
            dv[j] += c.float()
    for got, want in ((dq, qf.grad), (dk, kf.grad), (dv, vf.grad)):
        torch.testing.assert_close(torch.cat(got, 1), want, rtol=5e-2, atol=5e-2)


def test_ring_blocks_cpu_fp32():
    torch.manual_seed(0)
    B, S, H, D = 1, 16, 2, 8
    scale = 1.0 / math.sqrt(D)
    q, k, v = (torch.randn(B, S, H, D) for _ in range(3))
    for causal in (False, True):
        outs, _, _ = _blockwise(q, k, v, causal, scale, 4, "cpu")
        torch.testing.assert_close(torch.cat(outs, 1), _ref(q, k, v, causal, scale), rtol=1e-5, atol=1e-5)
