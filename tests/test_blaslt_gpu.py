"""hipBLASLt epilogue GEMMs (csrc/kernels/blaslt.hip) against PyTorch fp32
references: bias, GELU, and BGRADB (dW^T with the bias gradient)."""
import pytest
import torch
import torch.nn.functional as F

from flexflow_train_amd import kernels as K

pytestmark = pytest.mark.gpu


def _r(*s):
    return (torch.randn(*s, device="cuda") * 0.5).to(torch.bfloat16)


@pytest.mark.parametrize("M,N,Kd", [(256, 384, 128), (1024, 1024, 512), (200, 72, 96)])
def test_bias_and_gelu(M, N, Kd):
    x, w, b = _r(M, Kd), _r(Kd, N), _r(N)
    ref = x.float() @ w.float() + b.float()
    y = K.blaslt_gemm(x, w, epilogue=K.EPI_BIAS, bias=b)
    torch.testing.assert_close(y.float(), ref, rtol=2e-2, atol=5e-2)
    y = K.blaslt_gemm(x, w, epilogue=K.EPI_GELU_BIAS, bias=b)
    torch.testing.assert_close(y.float(), F.gelu(ref, approximate="tanh"), rtol=2e-2, atol=5e-2)


@pytest.mark.parametrize("T,I,O", [(512, 256, 384), (2048, 1024, 1024)])
def test_dw_transposed_with_bias_grad(T, I, O):
    # dW^T [O, I] = dY^T X, db = colsum(dY) (reduction of op(a) = dY^T over K = T)
    x, dy = _r(T, I), _r(T, O)
    db = torch.zeros(O, device="cuda")
    dwt = K.blaslt_gemm(dy, x, trans_a=True, epilogue=K.EPI_BGRADB, bias=db)
    torch.testing.assert_close(dwt.float(), dy.float().t() @ x.float(), rtol=2e-2, atol=0.3)
    torch.testing.assert_close(db, dy.float().sum(0), rtol=1e-2, atol=0.1)


def test_probe_reports_support():
    import flexflow_train_amd._ffkernels as k
    assert k.blaslt_probe(1024, 1024, 512, False, False, 4, 14, -1, 0) > 0   # BIAS, bf16 bias


@pytest.mark.parametrize("ta,tb", [(False, False), (True, False), (False, True)])
def test_every_heuristic_candidate_matches(ta, tb):
    # the GEMM autotuner times hipBLASLt's candidates; each must compute the same
    # product, including row-strided operand views, fp32 output and beta = 1
    M, N, Kd = 384, 512, 256
    a = _r(Kd, M + 8)[:, :M] if ta else _r(M, Kd + 8)[:, :Kd]
    b = _r(N, Kd) if tb else _r(Kd, N)
    A = a.float().t() if ta else a.float()
    B = b.float().t() if tb else b.float()
    bias = _r(N)
    out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    n = K.blaslt_num_algos(a, b, ta, tb, out, 0.0, True)
    assert n >= 1
    for i in range(n):
        K.blaslt_matmul(a, b, ta, tb, out, 0.0, bias, algo=i)
        torch.testing.assert_close(out.float(), A @ B + bias.float(), rtol=2e-2, atol=5e-2)
    acc = torch.ones(M, N, device="cuda")
    n32 = K.blaslt_num_algos(a, b, ta, tb, acc, 1.0)
    for i in range(n32):
        acc.fill_(1.0)
        K.blaslt_matmul(a, b, ta, tb, acc, 1.0, None, algo=i)
        torch.testing.assert_close(acc, A @ B + 1.0, rtol=1e-2, atol=2e-2)


def test_autotuner_lt_candidate_runs():
    from flexflow_train_amd.ops import gemm as G
    a, b, bias = _r(1024, 512), _r(512, 768), _r(768)
    G._CHOICE.clear()
    c = G._candidates(a, b, False, False, bias, "gelu", None)
    lts = [k for k in c if k.startswith("lt:")]
    assert lts, c.keys()
    ref = F.gelu(a.float() @ b.float() + bias.float(), approximate="tanh")
    for k in lts:
        y = c[k](a, b, False, False, bias, "gelu", None, 0.0, None)
        torch.testing.assert_close(y.float(), ref, rtol=2e-2, atol=5e-2)
