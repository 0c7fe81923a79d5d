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
