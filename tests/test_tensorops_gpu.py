"""Numerics of the general tensor-operator kernels (csrc/kernels/tensorops.hip)
against plain PyTorch fp32 references, plus the CPU mirror of the
counter-based initialiser.

Parity: reference kernel tests under lib/kernels/test/src/test_*_kernel.cc
(concat, split, reverse, gather, reduction, transpose, element-wise).
"""
import math

import numpy as np
import pytest
import torch

from flexflow_train_amd.runtime.initializers import counter_init_piece, counter_spec

gpu = pytest.mark.gpu


def _K():
    from flexflow_train_amd import kernels as K
    assert K.available(), "HIP kernel extension must be loaded on a GPU box"
    return K


def _close(a, b, dtype, rtol=None, atol=None):
    tol = {torch.float32: (1e-5, 1e-5), torch.bfloat16: (2e-2, 2e-2)}[dtype]
    torch.testing.assert_close(a.float(), b.float(), rtol=rtol or tol[0], atol=atol or tol[1])


# ---------------------------------------------------------------- CPU tests
def test_counter_init_is_layout_independent():
    spec = counter_spec({"type": "glorot_uniform"}, (24, 40))
    full = counter_init_piece(spec, (24, 40), [(0, 24), (0, 40)], 1234, "cpu")
    piece = counter_init_piece(spec, (24, 40), [(8, 16), (10, 30)], 1234, "cpu")
    assert torch.equal(full[8:16, 10:30], piece)
    b = math.sqrt(6.0 / 64)
    assert full.abs().max() <= b and full.std() > b / 3


def test_counter_init_distributions():
    n = 1 << 16
    x = counter_init_piece(counter_spec({"type": "normal", "mean": 1.0, "stddev": 2.0}, (n,)), (n,), [(0, n)], 7,
                           "cpu")
    assert abs(x.mean().item() - 1.0) < 0.05 and abs(x.std().item() - 2.0) < 0.05
    t = counter_init_piece(counter_spec({"type": "truncated_normal", "stddev": 1.0}, (n,)), (n,), [(0, n)], 7, "cpu")
    assert t.min() >= -2.0 and t.max() <= 2.0 and 0.8 < t.std().item() < 0.92
    c = counter_init_piece(counter_spec({"type": "constant", "value": 3.5}, (5, 3)), (5, 3), [(0, 5), (0, 3)], 7,
                           "cpu")
    assert torch.all(c == 3.5)


# ---------------------------------------------------------------- GPU tests
DT = [torch.float32, torch.bfloat16]
BCAST = [((4, 8, 16), (4, 8, 16)), ((4, 8, 16), (16,)), ((4, 1, 16), (1, 8, 1)), ((2, 3, 4, 5), (3, 1, 5)),
         ((7,), (1,))]


@gpu
@pytest.mark.parametrize("dtype", DT)
@pytest.mark.parametrize("shapes", BCAST)
@pytest.mark.parametrize("op", ["EW_ADD", "EW_SUB", "EW_MUL", "EW_DIV", "EW_MAX", "EW_MIN"])
def test_binary_broadcast_fwd_bwd(dtype, shapes, op):
    K = _K()
    torch.manual_seed(0)
    a = torch.randn(shapes[0], device="cuda").to(dtype)
    b = torch.randn(shapes[1], device="cuda").to(dtype)
    if op == "EW_DIV":
        b = b.sign().to(dtype) * (b.abs() + 0.5).to(dtype)
    fn = {"EW_ADD": torch.add, "EW_SUB": torch.sub, "EW_MUL": torch.mul, "EW_DIV": torch.div,
          "EW_MAX": torch.maximum, "EW_MIN": torch.minimum}[op]
    af, bf = a.float().requires_grad_(True), b.float().requires_grad_(True)
    ref = fn(af, bf)
    y = K.binary(a, b, op)
    _close(y, ref, dtype)
    dy = torch.randn(ref.shape, device="cuda").to(dtype)
    ref.backward(dy.float())
    ga = K.binary_grad(dy, a, b, op, 0)
    gb = K.binary_grad(dy, a, b, op, 1)
    assert ga.shape == a.shape and gb.shape == b.shape
    _close(ga, af.grad, dtype, rtol=3e-2 if dtype == torch.bfloat16 else 1e-4, atol=5e-2 if dtype == torch.bfloat16 else 1e-4)
    _close(gb, bf.grad, dtype, rtol=3e-2 if dtype == torch.bfloat16 else 1e-4, atol=1e-1 if dtype == torch.bfloat16 else 1e-4)


@gpu
@pytest.mark.parametrize("op,fn", [("EW_EQUAL", torch.eq), ("EW_GREATER", torch.gt), ("EW_LESS", torch.lt)])
def test_binary_compare(op, fn):
    K = _K()
    a = torch.randint(0, 3, (6, 5), device="cuda").float()
    b = torch.randint(0, 3, (5,), device="cuda").float()
    torch.testing.assert_close(K.binary(a, b, op), fn(a, b).float())


@gpu
@pytest.mark.parametrize("dtype", DT)
@pytest.mark.parametrize("shape,perm", [((4, 5, 6), (2, 0, 1)), ((2, 3, 4, 5), (0, 2, 1, 3)), ((8, 16), (1, 0)),
                                        ((2, 3, 4, 5, 6, 2), (5, 4, 3, 2, 1, 0))])
def test_permute(dtype, shape, perm):
    K = _K()
    x = torch.randn(shape, device="cuda").to(dtype)
    assert torch.equal(K.permute(x, perm), x.permute(perm).contiguous())


@gpu
@pytest.mark.parametrize("dtype", DT)
@pytest.mark.parametrize("axis", [0, 1, 2, -1])
def test_concat_split_reverse(dtype, axis):
    K = _K()
    xs = [torch.randn(3, 4, 5, device="cuda").to(dtype) for _ in range(2)]
    xs.append(torch.randn([3, 4, 5][:axis % 3] + [2] + [3, 4, 5][axis % 3 + 1:], device="cuda").to(dtype))
    y = K.concat(xs, axis)
    assert torch.equal(y, torch.cat(xs, axis))
    sizes = [int(x.shape[axis]) for x in xs]
    for a, b in zip(K.split(y, sizes, axis), torch.split(y, sizes, axis)):
        assert torch.equal(a, b.contiguous())
    assert torch.equal(K.reverse(y, axis), torch.flip(y, [axis]))


@gpu
@pytest.mark.parametrize("axis", [0, 1])
def test_concat_split_many_pieces(axis):
    """More pieces than one launch carries (16): chunked multi-piece copies,
    pieces of different lengths (DLRM's interaction concat has 9)."""
    K = _K()
    xs = []
    for i in range(21):
        shp = [6, 8]
        shp[axis] = 1 + i % 4
        xs.append(torch.randn(shp, device="cuda").to(torch.bfloat16))
    y = K.concat(xs, axis)
    assert torch.equal(y, torch.cat(xs, axis))
    sizes = [int(x.shape[axis]) for x in xs]
    for a, b in zip(K.split(y, sizes, axis), torch.split(y, sizes, axis)):
        assert torch.equal(a, b.contiguous())


@gpu
@pytest.mark.parametrize("dtype", DT)
@pytest.mark.parametrize("dim", [0, 1, 2])
@pytest.mark.parametrize("ibits", [torch.int32, torch.int64])
def test_gather_scatter(dtype, dim, ibits):
    K = _K()
    x = torch.randn(4, 6, 5, device="cuda").to(dtype)
    ishape = [4, 6, 5]
    ishape[dim] = 3
    idx = torch.randint(0, x.shape[dim], ishape, device="cuda", dtype=ibits)
    y = K.gather(x, idx, dim)
    assert torch.equal(y, torch.gather(x, dim, idx.long()))
    dy = torch.randn(ishape, device="cuda").to(dtype)
    dx = K.scatter_add(dy, idx, dim, list(x.shape))
    ref = torch.zeros(x.shape, device="cuda").scatter_add_(dim, idx.long(), dy.float())
    torch.testing.assert_close(dx, ref, rtol=1e-5, atol=1e-5)


@gpu
@pytest.mark.parametrize("dtype", DT)
@pytest.mark.parametrize("op", ["sum", "mean", "max", "min", "prod"])
@pytest.mark.parametrize("rng", [(0, 0), (1, 1), (2, 2), (1, 2), (0, 2)])
def test_reduce(dtype, op, rng):
    K = _K()
    x = (torch.rand(5, 7, 9, device="cuda") + 0.5).to(dtype)
    dims = tuple(range(rng[0], rng[1] + 1))
    xf = x.float()
    if op == "sum":
        ref = xf.sum(dims)
    elif op == "mean":
        ref = xf.mean(dims)
    elif op == "max":
        ref = xf.amax(dims)
    elif op == "min":
        ref = xf.amin(dims)
    else:
        ref = xf
        for d in sorted(dims, reverse=True):
            ref = ref.prod(d)
    y = K.reduce_contig(x, rng[0], rng[1], op)
    _close(y, ref, dtype, rtol=1e-4 if dtype == torch.float32 else 3e-2, atol=1e-4 if dtype == torch.float32 else 3e-2)


@gpu
@pytest.mark.parametrize("dtype", DT)
@pytest.mark.parametrize("n,k", [(10, 1), (100, 5), (1000, 16), (4096, 64)])
def test_topk(dtype, n, k):
    K = _K()
    x = torch.randn(13, n, device="cuda")
    x = x.to(dtype)
    v, i = K.topk(x, k)
    rv, _ = torch.topk(x.float(), k, dim=-1)
    torch.testing.assert_close(v.float(), rv)
    torch.testing.assert_close(torch.gather(x, -1, i).float(), rv)


@gpu
@pytest.mark.parametrize("dtype", DT)
@pytest.mark.parametrize("op,scalar", [("SCALAR_ADD", 1.5), ("SCALAR_SUB", 0.5), ("SCALAR_MULTIPLY", -2.0),
                                       ("SCALAR_TRUE_DIV", 4.0), ("POW", 3.0), ("LOG", 0.0), ("SQRT", 0.0),
                                       ("RSQRT", 0.0), ("SIN", 0.0), ("COS", 0.0), ("LEAKYRELU", 0.1),
                                       ("CEIL", 0.0), ("ROUND", 0.0), ("IDENTITY", 0.0)])
def test_unary(dtype, op, scalar):
    K = _K()
    torch.manual_seed(1)
    x = torch.randn(1000, device="cuda") * 3
    if op in ("LOG", "SQRT", "RSQRT"):
        x = x.abs() + 0.1
    x = x.to(dtype)
    xf = x.float().requires_grad_(True)
    F = torch.nn.functional
    ref = {"SCALAR_ADD": lambda t: t + scalar, "SCALAR_SUB": lambda t: t - scalar,
           "SCALAR_MULTIPLY": lambda t: t * scalar, "SCALAR_TRUE_DIV": lambda t: t / scalar,
           "POW": lambda t: t ** scalar, "LOG": torch.log, "SQRT": torch.sqrt, "RSQRT": torch.rsqrt,
           "SIN": torch.sin, "COS": torch.cos, "LEAKYRELU": lambda t: F.leaky_relu(t, scalar),
           "CEIL": torch.ceil, "ROUND": torch.round, "IDENTITY": lambda t: t}[op](xf)
    y = K.unary(x, op, scalar)
    tol = (1e-4, 1e-4) if dtype == torch.float32 else (2e-2, 5e-2)
    torch.testing.assert_close(y.float(), ref, rtol=tol[0], atol=tol[1] * (1 + ref.abs().max().item() / 10))
    dy = torch.randn(1000, device="cuda").to(dtype)
    ref.backward(dy.float())
    gx = K.unary(x, op, scalar, dy=dy)
    torch.testing.assert_close(gx.float(), xf.grad, rtol=tol[0] * 3,
                               atol=tol[1] * (1 + xf.grad.abs().max().item() / 10))


@gpu
@pytest.mark.parametrize("dtype", DT)
def test_mse(dtype):
    K = _K()
    p = torch.randn(37, 19, device="cuda").to(dtype)
    y = torch.randn(37, 19, device="cuda").to(dtype)
    g = torch.empty_like(p)
    m = torch.zeros(2, device="cuda")
    K.mse(p, y, g, m, 0.25)
    d = p.float() - y.float()
    _close(g, 0.25 * d, dtype)
    torch.testing.assert_close(m[0], (d * d).sum(), rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(m[1], d.abs().sum(), rtol=1e-4, atol=1e-3)


@gpu
@pytest.mark.parametrize("init", [{"type": "uniform", "min": -0.3, "max": 0.7}, {"type": "glorot_uniform"},
                                  {"type": "normal", "mean": 0.1, "stddev": 0.5}, {"type": "truncated_normal"},
                                  {"type": "constant", "value": -1.25}, {"type": "zero"}])
def test_init_gpu_matches_cpu_mirror(init):
    _K()
    full = (64, 48)
    box = [(16, 48), (8, 40)]
    spec = counter_spec(init, full)
    g = counter_init_piece(spec, full, box, 99, "cuda")
    c = counter_init_piece(spec, full, box, 99, "cpu")
    assert g.shape == (32, 32)
    torch.testing.assert_close(g.cpu(), c, rtol=1e-4, atol=1e-4)
    whole = counter_init_piece(spec, full, [(0, 64), (0, 48)], 99, "cuda")
    assert torch.equal(whole[16:48, 8:40], g)
