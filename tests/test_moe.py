"""EXPERTS operator numerics against a plain PyTorch autograd reference
(CPU fp32; the GPU bf16 variant is marked gpu)."""
import pytest
import torch

from flexflow_train_amd.ops import base as opbase


def _reference(x, ids, gate, w1, b1, w2, b2):
    out = torch.zeros(x.shape[0], w2.shape[2], dtype=torch.float32)
    for b in range(x.shape[0]):
        for j in range(ids.shape[1]):
            e = int(ids[b, j])
            h = torch.relu(x[b].float() @ w1[e].float() + b1[e].float())
            out[b] = out[b] + gate[b, j].float() * (h @ w2[e].float() + b2[e].float())
    return out


def _run(dev, dtype, tol):
    torch.manual_seed(0)
    B, D, H, O, E, k = 16, 24, 32, 8, 4, 2
    x = torch.randn(B, D)
    logits = torch.randn(B, E)
    gate_full = torch.softmax(logits, -1)
    vals, ids = torch.topk(gate_full, k, -1)
    w1, b1 = torch.randn(E, D, H) * 0.2, torch.randn(E, H) * 0.1
    w2, b2 = torch.randn(E, H, O) * 0.2, torch.randn(E, O) * 0.1
    leaves = [t.clone().requires_grad_(True) for t in (x, vals, w1, b1, w2, b2)]
    ref = _reference(leaves[0], ids, leaves[1], *leaves[2:])
    dout = torch.randn(B, O)
    ref.backward(dout)

    impl = opbase.get_impl("EXPERTS")
    ctx = opbase.OpContext(op_type="EXPERTS", attrs={"num_experts": E, "hidden_size": H, "out_dim": O,
                                                      "activation": "relu", "use_bias": True}, name="moe")
    to = lambda t: t.to(dev, dtype)  # noqa: E731
    ws = [to(w) for w in (w1, b1, w2, b2)]
    outs, saved = impl.forward(ctx, [to(x), ids.to(dev, torch.int32), to(vals)], ws)
    torch.testing.assert_close(outs[0].float().cpu(), ref.detach(), rtol=tol, atol=tol)
    grads = [torch.zeros(w.shape, device=dev, dtype=torch.float32) for w in ws]
    gins = impl.backward(ctx, saved, [to(dout)], grads, [True, False, True])
    torch.testing.assert_close(gins[0].float().cpu(), leaves[0].grad, rtol=tol, atol=tol)
    assert gins[1] is None
    torch.testing.assert_close(gins[2].float().cpu(), leaves[1].grad, rtol=tol, atol=tol)
    for got, leaf in zip(grads, leaves[2:]):
        if dtype == torch.float32:
            torch.testing.assert_close(got.cpu(), leaf.grad, rtol=tol, atol=tol * 4)
        else:  # bf16 inputs can flip a ReLU near 0: compare in norm
            err = (got.cpu() - leaf.grad).norm() / leaf.grad.norm()
            assert err < 3e-2, err


def test_experts_cpu_fp32():
    _run("cpu", torch.float32, 1e-4)


@pytest.mark.gpu
def test_experts_gpu_bf16():
    _run("cuda", torch.bfloat16, 6e-2)


def test_moe_model_trains():
    from flexflow_train_amd.core import AdamOptimizer, FFConfig, FFModel, LossType, MetricsType
    from flexflow_train_amd.models.moe import MoEConfig, build_moe, moe_synthetic
    import numpy as np

    cfg = MoEConfig(batch_size=32, input_dim=16, num_experts=4, num_select=2, expert_hidden=32, num_classes=4)
    m = FFModel(FFConfig())
    build_moe(m, cfg)
    m.compile(optimizer=AdamOptimizer(m, alpha=1e-2), loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY,
              metrics=[MetricsType.METRICS_ACCURACY])
    feeds, labels = moe_synthetic(cfg, np.random.default_rng(0))
    ex = m.executor
    losses = []
    for _ in range(30):
        ex.train_step({k: torch.from_numpy(v) for k, v in feeds.items()}, torch.from_numpy(labels))
        losses.append(float(ex.perf_metrics().loss))
        ex.zero_metrics()
    assert losses[-1] < losses[0] * 0.7, losses
