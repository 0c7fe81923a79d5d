"""flexflow.torch.compile: a PyTorch module trained by an ordinary PyTorch
loop (loss.backward(); optimizer.step()) while its forward / backward run on
the FlexFlow executor (reference: the designed torch.compile flow of
docs/plantuml/figures/pytorch-tracing.puml — design only in the reference).
Parity: losses and parameter gradients against the same module run eagerly."""
import pytest
import torch
import torch.nn as nn

import flexflow.torch as fft
from test_frontends import SmallCNN, TinyAttn


class MLP(nn.Module):
    def __init__(self):
        super().__init__()
        self.fc1 = nn.Linear(16, 32)
        self.fc2 = nn.Linear(32, 5)

    def forward(self, x):
        return self.fc2(torch.relu(self.fc1(x)))


class SmoothMLP(MLP):
    """tanh instead of ReLU: bf16 rounding cannot flip an activation mask
    (a flipped ReLU unit changes that unit's gradients wholesale)."""

    def forward(self, x):
        return self.fc2(torch.tanh(self.fc1(x)))


CASES = {
    "mlp": (MLP, lambda: torch.randn(8, 16), 5, False),
    "smooth_mlp": (SmoothMLP, lambda: torch.randn(8, 16), 5, False),
    "cnn": (SmallCNN, lambda: torch.randn(4, 3, 8, 8), 10, True),
    "attention": (TinyAttn, lambda: torch.randn(2, 6, 16), 5, True),
}


def _loss(out, y, probs):
    if probs:   # the module ends in softmax: NLL of its probabilities
        return nn.functional.nll_loss(torch.log(out.reshape(-1, out.shape[-1]) + 1e-9), y.reshape(-1))
    return nn.functional.cross_entropy(out, y)


def _run(case, device, steps=3):
    cls, mk, ncls, probs = CASES[case]
    torch.manual_seed(0)
    net, ref = cls(), cls()
    ref.load_state_dict(net.state_dict())
    x = mk()
    y = torch.randint(0, ncls, x.shape[:-1] if case == "attention" else x.shape[:1])
    from flexflow.core import FFConfig
    cfg = FFConfig()
    cfg.cpu_only = device == "cpu"     # on a GPU box the CPU case still runs the host executor
    cm = fft.compile(net, [x.to(device)], ffconfig=cfg)
    o_ff, o_ref = cm(x.to(device)).cpu(), ref(x)
    opt = torch.optim.SGD(net.parameters(), lr=0.1, momentum=0.9)
    opt_r = torch.optim.SGD(ref.parameters(), lr=0.1, momentum=0.9)
    losses, gerr = [], []
    for _ in range(steps):
        lf = _loss(cm(x.to(device)).cpu(), y, probs)
        lr_ = _loss(ref(x), y, probs)
        lf.backward()
        lr_.backward()
        losses.append((lf.item(), lr_.item()))
        for p, q in zip(net.parameters(), ref.parameters()):
            gerr.append(((p.grad.cpu() - q.grad).abs().max() / (q.grad.abs().max() + 1e-6)).item())
        opt.step()
        opt_r.step()
        opt.zero_grad()
        opt_r.zero_grad()
    return o_ff, o_ref, losses, gerr


@pytest.mark.parametrize("case", list(CASES))
def test_compiled_module_trains_like_eager(case):
    o_ff, o_ref, losses, gerr = _run(case, "cpu")
    torch.testing.assert_close(o_ff, o_ref, rtol=1e-4, atol=1e-5)
    for a, b in losses:
        assert abs(a - b) <= 1e-4 * max(1.0, abs(b)), losses
    assert max(gerr) < 1e-3, gerr


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["smooth_mlp", "attention"])
def test_compiled_module_trains_like_eager_gpu(case):
    """On the GPU the executor computes in bf16 (HIP kernels): same training
    trajectory within bf16 tolerance."""
    o_ff, o_ref, losses, gerr = _run(case, "cuda")
    torch.testing.assert_close(o_ff, o_ref, rtol=5e-2, atol=5e-2)
    for a, b in losses:
        assert abs(a - b) <= 5e-2 * max(1.0, abs(b)), losses
    assert max(gerr) < 0.1, gerr


@pytest.mark.parametrize("case", ["mlp", "cnn"])
def test_dynamo_backend_trains_like_eager(case):
    """torch.compile(model, backend="flexflow"): dynamo's flat graph
    (parameters as placeholders) is rebound to modules sharing the user's
    Parameters and compiled onto the executor; an ordinary PyTorch loop
    trains it like eager PyTorch."""
    import warnings

    from flexflow_train_amd.frontends import torch_compile as TC

    cls, mk, ncls, probs = CASES[case]
    torch.manual_seed(0)
    net, ref = cls(), cls()
    ref.load_state_dict(net.state_dict())
    x = mk()
    y = torch.randint(0, ncls, x.shape[:1])
    torch._dynamo.reset()
    assert "flexflow" in torch._dynamo.list_backends()
    before = len(TC.COMPILED)
    # "flexflow" is the registered name; the configured form pins the host
    # executor so the fp32 comparison holds on a GPU box too
    f = torch.compile(net, backend=fft.backend(cpu_only=True))
    opt = torch.optim.SGD(net.parameters(), lr=0.1)
    opt_r = torch.optim.SGD(ref.parameters(), lr=0.1)
    with warnings.catch_warnings():
        warnings.simplefilter("error")      # no eager fallback
        for _ in range(3):
            lf = _loss(f(x), y, probs)
            lr_ = _loss(ref(x), y, probs)
            lf.backward()
            lr_.backward()
            opt.step()
            opt_r.step()
            opt.zero_grad()
            opt_r.zero_grad()
            assert abs(lf.item() - lr_.item()) <= 1e-4 * max(1.0, abs(lr_.item()))
    assert len(TC.COMPILED) > before, "the flexflow backend compiled nothing"


@pytest.mark.gpu
def test_dynamo_backend_on_gpu():
    """backend="flexflow" on a GPU: the graph runs on the HIP executor (bf16)."""
    from flexflow_train_amd.frontends import torch_compile as TC

    torch.manual_seed(0)
    net, ref = SmoothMLP().cuda(), SmoothMLP().cuda()
    ref.load_state_dict(net.state_dict())
    x = torch.randn(8, 16, device="cuda")
    y = torch.randint(0, 5, (8,), device="cuda")
    torch._dynamo.reset()
    before = len(TC.COMPILED)
    f = torch.compile(net, backend="flexflow")
    opt = torch.optim.SGD(net.parameters(), lr=0.1)
    opt_r = torch.optim.SGD(ref.parameters(), lr=0.1)
    for _ in range(3):
        lf = nn.functional.cross_entropy(f(x), y)
        lr_ = nn.functional.cross_entropy(ref(x), y)
        lf.backward()
        lr_.backward()
        opt.step()
        opt_r.step()
        opt.zero_grad()
        opt_r.zero_grad()
        assert abs(lf.item() - lr_.item()) <= 5e-2 * max(1.0, abs(lr_.item()))
    assert len(TC.COMPILED) > before
    assert TC.COMPILED[-1].ex.cfg.device.type == "cuda"


def _cpu_cfg():
    from flexflow.core import FFConfig
    cfg = FFConfig()
    cfg.cpu_only = True
    return cfg


def test_two_forwards_before_one_backward():
    """loss = f(x1) + f(x2): each compiled call keeps its own saved
    activations until its backward, as eager autograd does."""
    torch.manual_seed(0)
    net, ref = SmoothMLP(), SmoothMLP()
    ref.load_state_dict(net.state_dict())
    x1, x2 = torch.randn(8, 16), torch.randn(8, 16)
    y1, y2 = torch.randint(0, 5, (8,)), torch.randint(0, 5, (8,))
    cm = fft.compile(net, [x1], ffconfig=_cpu_cfg())
    ce = nn.functional.cross_entropy
    lf = ce(cm(x1), y1) + 0.5 * ce(cm(x2), y2)
    lr_ = ce(ref(x1), y1) + 0.5 * ce(ref(x2), y2)
    lf.backward()
    lr_.backward()
    assert abs(lf.item() - lr_.item()) <= 1e-5
    for p, q in zip(net.parameters(), ref.parameters()):
        torch.testing.assert_close(p.grad, q.grad, rtol=1e-4, atol=1e-6)


class DropMLP(nn.Module):
    def __init__(self):
        super().__init__()
        self.fc1 = nn.Linear(16, 32)
        self.drop = nn.Dropout(0.5)
        self.fc2 = nn.Linear(32, 5)

    def forward(self, x):
        return self.fc2(self.drop(torch.tanh(self.fc1(x))))


def test_eval_mode_and_no_grad_follow_eager():
    """module.eval() turns dropout off; torch.no_grad() saves nothing and
    returns a tensor without a graph."""
    torch.manual_seed(0)
    net, ref = DropMLP(), DropMLP()
    ref.load_state_dict(net.state_dict())
    x = torch.randn(8, 16)
    cm = fft.compile(net, [x], ffconfig=_cpu_cfg())
    net.eval()
    ref.eval()
    torch.testing.assert_close(cm(x), ref(x), rtol=1e-4, atol=1e-5)
    with torch.no_grad():
        out = cm(x)
    assert not out.requires_grad
    torch.testing.assert_close(out, ref(x).detach(), rtol=1e-4, atol=1e-5)
    assert cm.ex._saved == {}
    net.train()
    assert not torch.allclose(cm(x), ref(x))     # training mode: dropout active
