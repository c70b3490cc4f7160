"""FlatParams + fused flat optimizers == torch.optim on the same parameters."""
import copy

import pytest
import torch

from solvingpapers_amd.train.optim import FlatAdam, FlatAdamW, FlatSGD, cosine_lr
from solvingpapers_amd.utils.flat import FlatParams
from solvingpapers_amd.ops.linear import Linear


class Tiny(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.a = Linear(8, 16)
        self.b = torch.nn.Linear(16, 4)   # plain torch module: grads via autograd -> hook path
        self.e = torch.nn.Parameter(torch.randn(3, 4))

    def forward(self, x):
        return (self.b(torch.relu(self.a(x))) * self.e.sum(0)).sum()


@pytest.mark.parametrize("kind", ["adamw", "adam", "sgd"])
def test_flat_optimizer_matches_torch(kind):
    torch.manual_seed(0)
    m1 = Tiny()
    m2 = copy.deepcopy(m1)
    flat = FlatParams(m1)
    from solvingpapers_amd.utils.flat import attach_autograd_grads
    attach_autograd_grads(flat)
    if kind == "adamw":
        o1 = FlatAdamW(flat, lr=1e-2, betas=(0.9, 0.95), weight_decay=0.1)
        o2 = torch.optim.AdamW(m2.parameters(), lr=1e-2, betas=(0.9, 0.95), weight_decay=0.1)
    elif kind == "adam":
        o1 = FlatAdam(flat, lr=1e-2, weight_decay=0.01)
        o2 = torch.optim.Adam(m2.parameters(), lr=1e-2, weight_decay=0.01)
    else:
        o1 = FlatSGD(flat, lr=1e-2, momentum=0.9, weight_decay=0.01)
        o2 = torch.optim.SGD(m2.parameters(), lr=1e-2, momentum=0.9, weight_decay=0.01)
    for _ in range(5):
        x = torch.randn(5, 8)
        o1.zero_grad()
        m1(x).backward()
        o1.step()
        o2.zero_grad()
        m2(x).backward()
        o2.step()
    for p1, p2 in zip(m1.parameters(), m2.parameters()):
        assert torch.allclose(p1, p2, atol=1e-5), (p1 - p2).abs().max()


def test_grad_clip_matches_torch():
    torch.manual_seed(1)
    m1 = Tiny()
    m2 = copy.deepcopy(m1)
    flat = FlatParams(m1)
    from solvingpapers_amd.utils.flat import attach_autograd_grads
    attach_autograd_grads(flat)
    o1 = FlatAdamW(flat, lr=1e-2, weight_decay=0.0, max_grad_norm=0.5)
    o2 = torch.optim.AdamW(m2.parameters(), lr=1e-2, weight_decay=0.0)
    x = torch.randn(5, 8) * 10
    o1.zero_grad(); m1(x).backward(); o1.step()
    o2.zero_grad(); m2(x).backward()
    n = torch.nn.utils.clip_grad_norm_(m2.parameters(), 0.5)
    o2.step()
    assert abs(o1.last_grad_norm.item() - n.item()) < 1e-3 * n.item()
    for p1, p2 in zip(m1.parameters(), m2.parameters()):
        assert torch.allclose(p1, p2, atol=1e-5)


def test_cosine_schedule_matches_reference_formula():
    # deepseekv3/deepseekv3.ipynb:1976-1986, warmup 400, total 10000, max 6e-4, min 6e-5
    assert abs(cosine_lr(0, 6e-4, 400, 10000, 6e-5) - 6e-4 / 401) < 1e-12
    assert abs(cosine_lr(400, 6e-4, 400, 10000, 6e-5) - 6e-4) < 1e-12
    assert abs(cosine_lr(10000, 6e-4, 400, 10000, 6e-5) - 6e-5) < 1e-12
    assert cosine_lr(20000, 6e-4, 400, 10000, 6e-5) == 6e-5


def test_linear_rows_joint_gemm_matches_separate():
    """ops.linear.linear_rows: row-stacked weights that FlatParams placed back to back run as ONE
    product over a joint view (forward, dX, dW into the joint main_grad view, accumulating on a
    second call); weights that are not adjacent fall back to separate products. Same values."""
    import importlib
    L = importlib.import_module("solvingpapers_amd.ops.linear")

    class Two(torch.nn.Module):
        def __init__(self):
            super().__init__()
            g = torch.Generator().manual_seed(0)
            self.a = torch.nn.Parameter(torch.randn(24, 16, generator=g))
            self.b = torch.nn.Parameter(torch.randn(8, 16, generator=g))
            self.c = torch.nn.Parameter(torch.randn(8, 16, generator=g))

    x = torch.randn(5, 16, requires_grad=True)
    grads = {}
    for joint in (True, False):
        m = Two()
        FlatParams(m)
        ws = (m.a, m.b) if joint else (m.a, m.c)      # a, c are not adjacent
        if joint:
            assert L._joint_views(ws) is not None
        else:
            assert L._joint_views(ws) is None
            with torch.no_grad():
                m.c.copy_(m.b)
        from solvingpapers_amd.utils.grad import next_generation
        next_generation()
        xx = x.detach().clone().requires_grad_()
        for _ in range(2):                           # second call accumulates
            y = L.linear_rows(xx, ws)
            assert y.shape == (5, 32)
            (y * torch.arange(32.0)).sum().backward()
        grads[joint] = (y.detach(), xx.grad.clone(), ws[0].main_grad.clone(), ws[1].main_grad.clone())
    for a, b in zip(grads[True], grads[False]):
        assert torch.allclose(a, b, atol=1e-5), (a - b).abs().max()
