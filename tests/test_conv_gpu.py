"""Implicit-GEMM MFMA conv kernels (csrc/kernels/conv.hip) vs the fp32 PyTorch conv2d on the same
bf16-rounded operands: output, input grad, weight grad, bias grad -- AlexNet layer geometries
(padded C=3 input, stride 4, 5x5 / 3x3 pad), a strided data grad, the ViT NCHW patchify, and
channels-last LRN / max-pool / ReLU / dropout chaining through AlexNet."""
import pytest
import torch
import torch.nn.functional as F

from solvingpapers_amd.ops import _ext, misc

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(autouse=True, scope="module")
def _ext_loaded():
    assert _ext.load()


def rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / b.norm().clamp_min(1e-12)).item()


CASES = [  # (N, C, H, W, OC, K, stride, pad, x_grad)
    (2, 3, 227, 227, 96, 11, 4, 1, False),    # AlexNet conv1 (C 3 -> 8 padded NHWC)
    (2, 96, 27, 27, 256, 5, 1, 2, True),      # conv2
    (2, 256, 13, 13, 384, 3, 1, 1, True),     # conv3
    (3, 40, 17, 15, 72, 3, 2, 1, True),       # strided data grad, ragged tiles
    (2, 3, 23, 23, 16, 11, 4, 1, True),       # padded-channel data grad back to NCHW
    (4, 3, 224, 224, 768, 16, 16, 0, False),  # ViT-B/16 patchify: NCHW direct gather
]


@pytest.mark.parametrize("case", CASES)
def test_conv_matches_fp32(case):
    N, C, H, W, OC, K, s, p, xg = case
    g = torch.Generator(device=DEV).manual_seed(0)
    x = torch.randn(N, C, H, W, device=DEV, generator=g).bfloat16().requires_grad_(xg)
    w = (torch.randn(OC, C, K, K, device=DEV, generator=g) / (C * K * K) ** 0.5).bfloat16().requires_grad_()
    b = (torch.randn(OC, device=DEV, generator=g) * 0.1).bfloat16().requires_grad_()
    y = misc.conv2d(x, w, b, s, p)
    assert y.is_contiguous(memory_format=torch.channels_last)      # implicit-GEMM path (NHWC out)
    gy = torch.randn(y.shape, device=DEV, generator=g).bfloat16()
    y.backward(gy)
    xr = x.detach().float().requires_grad_(xg)
    wr, br = w.detach().float().requires_grad_(), b.detach().float().requires_grad_()
    yr = F.conv2d(xr, wr, br, s, p)
    yr.backward(gy.float())
    assert rel(y, yr) < 1e-2
    assert rel(w.grad, wr.grad) < 1e-2
    assert rel(b.grad, br.grad) < 1e-2
    if xg:
        assert rel(x.grad, xr.grad) < 1e-2


def test_patch_embed_tokens():
    g = torch.Generator(device=DEV).manual_seed(1)
    x = torch.randn(3, 3, 64, 48, device=DEV, generator=g).bfloat16()
    w = (torch.randn(64, 3, 16, 16, device=DEV, generator=g) * 0.05).bfloat16().requires_grad_()
    b = torch.zeros(64, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    t = misc.patch_embed(x, w, b, 16)
    ref = F.conv2d(x.float(), w.float(), b.float(), 16).flatten(2).transpose(1, 2)
    assert t.shape == (3, 12, 64) and rel(t, ref) < 1e-2


def test_channels_last_pool_lrn_act_dropout():
    """NHWC kernels give the same values as the NCHW ones, grads included, and keep the layout."""
    g = torch.Generator(device=DEV).manual_seed(2)
    a = torch.randn(2, 24, 13, 11, device=DEV, generator=g).bfloat16()
    outs = {}
    for fmt in (torch.contiguous_format, torch.channels_last):
        x = a.clone(memory_format=fmt).detach().requires_grad_()
        y = misc.max_pool2d(misc.local_response_norm(x, 5), 3, 2)
        assert y.is_contiguous(memory_format=fmt)
        gy = torch.linspace(-1, 1, y.numel(), device=DEV).view(y.shape).bfloat16()
        y.backward(gy)
        outs[fmt] = (y.float(), x.grad.float())
    (y0, g0), (y1, g1) = outs.values()
    assert torch.equal(y0, y1) and rel(g1, g0) < 1e-3
    from solvingpapers_amd.ops import activation
    x = a.clone(memory_format=torch.channels_last).detach().requires_grad_()
    r = activation.relu(x)
    assert r.is_contiguous(memory_format=torch.channels_last) and torch.equal(r, torch.relu(a))
    d = misc.dropout(x, 0.5)
    keep = d != 0
    d.backward(torch.ones_like(d))
    assert torch.equal(x.grad != 0, keep)                              # mask follows storage order


def test_alexnet_bf16_channels_last_matches_fp32():
    from solvingpapers_amd.models import alexnet
    torch.manual_seed(0)
    m = alexnet.AlexNet(10).to(DEV)
    ref = alexnet.AlexNet(10).to(DEV)
    ref.load_state_dict(m.state_dict())
    m = m.bfloat16().eval()
    ref = ref.eval()
    x = torch.randn(2, 3, 224, 224, device=DEV).bfloat16()
    y = m(x)
    feats = x.float()
    for mod in ref.features:                                           # torch fp32 reference path
        if isinstance(mod, torch.nn.Module) and mod.__class__.__name__ == "Conv2d":
            feats = F.conv2d(feats, mod.weight.bfloat16().float(), mod.bias.bfloat16().float(), mod.stride,
                             mod.padding)
        elif mod.__class__.__name__ in ("ReLU", "Activation"):
            feats = torch.relu(feats)
        elif mod.__class__.__name__ == "LocalResponseNorm":
            feats = F.local_response_norm(feats, 5)
        else:
            feats = F.max_pool2d(feats, 3, 2)
    yr = feats.flatten(1)
    for mod in ref.classifier:
        if mod.__class__.__name__ == "Linear":
            yr = F.linear(yr, mod.weight.bfloat16().float(), mod.bias.bfloat16().float())
        elif mod.__class__.__name__ in ("ReLU", "Activation"):
            yr = torch.relu(yr)
    assert rel(y, yr) < 3e-2
    m.train()
    loss = F.cross_entropy(m(x).float(), torch.tensor([1, 2], device=DEV))
    loss.backward()
    assert all(p.grad is not None and torch.isfinite(p.grad.float()).all() for p in m.parameters())
