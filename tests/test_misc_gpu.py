"""HIP misc kernels (dropout, KD/VAE/MSE losses, LRN, max-pool, conv-as-GEMM,
patch-embed, Luong) vs PyTorch fp32 references."""
import pytest
import torch
import torch.nn.functional as F

from solvingpapers_amd.ops import _ext, misc

pytestmark = pytest.mark.gpu
DEV = "cuda"


def rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / b.norm().clamp_min(1e-12)).item()


@pytest.fixture(autouse=True, scope="module")
def _ext_loaded():
    assert _ext.load()


@pytest.mark.parametrize("shape,off", [((1000, 257), 0), ((1001, 259), 0), ((999, 64), 3)])
def test_dropout_mask_consistency(shape, off):
    """8-wide vector body, scalar tail (numel % 8 != 0) and an unaligned view (scalar path)."""
    base = torch.randn(shape[0] * shape[1] + off, device=DEV)
    # no exact zeros (torch's randn returns 0.0 when its uniform draw is exactly 1, ~1 in 2^24): the
    # kept set is read back as y != 0
    base = torch.where(base == 0, torch.ones_like(base), base)
    x = base[off:].view(shape).detach().requires_grad_(True)
    y = misc.dropout(x, 0.3)
    keep = (y != 0)
    frac = keep.float().mean().item()
    assert 0.65 < frac < 0.75
    assert torch.allclose(y[keep], (x / 0.7)[keep])
    y.backward(torch.ones_like(y))
    assert torch.equal(x.grad != 0, keep)  # same mask regenerated in backward


@pytest.mark.parametrize("C", [10, 16, 33, 100, 1000, 2048, 3000])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_kd_loss(dtype, C):
    """lane-per-row (C <= 16), wave-per-row register-resident (C <= 2048, every VPL bucket) and
    block fallback kernels."""
    s = torch.randn(130, C, device=DEV, dtype=dtype, requires_grad=True)
    t = torch.randn(130, C, device=DEV, dtype=dtype)
    y = torch.randint(0, C, (130,), device=DEV)
    tot, hard, soft = misc.distillation_loss(s, t, y, 7.0, 0.3)
    tot.backward()
    sf = s.detach().float().requires_grad_()
    slp = F.log_softmax(sf / 7, 1)
    tp = F.softmax(t.float() / 7, 1)
    h = F.cross_entropy(sf, y)
    so = F.kl_div(slp, tp, reduction="batchmean") * 49
    ref = 0.3 * h + 0.7 * so
    ref.backward()
    tol = 1e-4 if dtype == torch.float32 else 2e-2
    assert abs(tot.item() - ref.item()) < tol * max(1, abs(ref.item()))
    assert abs(hard.item() - h.item()) < tol * max(1, h.item())
    assert rel(s.grad, sf.grad) < (1e-3 if dtype == torch.float32 else 3e-2)


def test_vae_loss_and_reparam():
    r = torch.rand(64, 784, device=DEV).clamp(0.01, 0.99).requires_grad_()
    x = torch.rand(64, 784, device=DEV)
    mu = torch.randn(64, 128, device=DEV, requires_grad=True)
    lv = (torch.randn(64, 128, device=DEV) * 0.3).requires_grad_()
    loss = misc.vae_loss(r, x, mu, lv)
    loss.backward()
    rf, muf, lvf = (t.detach().clone().requires_grad_() for t in (r, mu, lv))
    ref = F.binary_cross_entropy(rf, x, reduction="sum") - 0.5 * torch.sum(1 + lvf - muf.pow(2) - lvf.exp())
    ref.backward()
    assert abs(loss.item() - ref.item()) < 1e-4 * abs(ref.item())
    assert rel(r.grad, rf.grad) < 1e-4 and rel(mu.grad, muf.grad) < 1e-5 and rel(lv.grad, lvf.grad) < 1e-5
    # reparameterisation: z - mu = eps * std with eps ~ N(0,1)
    mu2 = torch.zeros(4096, 64, device=DEV, requires_grad=True)
    lv2 = torch.zeros(4096, 64, device=DEV, requires_grad=True)
    z = misc.reparameterize(mu2, lv2)
    assert abs(z.mean().item()) < 0.02 and abs(z.std().item() - 1) < 0.02
    z.sum().backward()
    assert torch.all(mu2.grad == 1)
    assert torch.allclose(lv2.grad, 0.5 * z.detach(), atol=1e-6)  # d/dlv = eps * 0.5 * std


def test_mse():
    a = torch.rand(128, 784, device=DEV, requires_grad=True)
    b = torch.rand(128, 784, device=DEV)
    l = misc.mse_loss(a, b)
    l.backward()
    af = a.detach().clone().requires_grad_()
    r = F.mse_loss(af, b)
    r.backward()
    assert abs(l.item() - r.item()) < 1e-6 and rel(a.grad, af.grad) < 1e-6


def test_lrn_maxpool_conv():
    x = torch.randn(2, 16, 13, 13, device=DEV, requires_grad=True)
    xf = x.detach().clone().requires_grad_()
    y = misc.local_response_norm(x, 5)
    yr = F.local_response_norm(xf, 5)
    g = torch.randn_like(y)
    y.backward(g)
    yr.backward(g)
    assert rel(y, yr) < 1e-5 and rel(x.grad, xf.grad) < 1e-4
    x = torch.randn(2, 8, 27, 27, device=DEV, requires_grad=True)
    xf = x.detach().clone().requires_grad_()
    y = misc.max_pool2d(x, 3, 2)
    yr = F.max_pool2d(xf, 3, 2)
    g = torch.randn_like(y)
    y.backward(g)
    yr.backward(g)
    assert torch.equal(y, yr) and rel(x.grad, xf.grad) < 1e-6
    for (C, OC, k, s, p, H) in [(3, 96, 11, 4, 1, 224), (96, 32, 5, 1, 2, 27), (1, 64, 7, 7, 0, 28)]:
        x = torch.randn(2, C, H, H, device=DEV, requires_grad=True)
        w = (torch.randn(OC, C, k, k, device=DEV) * 0.05).requires_grad_()
        b = torch.randn(OC, device=DEV, requires_grad=True)
        y = misc.conv2d(x, w, b, s, p)
        xf, wf, bf = (t.detach().clone().requires_grad_() for t in (x, w, b))
        yr = F.conv2d(xf, wf, bf, s, p)
        g = torch.randn_like(y)
        y.backward(g)
        yr.backward(g)
        assert rel(y, yr) < 1e-4, (C, k)
        assert rel(x.grad, xf.grad) < 1e-4 and rel(w.grad, wf.grad) < 1e-4 and rel(b.grad, bf.grad) < 1e-4


def test_patch_embed_vit_b16():
    x = torch.randn(2, 3, 224, 224, device=DEV, dtype=torch.bfloat16)
    w = torch.randn(768, 3, 16, 16, device=DEV, dtype=torch.bfloat16) * 0.02
    b = torch.randn(768, device=DEV, dtype=torch.bfloat16)
    y = misc.patch_embed(x, w, b, 16)
    yr = F.conv2d(x.float(), w.float(), b.float(), 16).flatten(2).transpose(1, 2)
    assert y.shape == (2, 196, 768) and rel(y, yr) < 1e-2


def test_luong():
    st = torch.randn(4, 32, device=DEV, requires_grad=True)
    hs = torch.randn(4, 50, 32, device=DEV, requires_grad=True)
    c, w = misc.luong_attention(st, hs)
    stf, hsf = st.detach().clone().requires_grad_(), hs.detach().clone().requires_grad_()
    dot = (stf.unsqueeze(1) * hsf).sum(-1)
    wr = torch.softmax(dot, 1).unsqueeze(-1)
    cr = (wr * hsf).sum(1)
    g = torch.randn_like(c)
    c.backward(g)
    cr.backward(g)
    assert rel(c, cr) < 1e-5 and rel(w, wr) < 1e-5
    assert rel(st.grad, stf.grad) < 1e-4 and rel(hs.grad, hsf.grad) < 1e-4


def test_vit_train_step_bf16_matches_fp32_cpu():
    """A ViT (reference layout, 2 blocks of 128 wide, 197 tokens as in ViT-B/16) forward +
    backward on the GPU in bf16 -- HIP kernels throughout, with the residual pair carried through
    the fused LayerNorms and the dW / bias-grad kernels at >= 4096 tokens -- against the same
    model in fp32 on the CPU."""
    import copy
    from solvingpapers_amd.models import vit
    torch.manual_seed(0)
    c = vit.config("vit_b16", embedding_dim=128, attention_heads=2, transformer_blocks=2, mlp_hidden=512,
                   num_classes=10)
    ref = vit.ViT(c)
    gpu = copy.deepcopy(ref).to("cuda", torch.bfloat16)
    x = torch.randn(24, 3, 224, 224)
    y = torch.randint(0, 10, (24,))
    lr = ref(x, y)
    lr.backward()
    lg = gpu(x.to("cuda", torch.bfloat16), y.cuda())
    lg.backward()
    assert abs(lg.item() - lr.item()) < 3e-2 * abs(lr.item()) + 1e-2
    for (n, pr), pg in zip(ref.named_parameters(), gpu.parameters()):
        a, b = pr.grad.float(), pg.grad.float().cpu()
        assert (a - b).norm() <= 6e-2 * a.norm() + 1e-4, n
