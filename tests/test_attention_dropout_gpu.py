"""Fused attention-probability dropout (csrc/kernels/attention.hip, DROP kernels) against an
fp32 PyTorch oracle that applies the SAME counter-hash mask (ops/attention.py
dropout_keep_mask), forward and all three input gradients; plus the (q/k 192, v 128) MLA
head-dim pair run without padding."""
import math

import pytest
import torch

from solvingpapers_amd.ops import _ext
from solvingpapers_amd.ops.attention import _materialised, dropout_keep_mask, flash_attention

pytestmark = pytest.mark.gpu
DEV = "cuda"


def rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / b.norm().clamp_min(1e-12)).item()


@pytest.mark.parametrize("B,T,H,Hkv,hd,causal,p", [
    (2, 256, 1, 1, 256, True, 0.1),      # GPT-ref: one 256-wide head
    (2, 200, 8, 1, 64, True, 0.1),       # DeepSeek-ref: heads share one latent (MQA-like), ragged
    (1, 300, 4, 2, 128, True, 0.3),      # GQA
    (2, 197, 3, 3, 64, False, 0.5),      # non-causal
])
def test_fused_dropout_matches_masked_oracle(B, T, H, Hkv, hd, causal, p):
    assert _ext.load()
    torch.manual_seed(0)
    q = torch.randn(B, T, H, hd, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    k = torch.randn(B, T, Hkv, hd, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    v = torch.randn(B, T, Hkv, hd, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    seed = 123456789012345
    sc = 1.0 / math.sqrt(hd)
    o = flash_attention(q, k, v, causal, sc, dropout_p=p, seed=seed)
    do = torch.randn_like(o)
    o.backward(do)
    qf, kf, vf = (t.detach().float().requires_grad_() for t in (q, k, v))
    of = _materialised(qf, kf, vf, causal, sc, p, seed)
    of.backward(do.float())
    assert rel(o, of) < 2e-2, rel(o, of)
    for a, b in ((q.grad, qf.grad), (k.grad, kf.grad), (v.grad, vf.grad)):
        assert rel(a, b) < 3e-2, rel(a, b)
    # a different seed gives a different mask (the kernel really applies the seeded mask)
    o2 = flash_attention(q.detach(), k.detach(), v.detach(), causal, sc, dropout_p=p, seed=seed + 1)
    assert rel(o2, of) > 5e-2


def test_dropout_mask_statistics():
    m = dropout_keep_mask(987654321, 2, 4, 512, 512, 0.1, device=DEV)
    keep = m.float().mean().item()
    assert abs(keep - 0.9) < 3e-3, keep
    # no row / column structure: per-row keep rates stay near 0.9
    assert m.float().mean(-1).std().item() < 0.03


@pytest.mark.parametrize("Hkv,T", [(4, 300), (1, 256), (16, 1024)])
def test_mla_192_128_unpadded_matches_oracle(Hkv, T):
    """DeepSeek-V3 MLA heads (q/k 128 nope + 64 rope, v 128): the (192, 128) kernels, not the
    zero-padded 256 path; v passed as a strided view of a [.., 128 + 128] up-projection."""
    from solvingpapers_amd.ops import reference as R
    torch.manual_seed(3)
    B, H = 1, 16
    q = torch.randn(B, T, H, 192, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    k = torch.randn(B, T, Hkv, 192, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    kv = torch.randn(B, T, Hkv, 256, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    v = kv.detach()[..., 128:]
    o = flash_attention(q, k, kv[..., 128:], causal=True)    # v strided: 256 per head
    assert o.shape == (B, T, H, 128)
    do = torch.randn_like(o)
    o.backward(do)
    qf, kf, vf = (t.detach().float().requires_grad_() for t in (q, k, v))
    of, _ = R.attention(qf, kf, vf, True)
    of.backward(do.float())
    assert rel(o, of) < 2e-2, rel(o, of)
    for a, b in ((q.grad, qf.grad), (k.grad, kf.grad), (kv.grad[..., 128:], vf.grad)):
        assert a.shape == b.shape and rel(a, b) < 3e-2, rel(a, b)


@pytest.mark.parametrize("B,T,H,Hkv,D,causal", [(4, 128, 2, 1, 768, True), (2, 100, 2, 1, 768, True),
                                                 (2, 70, 4, 2, 512, False), (1, 300, 2, 1, 768, True)])
def test_wide_head_attention_matches_oracle(B, T, H, Hkv, D, causal):
    """Gemma-ref's 768-wide heads (csrc/kernels/attention_wide.hip): forward and every input
    gradient against the fp32 oracle; MQA (two q-heads on one K/V head) and ragged T."""
    from solvingpapers_amd.ops import reference as R
    torch.manual_seed(5)
    q = (torch.randn(B, T, H, D, device=DEV) * 0.5).bfloat16().requires_grad_()
    k = (torch.randn(B, T, Hkv, D, device=DEV) * 0.5).bfloat16().requires_grad_()
    v = torch.randn(B, T, Hkv, D, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    sc = 1.0 / math.sqrt(D)
    o = flash_attention(q, k, v, causal, sc)
    do = torch.randn_like(o)
    o.backward(do)
    qf, kf, vf = (t.detach().float().requires_grad_() for t in (q, k, v))
    of, _ = R.attention(qf, kf, vf, causal, sc)
    of.backward(do.float())
    assert rel(o, of) < 2e-2, rel(o, of)
    for a, b in ((q.grad, qf.grad), (k.grad, kf.grad), (v.grad, vf.grad)):
        assert rel(a, b) < 3e-2, rel(a, b)
