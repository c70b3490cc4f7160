"""CPU oracles for the DeepSeek-V3 glue ops added with the fused MLA path (ops/attention.py
split_last, mla_attention; ops/moe.py router_logits): values and gradients against the plain
torch formulations they replace. The GPU forms are checked in tests/test_kernels_gpu.py
(test_mla_attention_fused_matches_composition) and tests/test_moe_gpu.py
(test_router_logits_fp32_output)."""
import math

import torch

from solvingpapers_amd.ops import apply_rope
from solvingpapers_amd.ops import reference as R
from solvingpapers_amd.ops.attention import mla_attention, split_last
from solvingpapers_amd.ops.moe import router_logits


def test_split_last_grads_match_slicing():
    torch.manual_seed(0)
    x = torch.randn(2, 5, 9, dtype=torch.float64, requires_grad=True)
    a, b = split_last(x, 4)
    assert a.is_contiguous() and b.is_contiguous()
    assert torch.equal(a, x[..., :4]) and torch.equal(b, x[..., 4:])
    ga, gb = torch.randn_like(a), torch.randn_like(b)
    (a * ga).sum().backward(retain_graph=True)
    g1 = x.grad.clone()
    x.grad = None
    (b * gb).sum().backward()
    g2 = x.grad.clone()
    assert torch.equal(g1[..., :4], ga) and torch.equal(g1[..., 4:], torch.zeros_like(gb))
    assert torch.equal(g2[..., 4:], gb) and torch.equal(g2[..., :4], torch.zeros_like(ga))
    assert torch.autograd.gradcheck(lambda t: split_last(t, 3), (x.detach().requires_grad_(),))


def test_mla_attention_cpu_matches_manual_composition():
    torch.manual_seed(1)
    B, T, H, dn, dr, dv = 2, 11, 3, 8, 4, 6
    q = torch.randn(B, T, H, dn + dr, dtype=torch.float64, requires_grad=True)
    kv = torch.randn(B, T, H, dn + dv, dtype=torch.float64, requires_grad=True)
    kr = torch.randn(B, T, 1, dr, dtype=torch.float64, requires_grad=True)
    sc = 1 / math.sqrt(dn + dr)
    o = mla_attention(q, kv, kr, dn, sc, 10000.0, 2)
    qf = torch.cat([q[..., :dn], apply_rope(q[..., dn:], 10000.0, 2)], -1)
    k = torch.cat([kv[..., :dn], apply_rope(kr, 10000.0, 2).expand(B, T, H, dr)], -1)
    ref, _ = R.attention(qf, k, kv[..., dn:], True, sc)
    assert torch.allclose(o, ref.to(o.dtype), atol=1e-5)   # the oracle computes in fp32
    # gradients flow to all three inputs (the GPU test compares them with this path)
    o.sum().backward()
    assert all(t.grad is not None and torch.isfinite(t.grad).all() for t in (q, kv, kr))


def test_router_logits_cpu_is_fp32_mm():
    torch.manual_seed(2)
    x = torch.randn(7, 16).bfloat16()
    g = torch.randn(5, 16).bfloat16()
    out = router_logits(x, g)
    assert out.dtype == torch.float32
    assert torch.allclose(out, x.float() @ g.float().t())
