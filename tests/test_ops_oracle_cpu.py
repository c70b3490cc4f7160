"""T0: the CPU oracles every HIP kernel is tested against, checked
themselves — against independent PyTorch formulations on Hypothesis-generated shapes, and
with fp64 ``gradcheck`` for the ops whose CPU path is plain autograd (KD loss, VAE loss,
MSE, Luong attention, LRN, max-pool, conv2d, patch-embed)."""
import math

import pytest
import torch
import torch.nn.functional as F
from hypothesis import given, settings, strategies as st
from torch.autograd import gradcheck

from solvingpapers_amd.ops import misc, reference as R

SET = settings(max_examples=20, deadline=None)
F64 = dict(dtype=torch.float64)


def close(a, b, tol=1e-5):
    return torch.allclose(a.double(), b.double(), atol=tol, rtol=tol)


# ----------------------------------------------------------------------- oracle properties
@SET
@given(n=st.integers(1, 9), d=st.integers(1, 40), eps=st.sampled_from([1e-6, 1e-5]))
def test_rms_norm_oracle(n, d, eps):
    x, w = torch.randn(n, d), torch.randn(d)
    y, h = R.rms_norm(x, w, eps)
    assert close(y, F.rms_norm(x, (d,), w, eps)) and h is x
    r = torch.randn(n, d)
    y2, h2 = R.rms_norm(x, w, eps, residual=r)
    assert close(h2, x + r) and close(y2, F.rms_norm(x + r, (d,), w, eps))


@SET
@given(n=st.integers(1, 9), d=st.integers(2, 40))
def test_layer_norm_oracle(n, d):
    x, w, b = torch.randn(n, d), torch.randn(d), torch.randn(d)
    y, _ = R.layer_norm(x, w, b, 1e-5)
    mu, var = x.mean(-1, keepdim=True), x.var(-1, unbiased=False, keepdim=True)
    assert close(y, (x - mu) / torch.sqrt(var + 1e-5) * w + b, 1e-4)


@SET
@given(kind=st.sampled_from(["relu", "leaky_relu", "elu", "gelu_tanh", "gelu", "silu", "sigmoid", "tanh"]),
       n=st.integers(1, 64), alpha=st.floats(0.01, 1.0))
def test_activation_oracle(kind, n, alpha):
    x = torch.linspace(-10, 10, n)
    want = {"relu": F.relu(x), "leaky_relu": F.leaky_relu(x, alpha), "elu": F.elu(x, alpha),
            "gelu_tanh": F.gelu(x, approximate="tanh"), "gelu": F.gelu(x), "silu": F.silu(x),
            "sigmoid": torch.sigmoid(x), "tanh": torch.tanh(x)}[kind]
    assert close(R.act(x, kind, alpha), want, 1e-5)


@SET
@given(n=st.integers(1, 8), f=st.integers(1, 24), kind=st.sampled_from(["silu", "gelu", "gelu_tanh"]))
def test_glu_oracle(n, f, kind):
    gu = torch.randn(n, 2 * f)
    g, u = gu[:, :f], gu[:, f:]
    act = {"silu": F.silu, "gelu": F.gelu, "gelu_tanh": lambda t: F.gelu(t, approximate="tanh")}[kind]
    assert close(R.glu(gu, kind), act(g) * u)


@SET
@given(T=st.integers(1, 12), H=st.integers(1, 3), hd=st.sampled_from([2, 4, 8, 16]),
       off=st.integers(0, 5), theta=st.sampled_from([10000.0, 500000.0]))
def test_rope_oracle_is_complex_rotation(T, H, hd, off, theta):
    x = torch.randn(1, T, H, hd)
    cos, sin = R.rope_tables(T + off, hd, theta)
    y = R.rope(x, cos, sin, off, interleaved=True)
    freqs = 1.0 / theta ** (torch.arange(0, hd, 2, dtype=torch.float64) / hd)
    ang = torch.outer(torch.arange(off, off + T, dtype=torch.float64), freqs)
    z = torch.view_as_complex(x.double().reshape(1, T, H, hd // 2, 2).contiguous())
    want = torch.view_as_real(z * torch.polar(torch.ones_like(ang), ang)[None, :, None]).flatten(-2)
    assert close(y, want, 1e-5)
    assert close(R.rope(y, cos, sin, off, interleaved=True, inverse=True), x, 1e-5)


@SET
@given(B=st.integers(1, 2), Tq=st.integers(1, 9), extra=st.integers(0, 6), Hkv=st.integers(1, 2),
       rep=st.integers(1, 3), hd=st.sampled_from([4, 8]), causal=st.booleans())
def test_attention_oracle_vs_sdpa(B, Tq, extra, Hkv, rep, hd, causal):
    Tk, H = Tq + extra, Hkv * rep
    q, k, v = torch.randn(B, Tq, H, hd), torch.randn(B, Tk, Hkv, hd), torch.randn(B, Tk, Hkv, hd)
    o, lse = R.attention(q, k, v, causal)
    qh = q.transpose(1, 2)
    kh = k.repeat_interleave(rep, dim=2).transpose(1, 2)
    vh = v.repeat_interleave(rep, dim=2).transpose(1, 2)
    mask = None
    if causal:      # bottom-right aligned: query i sees keys j <= i + Tk - Tq
        mask = torch.arange(Tk)[None, :] <= torch.arange(Tq)[:, None] + (Tk - Tq)
    want = F.scaled_dot_product_attention(qh, kh, vh, attn_mask=mask).transpose(1, 2)
    assert close(o, want, 1e-5)
    s = qh @ kh.transpose(-1, -2) / math.sqrt(hd)
    if causal:
        s = s.masked_fill(~mask, float("-inf"))
    assert close(lse, torch.logsumexp(s, -1), 1e-5)


@SET
@given(n=st.integers(1, 16), V=st.integers(2, 50), sm=st.sampled_from([0.0, 0.1]))
def test_cross_entropy_oracle(n, V, sm):
    lg, t = torch.randn(n, V), torch.randint(0, V, (n,))
    t[0] = -100
    got = R.cross_entropy(lg, t, smoothing=sm)
    lp = torch.log_softmax(lg.double(), -1)
    want = -(1 - sm) * lp.gather(1, t.clamp(min=0)[:, None])[:, 0] - sm * lp.mean(-1)
    want[0] = 0.0
    assert close(got, want, 1e-5)


@SET
@given(V=st.integers(2, 30), D=st.integers(1, 16), T=st.integers(1, 8), scale=st.sampled_from([1.0, 3.5]))
def test_embedding_oracle(V, D, T, scale):
    W, idx, pos = torch.randn(V, D), torch.randint(0, V, (2, T)), torch.randn(T, D)
    assert close(R.embedding(W, idx, pos, scale), F.embedding(idx, W) * scale + pos)


@SET
@given(n=st.integers(1, 64), steps=st.integers(1, 3), wd=st.sampled_from([0.0, 0.1]))
def test_adamw_oracle_matches_torch(n, steps, wd):
    p0 = torch.randn(n)
    ref = torch.nn.Parameter(p0.clone())
    opt = torch.optim.AdamW([ref], lr=1e-2, betas=(0.9, 0.95), eps=1e-8, weight_decay=wd)
    p, master, m, v = p0.clone(), p0.clone(), torch.zeros(n), torch.zeros(n)
    for s in range(1, steps + 1):
        g = torch.randn(n)
        ref.grad = g.clone()
        opt.step()
        R.adamw_(p, master, g, m, v, 1e-2, 0.9, 0.95, 1e-8, wd, s)
    assert close(master, ref.detach(), 1e-5)


# --------------------------------------------------------------------- fp64 gradcheck
def _req(*shape, lo=None):
    t = torch.rand(*shape, **F64) * 0.9 + 0.05 if lo else torch.randn(*shape, **F64)
    return t.requires_grad_()


@pytest.mark.parametrize("name", ["kd", "vae", "mse", "luong", "lrn", "maxpool", "conv2d", "patch_embed"])
def test_gradcheck_fp64(name):
    torch.manual_seed(0)
    if name == "kd":
        t, y = torch.randn(4, 5, **F64), torch.randint(0, 5, (4,))
        fn, args = (lambda s: misc.distillation_loss(s, t, y, 3.0, 0.3)[0]), (_req(4, 5),)
    elif name == "vae":
        x = torch.rand(3, 6, **F64)
        fn = lambda xr, mu, lv: misc.vae_loss(xr, x, mu, lv)  # noqa: E731
        args = (_req(3, 6, lo=True), _req(3, 4), _req(3, 4))
    elif name == "mse":
        x = torch.randn(3, 6, **F64)
        fn, args = (lambda a: misc.mse_loss(a, x)), (_req(3, 6),)
    elif name == "luong":
        fn, args = (lambda s, h: misc.luong_attention(s, h)[0]), (_req(2, 4), _req(2, 5, 4))
    elif name == "lrn":
        fn, args = misc.local_response_norm, (_req(1, 6, 4, 4),)
    elif name == "maxpool":
        fn, args = misc.max_pool2d, (_req(1, 2, 7, 7),)
    elif name == "conv2d":
        fn = lambda a, w, b: misc.conv2d(a, w, b, stride=2, padding=1)  # noqa: E731
        args = (_req(1, 3, 6, 6), _req(4, 3, 3, 3), _req(4))
    else:
        fn = lambda a, w, b: misc.patch_embed(a, w, b, 4)  # noqa: E731
        args = (_req(2, 3, 8, 8), _req(5, 3, 4, 4), _req(5))
    assert gradcheck(fn, args, eps=1e-6, atol=1e-5)


def test_chunked_linear_cross_entropy_matches_torch():
    """ops/xent.py vocab-chunked fused head: loss and dh / dW / db equal
    F.cross_entropy on materialised logits, across chunk sizes (one chunk, ragged last
    chunk), label smoothing and ignored rows."""
    import torch.nn.functional as F
    from solvingpapers_amd.ops.xent import chunked_linear_cross_entropy
    g = torch.Generator().manual_seed(0)
    N, D, V = 24, 16, 1000
    h0 = torch.randn(N, D, generator=g, dtype=torch.float64)
    w0 = torch.randn(V, D, generator=g, dtype=torch.float64) * 0.3
    b0 = torch.randn(V, generator=g, dtype=torch.float64) * 0.1
    t = torch.randint(0, V, (N,), generator=g)
    t[3] = -100
    for chunk, sm in ((256, 0.0), (384, 0.1), (1000, 0.0)):
        ref_args = [x.clone().requires_grad_() for x in (h0, w0, b0)]
        ref = F.cross_entropy(F.linear(*ref_args), t, ignore_index=-100, label_smoothing=sm)
        ref.backward()
        args = [x.clone().requires_grad_() for x in (h0, w0, b0)]
        loss = chunked_linear_cross_entropy(args[0], args[1], t, bias=args[2], label_smoothing=sm, chunk_cols=chunk)
        (loss * 2.0).backward()
        assert torch.allclose(loss, ref, atol=1e-10), (chunk, loss, ref)
        for a, r in zip(args, ref_args):
            assert torch.allclose(a.grad, 2.0 * r.grad, atol=1e-10), chunk


def test_attention_dropout_cpu_mask_is_seeded_and_calibrated():
    """CPU path of attention_dropout: the same counter-hash mask the HIP kernels apply
    (ops/attention.py dropout_keep_mask) -- deterministic per seed, keep rate 1 - p."""
    from solvingpapers_amd.ops.attention import _materialised, dropout_keep_mask
    m1 = dropout_keep_mask(42, 2, 3, 64, 64, 0.25)
    m2 = dropout_keep_mask(42, 2, 3, 64, 64, 0.25)
    m3 = dropout_keep_mask(43, 2, 3, 64, 64, 0.25)
    assert torch.equal(m1, m2) and not torch.equal(m1, m3)
    assert abs(m1.float().mean().item() - 0.75) < 0.02
    g = torch.Generator().manual_seed(0)
    q, k, v = (torch.randn(2, 64, 3, 16, generator=g) for _ in range(3))
    o = _materialised(q, k, v, True, 0.25, 0.25, 42)
    s = torch.einsum("bqhd,bkhd->bhqk", q, k) * 0.25
    s = s.masked_fill(torch.triu(torch.ones(64, 64, dtype=torch.bool), 1), float("-inf"))
    pr = torch.softmax(s, -1) * m1 / 0.75
    want = torch.einsum("bhqk,bkhd->bqhd", pr, v)
    assert torch.allclose(o, want, atol=1e-5)


@pytest.mark.parametrize("kind", ["silu", "gelu_tanh"])
def test_swiglu_mlp_cpu_is_the_composition(kind):
    """ops.linear.swiglu_mlp off the GPU (and for tensors its kernels do not take) is exactly
    linear(glu(linear(x, w13), kind), w2) -- the fp64 reference composition, gradients included."""
    from solvingpapers_amd.ops.linear import swiglu_mlp
    torch.manual_seed(0)
    x = torch.randn(6, 16, dtype=torch.float64, requires_grad=True)
    w13 = torch.randn(2 * 24, 16, dtype=torch.float64, requires_grad=True)
    w2 = torch.randn(16, 24, dtype=torch.float64, requires_grad=True)
    y = swiglu_mlp(x, w13, w2, kind)
    h = x @ w13.t()
    g, u = h[:, :24], h[:, 24:]
    act = F.silu(g) if kind == "silu" else F.gelu(g, approximate="tanh")
    ref = (act * u) @ w2.t()
    assert torch.allclose(y, ref, rtol=1e-12, atol=1e-12)
    gy = torch.randn_like(y)
    ga = torch.autograd.grad(y, (x, w13, w2), gy)
    gb = torch.autograd.grad(ref, (x, w13, w2), gy)
    for a, b in zip(ga, gb):
        assert torch.allclose(a, b, rtol=1e-10, atol=1e-10)
