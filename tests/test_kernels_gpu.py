"""HIP kernel numerics vs plain-PyTorch fp32 oracles (SURVEY.md §4.2 tier T1).

Every test asserts the extension is loaded (no silent eager fallback) and runs
the torch.ops.spa kernel against the oracle in ops/reference.py on edge shapes
(T not a multiple of the tile, T=197 for ViT, hd 64/128/256, Hkv=1 MQA).
"""
import math

import pytest
import torch

from solvingpapers_amd.ops import _ext, reference as R

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(autouse=True, scope="module")
def _need_ext():
    assert _ext.load(), "HIP extension must load on the GPU box"
    torch.manual_seed(0)


def rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / b.norm().clamp_min(1e-12)).item()


@pytest.mark.parametrize("D", [64, 256, 768, 1000, 4096])
@pytest.mark.parametrize("ln", [False, True])
@pytest.mark.parametrize("res", [False, True])
def test_norm_fwd_bwd(D, ln, res):
    if D % 8:
        pytest.skip("D%8 required")
    from solvingpapers_amd.ops import layer_norm, rms_norm
    M = 300
    x = torch.randn(M, D, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    r = torch.randn(M, D, device=DEV, dtype=torch.bfloat16, requires_grad=True) if res else None
    w = (torch.rand(D, device=DEV) + 0.5).bfloat16().requires_grad_()
    b = torch.randn(D, device=DEV).bfloat16().requires_grad_() if ln else None
    dy = torch.randn(M, D, device=DEV, dtype=torch.bfloat16)
    dh = torch.randn(M, D, device=DEV, dtype=torch.bfloat16) if res else None
    out = layer_norm(x, w, b, 1e-5, residual=r) if ln else rms_norm(x, w, 1e-5, residual=r)
    y, h = (out if res else (out, None))
    loss = (y.float() * dy.float()).sum() + ((h.float() * dh.float()).sum() if res else 0)
    loss.backward()
    xs = [t.detach().float().requires_grad_() for t in (x, w)]
    rf = r.detach().float().requires_grad_() if res else None
    bf = b.detach().float().requires_grad_() if ln else None
    hf = xs[0] + rf if res else xs[0]
    if ln:
        yf = torch.nn.functional.layer_norm(hf, (D,), xs[1], bf, 1e-5)
    else:
        yf = hf * torch.rsqrt(hf.pow(2).mean(-1, keepdim=True) + 1e-5) * xs[1]
    lf = (yf * dy.float()).sum() + ((hf * dh.float()).sum() if res else 0)
    lf.backward()
    assert rel(y, yf) < 1e-2
    assert rel(x.grad, xs[0].grad) < 2e-2
    assert rel(w.grad, xs[1].grad) < 2e-2
    if ln:
        assert rel(b.grad, bf.grad) < 2e-2
    if res:
        assert rel(r.grad, rf.grad) < 2e-2


@pytest.mark.parametrize("kind", ["relu", "leaky_relu", "prelu", "elu", "gelu_tanh", "gelu", "silu", "sigmoid", "tanh"])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_activation(kind, dtype):
    from solvingpapers_amd.ops import act
    x = (torch.randn(1003, device=DEV) * 3).to(dtype).requires_grad_()
    alpha = {"prelu": 0.3, "elu": 0.4, "leaky_relu": 0.01}.get(kind)
    y = act(x, kind, alpha)
    g = torch.randn_like(y)
    (y.float() * g.float()).sum().backward()
    xf = x.detach().float().requires_grad_()
    yf = R.act(xf, kind, alpha or 0.0)
    (yf * g.float()).sum().backward()
    tol = 1e-5 if dtype == torch.float32 else 1e-2
    assert rel(y, yf) < tol
    assert rel(x.grad, xf.grad) < (1e-4 if dtype == torch.float32 else 2e-2)


@pytest.mark.parametrize("kind,R", [("gelu", 1000), ("gelu", 50432 // 8), ("relu", 77)])
def test_linear_act_fused_bias_grad(kind, R):
    """fc1 + activation with the fused activation-backward + bias-gradient pass vs fp32 torch."""
    from solvingpapers_amd.ops.linear import linear_act
    K, N = 256, 768
    x = (torch.randn(R, K, device=DEV) * 0.5).bfloat16().requires_grad_()
    w = (torch.randn(N, K, device=DEV) * K ** -0.5).bfloat16().requires_grad_()
    b = (torch.randn(N, device=DEV) * 0.1).bfloat16().requires_grad_()
    y = linear_act(x, w, b, kind)
    g = torch.randn_like(y)
    (y.float() * g.float()).sum().backward()
    xf, wf, bf = (t.detach().float().requires_grad_() for t in (x, w, b))
    yf = R_act(xf @ wf.t() + bf, kind)
    (yf * g.float()).sum().backward()
    assert rel(y, yf) < 1e-2
    for got, ref in ((x.grad, xf.grad), (w.grad, wf.grad), (b.grad, bf.grad)):
        assert rel(got, ref) < 2e-2


@pytest.mark.parametrize("kind,R,D,F", [("gelu", 1000, 256, 1024), ("gelu", 6304, 768, 3072), ("relu", 300, 128, 192)])
def test_mlp_matches_fp32(kind, R, D, F):
    """ops.mlp: fc2(act(fc1 x)) with the fused activation backward + fc1 bias gradient vs fp32 torch."""
    import importlib
    L = importlib.import_module("solvingpapers_amd.ops.linear")   # (ops.linear is also a function)
    x = (torch.randn(R, D, device=DEV) * 0.5).bfloat16().requires_grad_()
    w1 = (torch.randn(F, D, device=DEV) * D ** -0.5).bfloat16().requires_grad_()
    b1 = (torch.randn(F, device=DEV) * 0.1).bfloat16().requires_grad_()
    w2 = (torch.randn(D, F, device=DEV) * F ** -0.5).bfloat16().requires_grad_()
    b2 = (torch.randn(D, device=DEV) * 0.1).bfloat16().requires_grad_()
    y = L.mlp(x, w1, b1, w2, b2, kind)
    g = torch.randn_like(y)
    (y.float() * g.float()).sum().backward()
    ps = (x, w1, b1, w2, b2)
    fs = [t.detach().float().requires_grad_() for t in ps]
    yf = R_act(fs[0] @ fs[1].t() + fs[2], kind) @ fs[3].t() + fs[4]
    (yf * g.float()).sum().backward()
    assert rel(y, yf) < 1e-2
    for p_, f_ in zip(ps, fs):
        assert rel(p_.grad, f_.grad) < 2e-2, p_.shape


@pytest.mark.parametrize("kind", [6, 4])   # silu (LLaMA SwiGLU), gelu_tanh (Gemma GeGLU)
@pytest.mark.parametrize("M,F", [(1000, 200), (4096, 1024), (8, 8)])
def test_glu_bwd_t_matches_glu_bwd(M, F, kind):
    """glu_bwd_t (the GLU backward that also writes dgu^T for the both-token-contiguous dW) == glu_bwd
    (bitwise for silu), and its second output is exactly the transpose; ragged token / feature tiles."""
    from solvingpapers_amd.ops import _ext
    torch.manual_seed(8)
    gu = torch.randn(M, 2 * F, device=DEV).bfloat16()
    dy = torch.randn(M, F, device=DEV).bfloat16()
    ref = _ext.ops().glu_bwd(dy, gu, kind)
    dgu, dgut = _ext.ops().glu_bwd_t(dy, gu, kind)
    torch.cuda.synchronize()
    # silu: bitwise; gelu_tanh: hipcc contracts tanh's polynomial differently per kernel (fp32 last bits)
    assert torch.equal(dgu, ref) if kind == 6 else rel(dgu, ref) < 1e-2
    assert dgut.shape == (2 * F, M) and torch.equal(dgut, dgu.t())


@pytest.mark.parametrize("acc", [False, True])
def test_linear_glu_matches_composition(acc, monkeypatch):
    """ops.linear.linear_glu (glu_bwd_t + the both-transposed dW form) == glu(linear(x, w13)) on every
    gradient (SPA_GLU_T=0 arm), into a flat bf16 main_grad with and without accumulation."""
    import importlib
    L = importlib.import_module("solvingpapers_amd.ops.linear")
    T, D, F = 2048, 256, 512
    torch.manual_seed(9)
    x0 = (torch.randn(T, D, device=DEV) * 0.5).bfloat16()
    w0 = (torch.randn(2 * F, D, device=DEV) * D ** -0.5).bfloat16()
    g = torch.randn(T, F, device=DEV).bfloat16()
    res = {}
    for mode in ("1", "0"):
        monkeypatch.setenv("SPA_GLU_T", mode)
        x = x0.clone().requires_grad_()
        w = w0.clone().requires_grad_()
        w.main_grad = torch.full_like(w0, 0.25) if acc else torch.zeros_like(w0)
        from solvingpapers_amd.utils.grad import _Gen
        w._spa_gen = _Gen.value if acc else -1
        y = L.linear_glu(x, w, "silu")
        y.backward(g)
        res[mode] = (y.detach(), x.grad, w.main_grad.clone())
    assert torch.equal(res["1"][0], res["0"][0])
    assert torch.equal(res["1"][1], res["0"][1])
    assert rel(res["1"][2], res["0"][2]) < 1e-2, rel(res["1"][2], res["0"][2])
    xf, wf = x0.float().requires_grad_(), w0.float().requires_grad_()
    gate, up = (xf @ wf.t()).chunk(2, -1)
    (torch.nn.functional.silu(gate) * up).backward(g.float())
    assert rel(res["1"][2] - (0.25 if acc else 0.0), wf.grad) < 2e-2


@pytest.mark.parametrize("kind", [6, 4])
@pytest.mark.parametrize("M,F", [(1000, 200), (4096, 1024), (8, 8)])
def test_glu_fwd_t_matches_glu_fwd(M, F, kind):
    """glu_fwd_t == glu_fwd (bitwise for silu), its second output exactly the transpose (ragged tiles)."""
    from solvingpapers_amd.ops import _ext
    torch.manual_seed(10)
    gu = torch.randn(M, 2 * F, device=DEV).bfloat16()
    ref = _ext.ops().glu_fwd(gu, kind)
    y, yt = _ext.ops().glu_fwd_t(gu, kind)
    torch.cuda.synchronize()
    assert torch.equal(y, ref) if kind == 6 else rel(y, ref) < 1e-2
    assert yt.shape == (F, M) and torch.equal(yt, y.t())


@pytest.mark.parametrize("kind", ["silu", "gelu_tanh"])
@pytest.mark.parametrize("acc", [False, True])
def test_swiglu_mlp_matches_composition(acc, kind, monkeypatch):
    """ops.linear.swiglu_mlp (y^T kept from the forward, dH^T from the backward: both weight gradients
    in the both-transposed form) == linear(glu(linear(x, w13)), w2) (SPA_GLU_T=0) on every output and
    gradient, into flat bf16 main_grads with and without accumulation."""
    import importlib
    from solvingpapers_amd.utils.grad import _Gen
    L = importlib.import_module("solvingpapers_amd.ops.linear")
    T, D, F = 2048, 256, 512
    torch.manual_seed(11)
    x0 = (torch.randn(T, D, device=DEV) * 0.5).bfloat16()
    w13_0 = (torch.randn(2 * F, D, device=DEV) * D ** -0.5).bfloat16()
    w2_0 = (torch.randn(D, F, device=DEV) * F ** -0.5).bfloat16()
    g = torch.randn(T, D, device=DEV).bfloat16()
    res = {}
    for mode in ("2", "0"):
        monkeypatch.setenv("SPA_GLU_T", mode)
        x = x0.clone().requires_grad_()
        w13, w2 = w13_0.clone().requires_grad_(), w2_0.clone().requires_grad_()
        for w in (w13, w2):
            w.main_grad = torch.full_like(w, 0.25) if acc else torch.zeros_like(w)
            w._spa_gen = _Gen.value if acc else -1
        y = L.swiglu_mlp(x, w13, w2, kind)
        y.backward(g)
        res[mode] = (y.detach(), x.grad, w13.main_grad.clone(), w2.main_grad.clone())
    assert torch.equal(res["2"][0], res["0"][0])
    assert rel(res["2"][1], res["0"][1]) < 1e-2
    for i in (2, 3):
        assert rel(res["2"][i], res["0"][i]) < 1e-2, (i, rel(res["2"][i], res["0"][i]))


def R_act(x, kind):
    return R.act(x, kind, 0.0)


@pytest.mark.parametrize("kind", ["silu", "gelu", "gelu_tanh"])
def test_glu(kind):
    from solvingpapers_amd.ops import glu
    gu = torch.randn(64, 2 * 1536, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    y = glu(gu, kind)
    g = torch.randn_like(y)
    (y.float() * g.float()).sum().backward()
    gf = gu.detach().float().requires_grad_()
    yf = R.glu(gf, kind)
    (yf * g.float()).sum().backward()
    assert rel(y, yf) < 1e-2 and rel(gu.grad, gf.grad) < 2e-2


@pytest.mark.parametrize("interleaved", [True, False])
def test_rope(interleaved):
    from solvingpapers_amd.ops.rope import RopeCache
    B, T, NH, hd, nrot = 2, 77, 6, 128, 4
    x = torch.randn(B, T, NH, hd, device=DEV, dtype=torch.bfloat16)
    cos, sin = RopeCache.get(T + 5, hd, 500000.0, x.device)
    y = x.clone()
    _ext.ops().rope_(y, cos, sin, None, nrot, 3, 0 if interleaved else 1, False)
    ref = R.rope(x[:, :, :nrot], cos, sin, 3, interleaved)
    assert rel(y[:, :, :nrot], ref) < 1e-2
    assert torch.equal(y[:, :, nrot:], x[:, :, nrot:])
    _ext.ops().rope_(y, cos, sin, None, nrot, 3, 0 if interleaved else 1, True)  # inverse
    assert rel(y, x) < 1e-2


@pytest.mark.parametrize("V", [65, 50257, 128256])
def test_xent(V):
    from solvingpapers_amd.ops import cross_entropy
    N = 37
    logits = (torch.randn(N, V, device=DEV) * 2).bfloat16()
    tgt = torch.randint(0, V, (N,), device=DEV)
    tgt[3] = -100
    lf = logits.float().requires_grad_()
    ref = torch.nn.functional.cross_entropy(lf, tgt, ignore_index=-100)
    ref.backward()
    lg = logits.clone().requires_grad_()
    work = lg * 1  # non-leaf so it may be overwritten in place
    loss = cross_entropy(work, tgt)
    loss.backward()
    assert abs(loss.item() - ref.item()) < 2e-2 * max(1.0, abs(ref.item()))
    assert rel(lg.grad, lf.grad) < 2e-2


def test_embedding():
    from solvingpapers_amd.ops import embedding
    V, D = 1000, 256
    W = torch.randn(V, D, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    idx = torch.randint(0, V, (4, 33), device=DEV)
    idx[0, :5] = 7  # repeated rows -> atomics on one row
    y = embedding(W, idx)
    assert torch.equal(y, W.detach()[idx])
    g = torch.randn_like(y)
    (y.float() * g.float()).sum().backward()
    ref = torch.zeros(V, D, device=DEV).index_add_(0, idx.reshape(-1), g.reshape(-1, D).float())
    assert rel(W.grad, ref) < 1e-2


def test_embedding_negative_ids_are_zero_rows():
    """A negative id (vocab-parallel: another rank's token) reads a zero row and sends no gradient,
    on the dense-gradient and the main_grad (emb_bwd_into) paths."""
    from solvingpapers_amd.ops import embedding
    ops = _ext.ops()
    V, D = 300, 256
    W = torch.randn(V, D, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    idx = torch.randint(0, V, (2, 65), device=DEV)
    idx[:, ::3] = -1
    y = embedding(W, idx, scale=2.0)
    keep = (idx >= 0)
    assert torch.equal(y[~keep], torch.zeros_like(y[~keep]))
    assert torch.equal(y[keep], (W.detach()[idx.clamp_min(0)] * 2.0)[keep])
    g = torch.randn_like(y)
    (y.float() * g.float()).sum().backward()
    ref = torch.zeros(V, D, device=DEV).index_add_(0, idx[keep], 2.0 * g[keep].float())
    assert rel(W.grad, ref) < 1e-2
    out = torch.full((V, D), float("nan"), device=DEV, dtype=torch.bfloat16)
    ops.emb_bwd_into(g, idx, 2.0, out, False)
    assert rel(out, ref) < 1e-2


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_embedding_grad_into_main_grad(dtype):
    """emb_bwd_into: sparse row flush into a main_grad view (overwrite, then accumulate), repeated
    tokens, and a scratch that is clean again for the next call (three calls, fresh ids each)."""
    ops = _ext.ops()
    V, D = 5000, 264
    out = torch.full((V, D), float("nan"), device=DEV, dtype=dtype)
    ref = torch.zeros(V, D, device=DEV)
    for call in range(3):
        idx = torch.randint(0, V, (3, 70), device=DEV)
        idx[0, :9] = 11 + call      # repeated rows: one flush per row
        g = torch.randn(3, 70, D, device=DEV, dtype=dtype)
        ops.emb_bwd_into(g, idx, 0.5, out, call > 0)
        if call == 0:
            ref.zero_()
        ref.index_add_(0, idx.reshape(-1), 0.5 * g.reshape(-1, D).float())
        assert torch.isfinite(out).all()
        assert rel(out, ref) < (1e-2 if dtype == torch.bfloat16 else 1e-5), call


def test_dgrad_transposed_weight_cache_tracks_updates():
    """dX through the cached W^T (ops/linear.py transposed_weight) equals dY W after every kind of
    weight update: none (cache hit), a torch in-place op (version counter), and a write the
    version counter cannot see, as a fused optimizer kernel makes, announced by the weight epoch."""
    from solvingpapers_amd.ops import linear
    from solvingpapers_amd.ops.linear import _WT_CACHE
    from solvingpapers_amd.ops.moe import bump_weight_epoch
    torch.manual_seed(0)
    w = (torch.randn(2048, 2048, device=DEV) * 0.02).bfloat16().requires_grad_()
    x = torch.randn(64, 2048, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    dy = torch.randn(64, 2048, device=DEV, dtype=torch.bfloat16)

    def dx():
        x.grad = None
        linear(x, w).backward(dy)
        return x.grad

    assert rel(dx(), dy.float() @ w.detach().float()) < 1e-2
    assert id(w) in _WT_CACHE
    assert rel(dx(), dy.float() @ w.detach().float()) < 1e-2          # hit
    with torch.no_grad():
        w.mul_(-0.5)                                                 # version bump
    assert rel(dx(), dy.float() @ w.detach().float()) < 1e-2
    w.data.mul_(3.0)                                                 # invisible to the version counter
    bump_weight_epoch()
    assert rel(dx(), dy.float() @ w.detach().float()) < 1e-2


def test_dgrad_weight_cache_flat_writes_and_capture(tmp_path):
    """Writes through the FlatParams buffer (checkpoint.load's flat.param.copy_) invalidate the
    cached W^T; a HIP-graph capture never reads the eager cache (replays see weight updates)."""
    from solvingpapers_amd.ops import linear
    from solvingpapers_amd.train import checkpoint as ckpt
    from solvingpapers_amd.utils.flat import FlatParams
    torch.manual_seed(1)

    class M(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.w = torch.nn.Parameter((torch.randn(1024, 512, device=DEV) * 0.02).bfloat16())

    m = M()
    flat = FlatParams(m)
    x = torch.randn(64, 512, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    dy = torch.randn(64, 1024, device=DEV, dtype=torch.bfloat16)

    def dx():
        x.grad = None
        linear(x, m.w).backward(dy)
        return x.grad

    ckpt.save(str(tmp_path), 0, flat, None, {})
    saved = m.w.detach().clone()
    assert rel(dx(), dy.float() @ m.w.detach().float()) < 1e-2            # fills the cache
    with torch.no_grad():
        flat.param.mul_(-2.0)                                               # change the weights ...
    ckpt.load(str(tmp_path), flat, None, {}, restore_rng=False)            # ... and restore them
    assert torch.equal(m.w.detach(), saved)
    with torch.no_grad():
        flat.param.mul_(3.0)
    ckpt.load(str(tmp_path), flat, None, {}, restore_rng=False)
    assert rel(dx(), dy.float() @ saved.float()) < 1e-2

    # capture fwd + bwd with the cache warm, then change W eagerly (epoch bump) and replay
    static_x = x.detach().clone().requires_grad_()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            static_x.grad = None
            linear(static_x, m.w).backward(dy)
    torch.cuda.current_stream().wait_stream(s)
    static_x.grad = None
    with torch.cuda.graph(g):
        linear(static_x, m.w).backward(dy)
    with torch.no_grad():
        flat.param.mul_(-0.25)
    from solvingpapers_amd.ops.linear import invalidate_weight_caches
    invalidate_weight_caches()
    g.replay()
    torch.cuda.synchronize()
    assert rel(static_x.grad, dy.float() @ m.w.detach().float()) < 1e-2


def test_adamw_matches_torch():
    from solvingpapers_amd.ops import optim_kernels as K
    n = 10007
    p0 = torch.randn(n, device=DEV)
    grads = [torch.randn(n, device=DEV) for _ in range(3)]
    tp = p0.clone().requires_grad_()
    topt = torch.optim.AdamW([tp], lr=1e-2, betas=(0.9, 0.95), eps=1e-8, weight_decay=0.1)
    p = p0.clone()
    m = torch.zeros(n, device=DEV)
    v = torch.zeros(n, device=DEV)
    for s, g in enumerate(grads, 1):
        tp.grad = g.clone()
        topt.step()
        K.adamw_(p, None, g, m, v, 1e-2, 0.9, 0.95, 1e-8, 0.1, s)
    assert rel(p, tp.detach()) < 1e-6
    # bf16 params + fp32 master
    pb = p0.bfloat16()
    master = p0.clone()
    m.zero_(); v.zero_()
    for s, g in enumerate(grads, 1):
        K.adamw_(pb, master, g.bfloat16(), m, v, 1e-2, 0.9, 0.95, 1e-8, 0.1, s)
    assert rel(master, tp.detach()) < 1e-2
    assert abs(K.sqsum(grads[0]).item() - grads[0].pow(2).sum().item()) < 1e-2 * grads[0].pow(2).sum().item()


def test_adamw_large_flat_buffer_matches_torch():
    """> 2 x 4096 x 256 x 8 elements: several sweeps of the capped grid-stride loop, then a
    partial last chunk (odd n), as in the 8B-parameter buckets."""
    from solvingpapers_amd.ops import optim_kernels as K
    n = 20_000_003
    torch.manual_seed(0)
    p0 = torch.randn(n, device=DEV)
    grads = [torch.randn(n, device=DEV) for _ in range(2)]
    tp = p0.clone().requires_grad_()
    topt = torch.optim.AdamW([tp], lr=1e-2, betas=(0.9, 0.95), eps=1e-8, weight_decay=0.1)
    p, m, v = p0.clone(), torch.zeros(n, device=DEV), torch.zeros(n, device=DEV)
    pb, master = p0.bfloat16(), p0.clone()
    mb, vb = torch.zeros(n, device=DEV), torch.zeros(n, device=DEV)
    for s, g in enumerate(grads, 1):
        tp.grad = g.clone()
        topt.step()
        K.adamw_(p, None, g, m, v, 1e-2, 0.9, 0.95, 1e-8, 0.1, s)
        K.adamw_(pb, master, g.bfloat16(), mb, vb, 1e-2, 0.9, 0.95, 1e-8, 0.1, s)
    ref = tp.detach()
    assert (p - ref).abs().max().item() < 1e-5
    assert rel(master, ref) < 1e-2
    assert (pb.float() - master).abs().max().item() <= 1e-2 * master.abs().max().item()


def test_adamw_bf16_moments_match_cpu_oracle():
    """bf16 moments (DeepSeek-V3 recipe) with an fp32 master: the HIP kernel against the CPU
    oracle doing the same rounding, and close to the fp32-moment trajectory."""
    from solvingpapers_amd.ops import optim_kernels as K
    n = 10007
    torch.manual_seed(0)
    p0 = torch.randn(n)
    grads = [torch.randn(n) for _ in range(4)]
    res = {}
    for dev in ("cpu", DEV):
        pb, master = p0.bfloat16().to(dev), p0.clone().to(dev)
        m = torch.zeros(n, dtype=torch.bfloat16, device=dev)
        v = torch.zeros(n, dtype=torch.bfloat16, device=dev)
        for s, g in enumerate(grads, 1):
            K.adamw_(pb, master, g.bfloat16().to(dev), m, v, 1e-2, 0.9, 0.95, 1e-8, 0.1, s)
        res[dev] = (master.cpu(), m.float().cpu(), v.float().cpu())
    for a, b in zip(res["cpu"], res[DEV]):
        assert rel(b, a) < 2e-3        # fp32 math in a different order, then one bf16 rounding
    pf, mf32, vf32 = p0.clone(), torch.zeros(n), torch.zeros(n)
    for s, g in enumerate(grads, 1):
        K.adamw_(pf, None, g.bfloat16().float(), mf32, vf32, 1e-2, 0.9, 0.95, 1e-8, 0.1, s)
    assert rel(res[DEV][0], pf) < 1e-3


ATTN_CASES = [
    # B, Tq, Tk, H, Hkv, hd, causal
    (2, 128, 128, 4, 4, 64, True),
    (1, 200, 200, 8, 2, 128, True),    # GQA, ragged tail
    (2, 197, 197, 3, 3, 64, False),    # ViT-B/16 length
    (1, 256, 256, 4, 1, 256, True),    # MQA, Gemma head dim
    (1, 64, 320, 4, 2, 128, True),     # Tq < Tk (chunked prefill / decode alignment)
    (1, 1, 77, 4, 2, 128, True),       # single-token decode
    (1, 1024, 1024, 8, 8, 128, True),
]


@pytest.mark.parametrize("B,Tq,Tk,H,Hkv,hd,causal", ATTN_CASES)
def test_flash_attention(B, Tq, Tk, H, Hkv, hd, causal):
    from solvingpapers_amd.ops import flash_attention
    torch.manual_seed(1)
    q = torch.randn(B, Tq, H, hd, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    k = torch.randn(B, Tk, Hkv, hd, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    v = torch.randn(B, Tk, Hkv, hd, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    o = flash_attention(q, k, v, causal=causal)
    do = torch.randn_like(o)
    o.backward(do)
    qf, kf, vf = (t.detach().float().requires_grad_() for t in (q, k, v))
    of, _ = R.attention(qf, kf, vf, causal)
    of.backward(do.float())
    assert rel(o, of) < 2e-2, rel(o, of)
    assert rel(q.grad, qf.grad) < 3e-2, rel(q.grad, qf.grad)
    assert rel(k.grad, kf.grad) < 3e-2, rel(k.grad, kf.grad)
    assert rel(v.grad, vf.grad) < 3e-2, rel(v.grad, vf.grad)


@pytest.mark.parametrize("B,T,H,Hkv,causal,hd", [
    (1, 1024, 8, 8, True, 128),     # MHA: 4 q-blocks per dq_ds block
    (2, 200, 8, 2, True, 128),      # GQA 4, ragged tail (not a multiple of 32 / 64)
    (1, 300, 4, 4, False, 128),     # non-causal, ragged
    (1, 512, 16, 2, True, 128),     # GQA 8: two blocks per 64-query block
    (1, 96, 6, 3, True, 128),       # GQA 2
    (1, 2048, 32, 8, True, 128),    # LLaMA3-8B head layout
    (1, 4160, 8, 2, True, 128),     # long causal, T % 128 == 64 (a half key block; pipelined intervals)
    (1, 1024, 16, 1, True, 256),    # Gemma-7B MQA (q-head split dK/dV + dS stores)
    (1, 1024, 2, 1, True, 256),     # its TP=8 rank (dK/dV iteration split)
    (2, 200, 4, 2, True, 256),      # ragged tail
    (1, 300, 3, 1, False, 256),     # non-causal, G = 3 (units span two query tiles per block)
    (4, 2048, 8, 8, True, 256),     # hd 256 with >= 512 key blocks: no q-head split (bf16 dK / dV stores)
    (1, 1024, 8, 8, True, (192, 128)),   # MLA (q/k 128 nope + 64 rope, v 128)
    (2, 200, 4, 4, True, (192, 128)),    # MLA, ragged tail
    (1, 300, 2, 2, False, (192, 128)),   # MLA, non-causal
    (1, 1024, 64, 64, True, (192, 128)),  # MLA with >= 512 key blocks: the paired dK/dV kernel
    (1, 520, 128, 128, False, (192, 128)),  # paired, non-causal, ragged
])
def test_attn_bwd_ds_path(B, T, H, Hkv, causal, hd, monkeypatch):
    """Backward through the materialised dS (the dK/dV kernel stores dS, dQ = dS K in a separate
    streaming pass; the default at head dims 128, 256 and MLA's (192, 128)) == the dq kernel that
    recomputes S and dP (SPA_ATTN_DQ_DS=0), and both track the fp32 reference."""
    from solvingpapers_amd.ops import _ext
    torch.manual_seed(3)
    hd, hdv = hd if isinstance(hd, tuple) else (hd, hd)
    q = torch.randn(B, T, H, hd, device=DEV, dtype=torch.bfloat16)
    k = torch.randn(B, T, Hkv, hd, device=DEV, dtype=torch.bfloat16)
    v = torch.randn(B, T, Hkv, hdv, device=DEV, dtype=torch.bfloat16)
    sc = 1 / math.sqrt(hd)
    out, lse = _ext.ops().attn_fwd(q, k, v, sc, causal)
    do = torch.randn_like(out)
    grads = {}
    extra = ("mla1",) if hdv != hd else ("v3",) if hd == 128 else ("s1",)
    for mode in ("2", "0") + extra:   # 2: the dS path whatever the grid size
        if mode == "mla1":     # MLA dS path with the single-wave dK/dV kernel instead of the paired one
            monkeypatch.setenv("SPA_ATTN_DKDV_MLA", "1")
        if mode == "v3":       # hd 128: dkdv3 (register-staged) instead of the default dkdv5 (LDS-DMA staged)
            monkeypatch.setenv("SPA_ATTN_DKDV5", "0")
        if mode == "s1":       # hd 256: the single-wave dK/dV kernel instead of the paired dV-split one + dK pass
            monkeypatch.setenv("SPA_ATTN_DKDV256", "0")
        monkeypatch.setenv("SPA_ATTN_DQ_DS", "2" if mode in ("mla1", "v3", "s1") else mode)
        dq, dk, dv = torch.full_like(q, float("nan")), torch.empty_like(k), torch.empty_like(v)
        _ext.ops().attn_bwd(do, q, k, v, out, lse, dq, dk, dv, sc, causal)
        torch.cuda.synchronize()
        grads[mode] = (dq, dk, dv)
    for other in [m for m in grads if m != "2"]:
        for a, b in zip(grads["2"], grads[other]):
            assert torch.isfinite(a).all() and torch.isfinite(b).all()
            # v3: the same products in the same order as dkdv5 (bitwise up to the dQ pass's sums);
            # the others: same bf16 dS and fp32 sums, different order
            assert rel(a, b) < (1e-5 if other == "v3" else 1e-2), (other, rel(a, b))
    qf, kf, vf = (t.float().requires_grad_() for t in (q, k, v))
    of, _ = R.attention(qf, kf, vf, causal)
    of.backward(do.float())
    for a, r in zip(grads["2"], (qf.grad, kf.grad, vf.grad)):
        assert rel(a, r) < 3e-2, rel(a, r)


@pytest.mark.parametrize("Hkv,dqk,dv", [(4, 192, 128), (1, 96, 64), (2, 128, 64)])
def test_flash_attention_mixed_head_dims(Hkv, dqk, dv):
    """Mixed q/k vs v head dims: (192, 128) is the MLA shape (q/k 128 nope + 64 rope, v 128) and
    runs its own unpadded kernel pair; the other pairs have no instantiation and are zero-padded
    onto the smallest kernel pair (ops/attention.py flash_attention)."""
    from solvingpapers_amd.ops import flash_attention
    torch.manual_seed(3)
    B, T, H = 2, 300, 4
    q = torch.randn(B, T, H, dqk, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    k = torch.randn(B, T, Hkv, dqk, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    v = torch.randn(B, T, Hkv, dv, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    o = flash_attention(q, k, v, causal=True)
    assert o.shape == (B, T, H, dv)
    do = torch.randn_like(o)
    o.backward(do)
    qf, kf, vf = (t.detach().float().requires_grad_() for t in (q, k, v))
    of, _ = R.attention(qf, kf, vf, True)
    of.backward(do.float())
    assert rel(o, of) < 2e-2, rel(o, of)
    for a, b in ((q.grad, qf.grad), (k.grad, kf.grad), (v.grad, vf.grad)):
        assert a.shape == b.shape and rel(a, b) < 3e-2, rel(a, b)


@pytest.mark.parametrize("pos_off", [0, 5])
@pytest.mark.parametrize("dn", [128, 64])
def test_mla_attention_fused_matches_composition(pos_off, dn):
    """ops.mla_attention (rope + head assembly fused around the (192, 128) flash kernels -- or the
    hd-128 ones at dsv3_style's 64 nope + 64 rope --, dV written into the dkv buffer, rope key grad
    summed over heads) vs the op-by-op fp32 CPU path."""
    from solvingpapers_amd.ops.attention import mla_attention
    torch.manual_seed(7)
    B, T, H, dr, dv = 2, 300, 4, 64, 128
    q = torch.randn(B, T, H, dn + dr, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    kv = torch.randn(B, T, H, dn + dv, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    kr = torch.randn(B, T, 1, dr, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    o = mla_attention(q, kv, kr, dn, 0.07, 10000.0, pos_off)
    do = torch.randn_like(o)
    o.backward(do)
    qc, kvc, krc = (t.detach().float().cpu().requires_grad_() for t in (q, kv, kr))
    oc = mla_attention(qc, kvc, krc, dn, 0.07, 10000.0, pos_off)
    oc.backward(do.float().cpu())
    assert rel(o.cpu(), oc) < 2e-2, rel(o.cpu(), oc)
    for a, b in ((q.grad, qc.grad), (kv.grad, kvc.grad), (kr.grad, krc.grad)):
        assert rel(a.cpu(), b) < 3e-2, rel(a.cpu(), b)


@pytest.mark.parametrize("causal,Hkv,Tq,Tk", [(True, 1, 333, 333), (False, 2, 333, 333), (True, 1, 200, 333),
                                              (True, 1, 1024, 1024)])
def test_attn_fwd_hd256_variants_match(causal, Hkv, Tq, Tk, monkeypatch):
    """Head dim 256 forward: the S-sharing wave-pair kernel (default) == the two (256, 128) half-V
    column slices (SPA_ATTN_FWD256=0) == the single 4-wave kernel (and SPA_ATTN_SPLITV=0), output
    and lse, with and without a key split; and the fp32 oracle."""
    ops = _ext.ops()
    torch.manual_seed(4)
    q = torch.randn(2, Tq, 4, 256, device=DEV, dtype=torch.bfloat16)
    k = torch.randn(2, Tk, Hkv, 256, device=DEV, dtype=torch.bfloat16)
    v = torch.randn(2, Tk, Hkv, 256, device=DEV, dtype=torch.bfloat16)
    res = {}
    for name, env in (("single", {"SPA_ATTN_FWD256": "0", "SPA_ATTN_SPLITV": "0"}),
                      ("splitv", {"SPA_ATTN_FWD256": "0", "SPA_ATTN_SPLITV": "1"}),
                      ("pshare", {"SPA_ATTN_FWD256": "1", "SPA_ATTN_KSPLIT": "1"}),
                      ("pshare_ks3", {"SPA_ATTN_FWD256": "1", "SPA_ATTN_KSPLIT": "3"})):
        for kk in ("SPA_ATTN_FWD256", "SPA_ATTN_SPLITV", "SPA_ATTN_KSPLIT"):
            monkeypatch.delenv(kk, raising=False)
        for kk, vv in env.items():
            monkeypatch.setenv(kk, vv)
        res[name] = ops.attn_fwd(q, k, v, 0.0625, causal)
    o0, l0 = res["single"]
    for name in ("splitv", "pshare", "pshare_ks3"):
        o1, l1 = res[name]
        assert torch.isfinite(o1).all(), name
        assert rel(o1, o0) < 5e-3 and (l1 - l0).abs().max().item() < 1e-3, (name, rel(o1, o0))
    of, lf = R.attention(q.float(), k.float(), v.float(), causal, scale=0.0625)
    assert rel(res["pshare"][0], of) < 2e-2
    assert (res["pshare"][1] - lf).abs().max().item() < 1e-2


@pytest.mark.parametrize("B,Tq,Tk,H,Hkv,hd,causal", [
    (1, 1024, 1024, 2, 1, 256, True),     # TP=8 Gemma-7B rank: 2 q-heads, MQA, head dim 256
    (1, 700, 700, 2, 1, 256, False),      # ragged, non-causal
    (1, 256, 900, 4, 2, 128, True),       # Tq < Tk, GQA
])
def test_attn_key_split_matches(B, Tq, Tk, H, Hkv, hd, causal, monkeypatch):
    """Key-split query-parallel kernels (fp32 partials + merge; few (b, head) pairs) and the
    iteration-split dK/dV kernel == the unsplit kernels (SPA_ATTN_KSPLIT=1): forward output, lse
    and all three gradients, for the automatic split and a forced odd one; and the fp32 oracle."""
    ops = _ext.ops()
    torch.manual_seed(5)
    q = torch.randn(B, Tq, H, hd, device=DEV, dtype=torch.bfloat16)
    k = torch.randn(B, Tk, Hkv, hd, device=DEV, dtype=torch.bfloat16)
    v = torch.randn(B, Tk, Hkv, hd, device=DEV, dtype=torch.bfloat16)
    do = torch.randn(B, Tq, H, hd, device=DEV, dtype=torch.bfloat16)
    sc = 1 / math.sqrt(hd)
    res = {}
    for ks in ("1", None, "3"):
        if ks is None:
            monkeypatch.delenv("SPA_ATTN_KSPLIT", raising=False)
        else:
            monkeypatch.setenv("SPA_ATTN_KSPLIT", ks)
        out, lse = ops.attn_fwd(q, k, v, sc, causal)
        dq, dk, dv = torch.full_like(q, float("nan")), torch.empty_like(k), torch.empty_like(v)
        ops.attn_bwd(do, q, k, v, out, lse, dq, dk, dv, sc, causal)
        torch.cuda.synchronize()
        res[ks] = (out, lse, dq, dk, dv)
    for ks in (None, "3"):
        for i, (a, b) in enumerate(zip(res[ks], res["1"])):
            assert torch.isfinite(a).all(), (ks, i)
            if i == 1:
                assert (a - b).abs().max().item() < 1e-3, (ks, "lse")
            else:
                assert rel(a, b) < 1e-2, (ks, i, rel(a, b))
    qf, kf, vf = (t.float().requires_grad_() for t in (q, k, v))
    of, _ = R.attention(qf, kf, vf, causal)
    of.backward(do.float())
    assert rel(res[None][0], of) < 2e-2
    for a, r in zip(res[None][2:], (qf.grad, kf.grad, vf.grad)):
        assert rel(a, r) < 3e-2, rel(a, r)


@pytest.mark.parametrize("H,Hkv,hd,Ta,Tb", [(2, 1, 256, 512, 512), (4, 2, 128, 300, 200)])
def test_attention_packed_prefix_matches_whole_sequence(H, Hkv, hd, Ta, Tb):
    """ops.attention_packed_prefix (chunk B of a sequence split over chunk A's keys + its own, packed
    buffers) == causal attention of the whole sequence restricted to chunk B's rows, and its
    gradients into both packed buffers == the whole-sequence gradients."""
    from solvingpapers_amd.ops import attention_packed
    from solvingpapers_amd.ops.attention import attention_packed_prefix
    torch.manual_seed(6)
    W = (H + 2 * Hkv) * hd
    full = torch.randn(1, Ta + Tb, W, device=DEV, dtype=torch.bfloat16)
    a = full[:, :Ta].clone().requires_grad_()
    b = full[:, Ta:].clone().requires_grad_()
    o = attention_packed_prefix(b, a, H, Hkv, hd)
    do = torch.randn_like(o)
    o.backward(do)
    f = full.clone().requires_grad_()
    of = attention_packed(f, H, Hkv, causal=True, head_dim=hd)
    of[:, Ta:].backward(do)
    assert rel(o, of[:, Ta:]) < 1e-2
    assert rel(b.grad, f.grad[:, Ta:]) < 2e-2 and rel(a.grad, f.grad[:, :Ta]) < 2e-2


@pytest.mark.parametrize("ksplit", [None, "3"])
def test_flash_lse_and_spike(ksplit, monkeypatch):
    """Force the online-softmax rescale: one key spiked against one query (rule 26); with a forced
    key split the spike sits in one share and the merge rescales the others."""
    if ksplit:
        monkeypatch.setenv("SPA_ATTN_KSPLIT", ksplit)
    B, T, H, hd = 1, 300, 2, 128
    q = torch.randn(B, T, H, hd, device=DEV, dtype=torch.bfloat16) * 0.1
    k = torch.randn(B, T, H, hd, device=DEV, dtype=torch.bfloat16) * 0.1
    v = torch.randn(B, T, H, hd, device=DEV, dtype=torch.bfloat16)
    q[0, 250, 0] = 3.0
    k[0, 200, 0] = 3.0  # late tile with a huge score for query 250
    out, lse = _ext.ops().attn_fwd(q, k, v, 1 / math.sqrt(hd), True)
    of, lf = R.attention(q.float(), k.float(), v.float(), True)
    assert rel(out, of) < 2e-2
    assert (lse - lf).abs().max().item() < 5e-2


@pytest.mark.parametrize("step", [0.3, 0.735, 2.0])
def test_flash_deferred_rescale(step):
    """Scores that grow along the key axis so the running row max creeps up tile after
    tile by less than (0.3, 0.735: ~1 and ~3 log2 units per 32-key sub-tile) and more
    than (2.0) the 2^8 deferral threshold: exercises the deferred-rescale path, whose
    branch random data almost never takes (guide rule 26)."""
    from solvingpapers_amd.ops import flash_attention
    torch.manual_seed(3)
    B, T, H, hd = 1, 640, 2, 128
    q = (torch.randn(B, T, H, hd, device=DEV) * 0.2)
    k = (torch.randn(B, T, H, hd, device=DEV) * 0.2)
    q[..., 0] = 1.0
    k[..., 0] = step * torch.arange(T, device=DEV, dtype=torch.float32).view(1, T, 1) / 32
    q, k = q.bfloat16().requires_grad_(), k.bfloat16().requires_grad_()
    v = torch.randn(B, T, H, hd, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    o = flash_attention(q, k, v, causal=True)
    do = torch.randn_like(o)
    o.backward(do)
    qf, kf, vf = (t.detach().float().requires_grad_() for t in (q, k, v))
    of, _ = R.attention(qf, kf, vf, True)
    of.backward(do.float())
    assert rel(o, of) < 2e-2, rel(o, of)
    for a, b in ((q.grad, qf.grad), (k.grad, kf.grad), (v.grad, vf.grad)):
        assert rel(a, b) < 3e-2, rel(a, b)


def test_packed_attention_matches_split():
    from solvingpapers_amd.ops import attention_packed, flash_attention
    B, T, H, Hkv, hd = 2, 150, 8, 2, 128
    qkv = torch.randn(B, T, (H + 2 * Hkv) * hd, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    o = attention_packed(qkv, H, Hkv, head_dim=hd)
    g = torch.randn_like(o)
    o.backward(g)
    q2 = qkv.detach().clone().view(B, T, H + 2 * Hkv, hd).requires_grad_()
    o2 = flash_attention(q2[:, :, :H], q2[:, :, H:H + Hkv], q2[:, :, H + Hkv:]).reshape(B, T, H * hd)
    o2.backward(g)
    assert torch.equal(o, o2)
    assert rel(qkv.grad, q2.grad.reshape(B, T, -1)) < 1e-3


@pytest.mark.parametrize("B,Tq,Tk,H,causal", [(4, 197, 197, 12, False), (2, 256, 256, 4, True), (3, 33, 33, 2, True),
                                              (2, 100, 100, 3, False), (1, 64, 200, 2, True), (2, 256, 131, 2, False)])
def test_attention_short_bwd(B, Tq, Tk, H, causal, monkeypatch):
    """Fused short-sequence backward (T <= 256, hd 64: one block per (b, h), whole sequence in
    LDS) against the fp32 oracle and against the split dq + dK/dV kernels (SPA_ATTN_SHORT=0)."""
    ops = _ext.ops()
    torch.manual_seed(5)
    hd = 64
    q = torch.randn(B, Tq, H, hd, device=DEV, dtype=torch.bfloat16)
    k = torch.randn(B, Tk, H, hd, device=DEV, dtype=torch.bfloat16)
    v = torch.randn(B, Tk, H, hd, device=DEV, dtype=torch.bfloat16)
    sc = 1 / math.sqrt(hd)
    o, lse = ops.attn_fwd(q, k, v, sc, causal)
    do = torch.randn_like(o)
    grads = {}
    for mode in ("1", "0"):
        monkeypatch.setenv("SPA_ATTN_SHORT", mode)
        g = (torch.full_like(q, float("nan")), torch.full_like(k, float("nan")), torch.full_like(v, float("nan")))
        ops.attn_bwd(do, q, k, v, o, lse, *g, sc, causal)
        grads[mode] = g
    qf, kf, vf = (t.float().requires_grad_() for t in (q, k, v))
    of, _ = R.attention(qf, kf, vf, causal)
    of.backward(do.float())
    assert rel(o, of) < 2e-2, rel(o, of)
    for a, ref in zip(grads["1"], (qf.grad, kf.grad, vf.grad)):
        assert torch.isfinite(a).all()
        assert rel(a, ref) < 3e-2, rel(a, ref)
    for a, b in zip(grads["1"], grads["0"]):
        assert rel(a, b) < 1e-2, rel(a, b)


@pytest.mark.parametrize("env", [{"SPA_ATTN_BWD_FUSED": "1"}, {"SPA_ATTN_DKDV": "0"},
                                 {"SPA_ATTN_DKDV": "3"}])
def test_attention_bwd_variants_match_default(env):
    """The optional backward variants -- fused (dQ via fp32 atomics inside the dK/dV kernel)
    and the paired-wave dK/dV kernel -- against the default kernels, each run in a subprocess
    because the mode is read once per process. Shapes cover the q-head split (MQA / GQA
    grids too small for the chip) and the unsplit path."""
    import os, subprocess, sys, textwrap
    code = textwrap.dedent("""
        import math, torch, sys
        from solvingpapers_amd.ops import _ext
        ops = _ext.ops()
        torch.manual_seed(0)
        for (T, H, Hkv, hd, causal) in CASES:
            q = torch.randn(2, T, H, hd, device='cuda', dtype=torch.bfloat16)
            k = torch.randn(2, T, Hkv, hd, device='cuda', dtype=torch.bfloat16)
            v = torch.randn(2, T, Hkv, hd, device='cuda', dtype=torch.bfloat16)
            sc = 1 / math.sqrt(hd)
            o, lse = ops.attn_fwd(q, k, v, sc, causal)
            do = torch.randn_like(o)
            dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
            ops.attn_bwd(do, q, k, v, o, lse, dq, dk, dv, sc, causal)
            torch.save([dq.cpu(), dk.cpu(), dv.cpu()], sys.argv[1] + f'_{T}.pt')
    """)
    cases = [(300, 4, 2, 128, True), (256, 4, 4, 64, False), (129, 2, 1, 128, True), (1100, 8, 8, 128, True)]
    code = code.replace("CASES", repr(cases))
    outs = {}
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    # baseline: the single-wave dK/dV kernel (the default for hd 128 is the pipelined one)
    for name, extra in (("default", {"SPA_ATTN_DKDV": "1"}), ("variant", env)):
        e = dict(os.environ, PYTHONPATH=root, **extra)
        for key in ("SPA_ATTN_BWD_FUSED", "SPA_ATTN_DKDV"):
            if key not in extra:
                e.pop(key, None)
        pref = f"/tmp/spa_attn_bwd_{name}_{'_'.join(env)}"
        subprocess.run([sys.executable, "-c", code, pref], check=True, env=e, cwd=root, timeout=100)
        outs[name] = pref
    for T, *_ in cases:
        a = torch.load(outs["default"] + f"_{T}.pt", weights_only=True)
        b = torch.load(outs["variant"] + f"_{T}.pt", weights_only=True)
        for x, y in zip(a, b):
            assert (x.float() - y.float()).norm() / x.float().norm() < 2e-2


@pytest.mark.parametrize("R,C,dt", [(8192, 4096, torch.bfloat16), (200, 136, torch.bfloat16), (64, 4100, torch.float32),
                                    (50432, 768, torch.bfloat16), (8, 8, torch.bfloat16), (136, 200, torch.float32)])
def test_transpose2d(R, C, dt):
    from solvingpapers_amd.ops.layout import transpose2d
    x = torch.randn(R, C, device="cuda", dtype=dt)
    assert torch.equal(transpose2d(x), x.t().contiguous())
    xs = torch.randn(R, C + 16, device="cuda", dtype=dt)[:, 8:C + 8]
    assert torch.equal(transpose2d(xs), xs.t().contiguous())
    xb = torch.randn(3, R, C, device="cuda", dtype=dt) if R * C <= 1 << 22 else None
    if xb is not None:
        assert torch.equal(transpose2d(xb), xb.transpose(1, 2).contiguous())


@pytest.mark.parametrize("R,N", [(50432, 768), (100, 24), (7, 3072), (0, 16), (8192, 2304), (300, 264)])
def test_bias_grad_rowsum(R, N):
    from solvingpapers_amd.ops import _ext
    from solvingpapers_amd.ops.layout import bias_grad
    x = torch.randn(R, N + 8, device="cuda", dtype=torch.bfloat16)
    for t in (x[:, :N].contiguous(), x[:, 8:]):     # contiguous and a row-strided view
        ref = t.float().sum(0)
        out = _ext.ops().rowsum_bf16(t)
        assert out.dtype == torch.float32 and out.shape == (N,)
        assert torch.allclose(out, ref, rtol=1e-4, atol=1e-3)
        assert torch.equal(bias_grad(t), out)


@pytest.mark.parametrize("T,N,K", [(50432, 768, 3072), (50432, 2304, 768), (5000, 24, 40), (4096, 264, 520), (700, 64, 64)])
def test_wgrad8_dense_dw(T, N, K):
    """wgrad8 (split-K dense dW on the gemm8 kernel's token-major path, fp32 partials + reduce),
    contiguous and row-strided operands."""
    from solvingpapers_amd.ops import _ext
    ops = _ext.ops()
    dyb = torch.randn(T, N + 8, device="cuda", dtype=torch.bfloat16)
    xb = torch.randn(T, K + 16, device="cuda", dtype=torch.bfloat16)
    for dy, x in ((dyb[:, :N].contiguous(), xb[:, :K].contiguous()), (dyb[:, 8:], xb[:, 16:])):
        ref = dy.float().t() @ x.float()
        tol = 2e-3 * ref.norm()
        out = ops.wgrad8(dy, x, None, False, 0)
        assert out.dtype == torch.bfloat16 and out.shape == (N, K)
        assert (out.float() - ref).norm() < tol
        acc = out.clone()
        ops.wgrad8(dy, x, acc, True, 0)
        assert (acc.float() - 2 * ref).norm() < 2 * tol
        f32 = torch.full((N, K), 1.0, device="cuda")
        ops.wgrad8(dy, x, f32, True, 3)
        assert (f32 - 1.0 - ref).norm() < 1e-4 * ref.norm()
        ops.wgrad8(dy, x, f32, False, 1)
        assert (f32 - ref).norm() < 1e-4 * ref.norm()


def test_wgrad_nt_matches_tn():
    from solvingpapers_amd.ops.layout import wgrad
    dy = torch.randn(4096, 1024, device="cuda", dtype=torch.bfloat16)
    x = torch.randn(4096, 512, device="cuda", dtype=torch.bfloat16)
    ref = dy.float().t() @ x.float()
    out = wgrad(dy, x)
    assert ((out.float() - ref).norm() / ref.norm()) < 1e-2
    acc = out.clone()
    wgrad(dy, x, acc, True)
    assert ((acc.float() - 2 * ref).norm() / ref.norm()) < 1e-2


def test_wgrad_odd_token_count_falls_back():
    """dW = dY^T X for a token count that is not a multiple of 8 (MTP heads: T - k rows) takes
    the direct product instead of the transposed-operand path."""
    from solvingpapers_amd.ops.layout import wgrad, wgrad_nt_ok
    dy = torch.randn(4095, 256, device="cuda", dtype=torch.bfloat16)
    x = torch.randn(4095, 512, device="cuda", dtype=torch.bfloat16)
    assert not wgrad_nt_ok(dy, x)
    assert rel(wgrad(dy, x), dy.float().t() @ x.float()) < 1e-2
    dy8, x8 = dy[:4088], x[:4088]
    assert wgrad_nt_ok(dy8, x8)
    assert rel(wgrad(dy8, x8), dy8.float().t() @ x8.float()) < 1e-2


F32_ATTN_CASES = [
    # B, Tq, Tk, H, Hkv, hd, causal, dropout
    (2, 128, 128, 4, 2, 64, True, 0.0),      # LLaMA-ref parity shape (B1), GQA
    (2, 256, 256, 1, 1, 256, True, 0.0),     # GPT-ref parity shape (B5): one 256-wide head
    (2, 256, 256, 1, 1, 256, True, 0.2),     # ... with the reference's attention dropout
    (3, 50, 50, 4, 4, 16, False, 0.0),       # ViT-MNIST head dim 16, non-causal, ragged
    (1, 200, 333, 6, 2, 128, True, 0.1),     # Tq < Tk, ragged tails, GQA + dropout
    (1, 77, 77, 2, 1, 48, True, 0.0),        # head dim 48 zero-padded to 64
]


@pytest.mark.parametrize("B,Tq,Tk,H,Hkv,hd,causal,p", F32_ATTN_CASES)
def test_flash_attention_fp32(B, Tq, Tk, H, Hkv, hd, causal, p):
    """fp32 flash attention (csrc/kernels/attention_f32.hip, fp32 MFMA) == the fp64 GEMM + softmax
    oracle with the kernels' own dropout mask, forward and every gradient (fp32 rounding)."""
    from solvingpapers_amd.ops import flash_attention
    from solvingpapers_amd.ops.attention import _materialised
    torch.manual_seed(2)
    q = torch.randn(B, Tq, H, hd, device=DEV, requires_grad=True)
    k = torch.randn(B, Tk, Hkv, hd, device=DEV, requires_grad=True)
    v = torch.randn(B, Tk, Hkv, hd, device=DEV, requires_grad=True)
    seed = 1234567
    o = flash_attention(q, k, v, causal=causal, dropout_p=p, seed=seed)
    do = torch.randn_like(o)
    o.backward(do)
    qd, kd, vd = (t.detach().double().requires_grad_() for t in (q, k, v))
    od = _materialised(qd, kd, vd, causal, 1.0 / math.sqrt(hd), p, seed)
    od.backward(do.double())
    assert rel(o, od) < 2e-5, rel(o, od)
    assert rel(q.grad, qd.grad) < 5e-5, rel(q.grad, qd.grad)
    assert rel(k.grad, kd.grad) < 5e-5, rel(k.grad, kd.grad)
    assert rel(v.grad, vd.grad) < 5e-5, rel(v.grad, vd.grad)


def test_fp32_models_take_the_hip_attention(monkeypatch):
    """the fp32 parity models (GPT-ref, LLaMA-ref) attend on the fp32 HIP kernel, not the fallback"""
    from solvingpapers_amd.models import gpt, llama3
    from solvingpapers_amd.ops import attention as A
    calls = []
    real = A._FlashF32Fn.apply
    monkeypatch.setattr(A._FlashF32Fn, "apply", lambda *a: (calls.append(a[0].shape), real(*a))[1])
    monkeypatch.setattr(A, "_materialised", lambda *a, **k: (_ for _ in ()).throw(AssertionError("fallback")))
    for m in (gpt.GPT(gpt.config("gpt_ref"), device=DEV, dtype=torch.float32, seed=0),
              llama3.Llama3(llama3.config("llama3_ref"), device=DEV, dtype=torch.float32, seed=0)):
        m.train()
        ids = torch.randint(0, 60, (2, 65), device=DEV)
        m(ids[:, :-1], ids[:, 1:]).backward()
    assert len(calls) >= 2, calls
