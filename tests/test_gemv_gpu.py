"""Decode-path kernels: weight-streaming GEMV (csrc/kernels/gemv.hip) and the fused RoPE +
KV-cache write (csrc/kernels/rope.hip, rope_kv_write_) against plain PyTorch fp32 / the
unfused ops."""
import pytest
import torch

from solvingpapers_amd.ops import _ext

pytestmark = pytest.mark.gpu
DEV = "cuda"


def rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12)).item()


@pytest.mark.parametrize("M,N,K", [
    (1, 4096, 4096),      # LLaMA3-8B o-proj
    (1, 6144, 4096),      # qkv
    (2, 28672, 4096),     # gate|up (RW = 4 path)
    (4, 4096, 14336),     # down-proj, 4 rows
    (3, 130, 136),        # N tail (not a multiple of 2 / 4), K tail (not a multiple of 512)
    (1, 8197, 520),       # RW = 4 path with a ragged last wave
    (4, 1, 8),            # degenerate
])
def test_gemv_matches_fp32(M, N, K):
    torch.manual_seed(0)
    x = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
    w = torch.randn(N, K, device=DEV, dtype=torch.bfloat16)
    y = _ext.ops().gemv(x, w)
    ref = x.float() @ w.float().t()
    assert y.shape == (M, N) and y.dtype == torch.bfloat16
    assert rel(y, ref) < 1e-2, rel(y, ref)


def test_gemv_strided_rows():
    # x rows with a padded stride (e.g. the last token of a [B, T, D] buffer)
    torch.manual_seed(1)
    xb = torch.randn(3, 4096 + 64, device=DEV, dtype=torch.bfloat16)
    x = xb[:, :4096]
    w = torch.randn(1000, 4096, device=DEV, dtype=torch.bfloat16)
    assert rel(_ext.ops().gemv(x, w), x.float() @ w.float().t()) < 1e-2


def test_linear_routes_decode_rows_to_gemv():
    from solvingpapers_amd.ops.linear import _gemv_ok, linear
    torch.manual_seed(2)
    w = torch.randn(2048, 1024, device=DEV, dtype=torch.bfloat16)
    x = torch.randn(2, 1, 1024, device=DEV, dtype=torch.bfloat16)
    with torch.no_grad():
        assert _gemv_ok(x, w, None)
        y = linear(x, w)
    assert y.shape == (2, 1, 2048)
    assert rel(y, x.float() @ w.float().t()) < 1e-2
    # training (autograd) and prefill-sized inputs keep the GEMM path
    wg = w.clone().requires_grad_()
    assert not _gemv_ok(x, wg, None)
    assert not _gemv_ok(torch.randn(8, 1024, device=DEV, dtype=torch.bfloat16), w, None)


def test_rope_kv_write_matches_unfused():
    from solvingpapers_amd.ops.rope import RopeCache
    torch.manual_seed(3)
    B, T, H, KV, hd, Tmax = 2, 1, 8, 2, 128, 40
    x = torch.randn(B, T, H + 2 * KV, hd, device=DEV, dtype=torch.bfloat16)
    cos, sin = RopeCache.get(Tmax, hd, 500000.0, x.device)
    index = torch.tensor([17], device=DEV, dtype=torch.long)
    positions = torch.full((B, T), 17, device=DEV, dtype=torch.int32)
    kc = torch.randn(B, Tmax, KV, hd, device=DEV, dtype=torch.bfloat16)
    vc = torch.randn(B, Tmax, KV, hd, device=DEV, dtype=torch.bfloat16)
    # unfused reference: rope_ on q and k, then index_copy_ of k and v
    xr, kr, vr = x.clone(), kc.clone(), vc.clone()
    _ext.ops().rope_(xr, cos, sin, positions, H + KV, 0, 0, False)
    kr.index_copy_(1, index, xr[:, :, H:H + KV])
    vr.index_copy_(1, index, xr[:, :, H + KV:])
    _ext.ops().rope_kv_write_(x, cos, sin, positions, index, kc, vc, H, KV)
    assert torch.equal(x[:, :, :H], xr[:, :, :H])
    assert torch.equal(kc, kr) and torch.equal(vc, vr)
    # a row past the cache end is dropped, nothing else is touched
    k0, v0 = kc.clone(), vc.clone()
    _ext.ops().rope_kv_write_(x, cos, sin, positions, torch.tensor([Tmax], device=DEV), kc, vc, H, KV)
    assert torch.equal(kc, k0) and torch.equal(vc, v0)


def test_rope_kv_write_rotate_half_matches_unfused():
    from solvingpapers_amd.ops.rope import RopeCache
    torch.manual_seed(4)
    B, T, H, KV, hd, Tmax = 1, 1, 16, 1, 256, 24
    x = torch.randn(B, T, H + 2 * KV, hd, device=DEV, dtype=torch.bfloat16)
    cos, sin = RopeCache.get(Tmax, hd, 10000.0, x.device)
    index = torch.tensor([5], device=DEV, dtype=torch.long)
    positions = torch.full((B, T), 5, device=DEV, dtype=torch.int32)
    kc = torch.zeros(B, Tmax, KV, hd, device=DEV, dtype=torch.bfloat16)
    vc = torch.zeros(B, Tmax, KV, hd, device=DEV, dtype=torch.bfloat16)
    xr, kr, vr = x.clone(), kc.clone(), vc.clone()
    _ext.ops().rope_(xr, cos, sin, positions, H + KV, 0, 1, False)
    kr.index_copy_(1, index, xr[:, :, H:H + KV])
    vr.index_copy_(1, index, xr[:, :, H + KV:])
    _ext.ops().rope_kv_write_(x, cos, sin, positions, index, kc, vc, H, KV, 1)
    assert torch.equal(x[:, :, :H], xr[:, :, :H])
    assert torch.equal(kc, kr) and torch.equal(vc, vr)
