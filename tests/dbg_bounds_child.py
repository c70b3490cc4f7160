"""Cases run by tests/test_debug_bounds_gpu.py inside a child pytest that loads the debug-bounds build
(SPA_EXT_SO=ab/_C_dbg.so, SPA_DEBUG_SYNC=1; csrc/include/spa_debug.h). Not collected on its own (no
test_ prefix): in that child every op call synchronises and reads the device guard records, and
tests/conftest.py fails any test after which a guard fired.

Besides the existing ragged-shape GPU tests the parent selects, this file covers the cases the
debug build is for: ragged attention lengths at every head-dim family (forward + backward through
the shipped dispatch), empty / tiny / odd expert segments through the grouped GEMMs, and one
deliberate violation (an out-of-range token id) that must be REPORTED -- with file and line --
instead of faulting the GPU."""
import os

import pytest
import torch

from solvingpapers_amd.ops import _ext

pytestmark = pytest.mark.gpu


def test_debug_build_is_loaded():
    assert os.environ.get("SPA_DEBUG_SYNC") == "1"
    assert _ext.so_path().endswith("_C_dbg.so"), _ext.so_path()
    assert _ext.debug_bounds_enabled()
    assert _ext.debug_bounds_report() == ""


@pytest.mark.parametrize("T", [197, 200, 300, 520])
@pytest.mark.parametrize("H,Hkv,dqk,dv,causal", [(4, 4, 64, 64, False), (8, 2, 128, 128, True),
                                                  (4, 1, 256, 256, True), (4, 4, 192, 128, True)])
def test_ragged_attention_fwd_bwd_clean(T, H, Hkv, dqk, dv, causal):
    from solvingpapers_amd.ops.attention import flash_attention
    g = torch.Generator(device="cuda").manual_seed(T)
    q = torch.randn(2, T, H, dqk, device="cuda", generator=g).bfloat16().requires_grad_()
    k = torch.randn(2, T, Hkv, dqk, device="cuda", generator=g).bfloat16().requires_grad_()
    v = torch.randn(2, T, Hkv, dv, device="cuda", generator=g).bfloat16().requires_grad_()
    o = flash_attention(q, k, v, causal=causal)
    o.float().square().sum().backward()
    torch.cuda.synchronize()
    assert torch.isfinite(q.grad.float()).all() and torch.isfinite(v.grad.float()).all()
    assert _ext.debug_bounds_report() == ""


@pytest.mark.parametrize("counts", [[0, 0, 5, 0], [1, 255, 257, 0, 3], [0] * 7 + [513], [17]])
def test_grouped_gemm_ragged_segments_clean(counts):
    from solvingpapers_amd.ops.moe import grouped_gemm
    E, N, K = len(counts), 264, 136
    M = sum(counts)
    off = torch.tensor([0] + list(torch.tensor(counts).cumsum(0)), dtype=torch.int32, device="cuda")
    a = torch.randn(M, K, device="cuda").bfloat16()
    w = torch.randn(E, N, K, device="cuda").bfloat16()
    y = grouped_gemm(a, w, off, 0)
    dy = torch.randn(M, N, device="cuda").bfloat16()
    dx = grouped_gemm(dy, w, off, 1)
    dw = grouped_gemm(dy, a, off, 2)
    torch.cuda.synchronize()
    assert y.shape == (M, N) and dx.shape == (M, K) and dw.shape == (E, N, K)
    assert _ext.debug_bounds_report() == ""


def test_out_of_range_token_is_reported_not_faulted():
    """An id == V would read past the table in the release build; the debug build's guard skips the
    load, records embedding.hip:line, and the checked op wrapper raises BoundsViolation."""
    from solvingpapers_amd.ops.embedding import embedding
    V, D = 1000, 64
    W = torch.randn(V, D, device="cuda").bfloat16()
    ids = torch.tensor([[3, V, 7]], device="cuda")
    with pytest.raises(_ext.BoundsViolation) as ei:
        embedding(W, ids)
    msg = str(ei.value)
    assert "embedding.hip:" in msg and f"{V} outside [0, {V})" in msg, msg
    assert _ext.debug_bounds_report() == ""   # the wrapper consumed (reset) the record
