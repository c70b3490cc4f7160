"""gemm4a.hip (4 waves x 128x128 per 256x256 tile, accumulators pinned in AGPRs by inline-asm MFMAs)
against an fp32 torch oracle: every mode (fwd X W^T, dX = dY W, per-expert dW = dY^T X with and
without accumulate), every pipeline (two-buffer LDS-DMA "gemm4d", register staging "gemm4r", the
32-deep DMA ring), ragged / empty / single-row experts, and the dense split-K weight gradient
(wgrad8 -> gemm4r fp32 partials)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def rel(x, y):
    return ((x.float() - y.float()).norm() / y.float().norm().clamp_min(1e-12)).item()


def _offs(counts):
    c = torch.tensor(counts, dtype=torch.int32)
    return torch.cat([torch.zeros(1, dtype=torch.int32), c.cumsum(0).to(torch.int32)]).to(DEV), \
        [0] + c.cumsum(0).tolist()


CASES = [
    [0, 1, 255, 257, 0, 513, 3, 64],     # ragged, empty, single-row experts
    [768] * 16,                          # balanced
    [4096],                              # dense (E = 1)
]


@pytest.mark.parametrize("impl", [2, 1, 0])
@pytest.mark.parametrize("counts", CASES)
def test_gemm4a_modes_match_fp32(impl, counts):
    from solvingpapers_amd.ops._ext import ops
    torch.manual_seed(len(counts) * 7 + impl)
    E = len(counts)
    off, o = _offs(counts)
    Mtot = o[-1]
    N, K = 320, 512                                  # N not a multiple of 256: ragged column tiles
    x = torch.randn(Mtot, K, device=DEV, dtype=torch.bfloat16)
    w = torch.randn(E, N, K, device=DEV, dtype=torch.bfloat16) * 0.05
    y = ops().gemm4a(x, w, off, 0, None, False, impl)
    ref = torch.cat([x[o[e]:o[e + 1]].float() @ w[e].float().t() for e in range(E)])
    assert rel(y, ref) < 1e-2, ("fwd", rel(y, ref))
    dy = torch.randn(Mtot, N * 2, device=DEV, dtype=torch.bfloat16)
    wt = torch.randn(E, N * 2, K, device=DEV, dtype=torch.bfloat16) * 0.05   # dX = dy_e @ w_e: [M, K]
    dx = ops().gemm4a(dy, wt, off, 1, None, False, impl)
    ref = torch.cat([dy[o[e]:o[e + 1]].float() @ wt[e].float() for e in range(E)])
    assert rel(dx, ref) < 1e-2, ("dX", rel(dx, ref))
    dw = ops().gemm4a(dy, x, off, 2, None, False, impl)
    ref = torch.stack([dy[o[e]:o[e + 1]].float().t() @ x[o[e]:o[e + 1]].float() for e in range(E)])
    nz = [e for e in range(E) if counts[e] > 0]
    assert rel(dw[nz], ref[nz]) < 1e-2, ("dW", rel(dw[nz], ref[nz]))
    for e in range(E):                              # an expert without tokens gets an exact zero dW
        if counts[e] == 0:
            assert dw[e].abs().max().item() == 0
    acc0 = torch.randn_like(dw)
    dwa = ops().gemm4a(dy, x, off, 2, acc0.clone(), True, impl)
    assert rel(dwa, ref + acc0.float()) < 1e-2, ("dW accumulate", rel(dwa, ref + acc0.float()))


@pytest.mark.parametrize("T,N,K", [(8192, 768, 768), (50432, 3072, 768), (6000, 256, 1024)])
def test_wgrad8_on_gemm4r_partials_matches_fp32(T, N, K, monkeypatch):
    from solvingpapers_amd.ops._ext import ops
    torch.manual_seed(T + N)
    dy = torch.randn(T, N, device=DEV, dtype=torch.bfloat16)
    x = torch.randn(T, K, device=DEV, dtype=torch.bfloat16)
    ref = dy.float().t() @ x.float()
    got = ops().wgrad8(dy, x, None, False, 0)                  # default: gemm4r partials
    assert rel(got, ref) < 1e-2, rel(got, ref)
    out = torch.randn(N, K, device=DEV, dtype=torch.float32)
    exp = out + ref
    ops().wgrad8(dy, x, out, True, 0)
    assert rel(out, exp) < 1e-3, rel(out, exp)


def test_moe_grouped_dw_routes_to_gemm4r():
    from solvingpapers_amd.ops import moe as M
    assert M.GG_DW_G4
    torch.manual_seed(0)
    off, o = _offs([100, 0, 900, 37])
    dy = torch.randn(o[-1], 256, device=DEV, dtype=torch.bfloat16)
    x = torch.randn(o[-1], 512, device=DEV, dtype=torch.bfloat16)
    got = M.grouped_gemm(dy, x, off, 2)
    ref = torch.stack([dy[o[e]:o[e + 1]].float().t() @ x[o[e]:o[e + 1]].float() for e in range(4)])
    assert rel(got, ref) < 1e-2
