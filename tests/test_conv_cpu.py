"""Implicit-GEMM conv address tables (ops/conv.py) on the CPU.

The HIP kernels (csrc/kernels/conv.hip) compute every address as row_base + ktab[group].offset
with bounds checks on (h0 + dh, w0 + dw) -- for the strided data grad, divisibility by the stride.
This test replays exactly that gather in torch for the fwd, data-grad and weight-grad GEMMs over
NHWC (padded channels), NCHW-direct (patchify) and strided / padded geometries, and checks the
GEMM results against torch's conv2d and its autograd.
"""
import pytest
import torch
import torch.nn.functional as F

from solvingpapers_amd.ops import conv as C


def _rows(geo, for_dgrad=False):
    nhwc, N, Cc, H, W, Cp, OC, KH, KW, sh, sw, ph, pw, OH, OW = geo
    if for_dgrad:
        n, i, j = torch.meshgrid(torch.arange(N), torch.arange(H), torch.arange(W), indexing="ij")
        return n.reshape(-1), (i + ph).reshape(-1), (j + pw).reshape(-1)
    n, i, j = torch.meshgrid(torch.arange(N), torch.arange(OH), torch.arange(OW), indexing="ij")
    return n.reshape(-1), (i * sh - ph).reshape(-1), (j * sw - pw).reshape(-1)


def _gather_fwd(xg, geo, ktab):
    """X~ [rows, K] exactly as conv_gemm_kernel<0> / <3> load it."""
    nhwc, N, Cc, H, W, Cp, OC, KH, KW, sh, sw, ph, pw, OH, OW = geo
    flat = xg.reshape(-1)
    gN = Cp * H * W
    sH, sW = (W * Cp, Cp) if nhwc else (W, 1)
    n, h0, w0 = _rows(geo)
    base = n * gN + h0 * sH + w0 * sW
    off, dh, dw = ktab[:, 0].long(), ktab[:, 1].long(), ktab[:, 2].long()
    h = h0[:, None] + dh[None]
    w = w0[:, None] + dw[None]
    ok = (h >= 0) & (h < H) & (w >= 0) & (w < W)
    idx = (base[:, None] + off[None])[..., None] + torch.arange(8)
    vals = flat[idx.clamp(0, flat.numel() - 1)] * ok[..., None]
    return vals.reshape(base.shape[0], -1)


def _gather_dgrad(dy, geo, ktab):
    nhwc, N, Cc, H, W, Cp, OC, KH, KW, sh, sw, ph, pw, OH, OW = geo
    flat = dy.reshape(-1)
    gN, sH, sW = OH * OW * OC, OW * OC, OC
    n, h0, w0 = _rows(geo, for_dgrad=True)
    off, dh, dw = ktab[:, 0].long(), ktab[:, 1].long(), ktab[:, 2].long()
    h = h0[:, None] + dh[None]
    w = w0[:, None] + dw[None]
    if sh == 1 and sw == 1:
        ok = (h >= 0) & (h < OH) & (w >= 0) & (w < OW)
        addr = (n * gN + h0 * sH + w0 * sW)[:, None] + off[None]
    else:
        ok = (h >= 0) & (w >= 0) & (h % sh == 0) & (w % sw == 0) & (h // sh < OH) & (w // sw < OW)
        addr = (n * gN)[:, None] + (h // sh) * sH + (w // sw) * sW + off[None]
    idx = addr[..., None] + torch.arange(8)
    vals = flat[idx.clamp(0, flat.numel() - 1)] * ok[..., None]
    return vals.reshape(n.shape[0], -1)


def _to_nhwc(x, Cp):
    y = torch.zeros(x.shape[0], x.shape[2], x.shape[3], Cp, dtype=x.dtype)
    y[..., :x.shape[1]] = x.permute(0, 2, 3, 1)
    return y


def _pack(w, Cp):
    OC, Cc, KH, KW = w.shape
    p = torch.zeros(OC, KH, KW, Cp, dtype=w.dtype)
    p[..., :Cc] = w.permute(0, 2, 3, 1)
    return p


CASES = [  # (N, C, H, W, OC, K, stride, pad)
    (2, 3, 23, 23, 16, 11, 4, 1),     # AlexNet conv1 shape class: C padded 3 -> 8, stride 4
    (2, 16, 9, 9, 24, 5, 1, 2),       # conv2 class
    (1, 8, 7, 6, 8, 3, 1, 1),
    (2, 8, 8, 9, 16, 3, 2, 1),        # strided data grad
    (2, 3, 32, 32, 16, 16, 16, 0),    # ViT patchify: NCHW direct
]


@pytest.mark.parametrize("case", CASES)
def test_conv_tables_reproduce_conv2d(case):
    N, Cc, H, W, OC, K, s, p = case
    g = torch.Generator().manual_seed(0)
    x = torch.randn(N, Cc, H, W, generator=g, dtype=torch.float64, requires_grad=True)
    w = torch.randn(OC, Cc, K, K, generator=g, dtype=torch.float64, requires_grad=True)
    y = F.conv2d(x, w, None, s, p)
    gy = torch.randn(y.shape, generator=g, dtype=torch.float64)
    y.backward(gy)
    nhwc = not C.nchw_direct_ok(Cc, H, W, K, K, s, s, p, p)
    assert nhwc == (case[6] != 16)
    geo = C.geometry(x.shape, w.shape, (s, s), (p, p), nhwc)
    Cp, OH, OW = geo[5], geo[13], geo[14]
    xd, wd = x.detach(), w.detach()
    xg = _to_nhwc(xd, Cp) if nhwc else xd
    wp = _pack(wd, Cp).reshape(OC, -1) if nhwc else wd.reshape(OC, -1)
    ktab = C.fwd_table(geo)
    A = _gather_fwd(xg, geo, ktab)                                    # [N*OH*OW, K]
    yg = (A @ wp.t()).view(N, OH, OW, OC).permute(0, 3, 1, 2)
    torch.testing.assert_close(yg, y.detach())
    # weight grad: dY^T X~, then the wgrad_reduce_kernel column map back to [OC, C, KH, KW]
    dy = gy.permute(0, 2, 3, 1).reshape(-1, OC)
    dwk = dy.t() @ A                                                  # [OC, K]
    if nhwc:
        dwk = dwk.view(OC, K, K, Cp)[..., :Cc].permute(0, 3, 1, 2)
    torch.testing.assert_close(dwk.reshape(w.shape), w.grad)
    # data grad (always NHWC-packed weights)
    gn = C.geometry(x.shape, w.shape, (s, s), (p, p), True)
    ktd, btab = C.dgrad_tables(gn)
    Ad = _gather_dgrad(gy.permute(0, 2, 3, 1).contiguous(), gn, ktd)  # [N*H*W, K*K*OC]
    wpn = _pack(wd, gn[5]).reshape(-1)
    B = wpn[btab.long()[:, None] + torch.arange(gn[5])]               # [K*K*OC, Cp]
    dx = (Ad @ B).view(N, H, W, gn[5])[..., :Cc].permute(0, 3, 1, 2)
    torch.testing.assert_close(dx, x.grad)


def test_fastdiv_formula():
    """host make_fastdiv / device fdiv (gemm_common.h) replayed in Python for the divisors the
    conv rows use."""
    for d in (1, 2, 3, 7, 27, 55, 169, 196, 729, 3025, 50176):
        s = 0
        while (1 << s) < d:
            s += 1
        m = ((1 << 32) * ((1 << s) - d)) // d + 1
        for n in list(range(0, 5000)) + [2 ** 31 - 1, 2 ** 31 - 2, 123456789]:
            q = (((n * m) >> 32) + n) >> s
            assert q == n // d, (d, n)
