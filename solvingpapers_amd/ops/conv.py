"""Implicit-GEMM convolution (HIP: csrc/kernels/conv.hip), K20.

Reference ops: the AlexNet convs (alexnet/alexnet.py:11-25) and the ViT patch embedding
(vision transformer/ViT.ipynb:186). The three conv GEMMs (fwd, data grad, weight grad) gather
their activation operand tile-by-tile from the image -- no im2col / col2im buffer.

Layouts. The kernels work on NHWC (channels padded to a multiple of 8) with K ordered
(kh, kw, c), or -- when KW, stride_w, pad_w and W are all multiples of 8, i.e. the ViT
patchify -- directly on the NCHW image with K ordered (c, kh, kw). Outputs are NHWC, returned
as channels-last tensors (logically NCHW), so a conv net stays channels-last from layer to layer
(LRN / max-pool / activations / dropout keep the layout) and no layout pass runs between convs.

Column tables. For every 8-column group of the implicit matrix, ``ktab`` holds (element offset,
dh, dw): the kernel adds the offset to the row's base address and bounds-checks h0 + dh,
w0 + dw for the padding taps. ``btab`` gives the packed-weight row of every data-grad K index.
Tables are built once per geometry (host, cached per device).
"""
from __future__ import annotations

import torch

from . import _ext

_TABLES: dict = {}


def _round8(c: int) -> int:
    return (c + 7) // 8 * 8


def nchw_direct_ok(C, H, W, KH, KW, sh, sw, ph, pw) -> bool:
    """NCHW gather with K = (c, kh, kw): 8 consecutive columns = 8 aligned contiguous pixels."""
    return KW % 8 == 0 and sw % 8 == 0 and pw % 8 == 0 and W % 8 == 0


def geometry(x_shape, w_shape, stride, padding, nhwc: bool):
    N, C, H, W = x_shape
    OC, _, KH, KW = w_shape
    sh, sw = stride
    ph, pw = padding
    OH, OW = (H + 2 * ph - KH) // sh + 1, (W + 2 * pw - KW) // sw + 1
    Cp = _round8(C) if nhwc else C
    return [int(nhwc), N, C, H, W, Cp, OC, KH, KW, sh, sw, ph, pw, OH, OW]


def fwd_table(geo) -> torch.Tensor:
    """int32 [K/8, 4]: (offset, dh, dw, 0) of each 8-column group of the implicit im2col X~."""
    nhwc, N, C, H, W, Cp, OC, KH, KW, sh, sw, ph, pw, OH, OW = geo
    k = torch.arange(0, KH * KW * Cp, 8, dtype=torch.int64)
    if nhwc:
        kh, kw, c = k // (KW * Cp), (k // Cp) % KW, k % Cp
        off = (kh * W + kw) * Cp + c
    else:
        c, kh, kw = k // (KH * KW), (k // KW) % KH, k % KW
        off = c * H * W + kh * W + kw
    return torch.stack([off, kh, kw, torch.zeros_like(k)], 1).to(torch.int32)


def dgrad_tables(geo):
    """(ktab over dY~ columns (kh, kw, oc), btab: packed-weight row offset of each such column)."""
    nhwc, N, C, H, W, Cp, OC, KH, KW, sh, sw, ph, pw, OH, OW = geo
    assert nhwc
    k = torch.arange(KH * KW * OC, dtype=torch.int64)
    kh, kw, oc = k // (KW * OC), (k // OC) % KW, k % OC
    btab = (oc * (KH * KW * Cp) + (kh * KW + kw) * Cp).to(torch.int32)
    g = k[::8]
    gkh, gkw, goc = kh[::8], kw[::8], oc[::8]
    if sh == 1 and sw == 1:
        off = -(gkh * OW + gkw) * OC + goc
    else:
        off = goc
    ktab = torch.stack([off, -gkh, -gkw, torch.zeros_like(g)], 1).to(torch.int32)
    return ktab, btab


def _cached(kind, geo, device, build):
    key = (kind, tuple(geo), str(device))
    t = _TABLES.get(key)
    if t is None:
        t = build(geo)
        t = tuple(v.to(device) for v in t) if isinstance(t, tuple) else t.to(device)
        if len(_TABLES) > 256:
            _TABLES.clear()
        _TABLES[key] = t
    return t


def _gathered(x, geo):
    """The image the kernels gather from: NCHW as is, or NHWC [N, H, W, Cp] bf16."""
    if not geo[0]:
        return x.contiguous()
    C, Cp = geo[2], geo[5]
    if C == Cp and x.dtype == torch.bfloat16 and x.is_contiguous(memory_format=torch.channels_last):
        return x.permute(0, 2, 3, 1)                       # already NHWC storage: free view
    return _ext.ops().conv_to_nhwc(x, Cp)


def _nhwc_dy(g):
    """dY as NHWC [N, OH, OW, OC] storage (free for the channels-last grads of our own outputs)."""
    if g.dtype == torch.bfloat16 and g.is_contiguous(memory_format=torch.channels_last):
        return g.permute(0, 2, 3, 1)
    return _ext.ops().conv_to_nhwc(g, g.shape[1])


class _ConvFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, stride, padding):
        N, C, H, W = x.shape
        KH, KW = w.shape[2], w.shape[3]
        nhwc = not (x.is_contiguous() and nchw_direct_ok(C, H, W, KH, KW, *stride, *padding))
        geo = geometry(x.shape, w.shape, stride, padding, nhwc)
        xg = _gathered(x, geo)
        wp = _ext.ops().conv_pack_weight(w, geo[5]) if nhwc else w.reshape(w.shape[0], -1).contiguous()
        ktab = _cached("fwd", geo, x.device, fwd_table)
        y = _ext.ops().conv_fwd(xg, wp, ktab, b, geo)       # NHWC [N, OH, OW, OC]
        ctx.save_for_backward(xg, w, wp if nhwc else None)
        ctx.geo, ctx.stride, ctx.padding, ctx.has_b = geo, stride, padding, b is not None
        ctx.x_cl = x.is_contiguous(memory_format=torch.channels_last) and not x.is_contiguous()
        return y.permute(0, 3, 1, 2)

    @staticmethod
    def backward(ctx, gy):
        xg, w, wp = ctx.saved_tensors
        geo = ctx.geo
        dy = _nhwc_dy(gy)
        dx = dw = db = None
        if ctx.needs_input_grad[1] or ctx.needs_input_grad[2]:
            dw, db = _ext.ops().conv_wgrad(dy, xg, _cached("fwd", geo, dy.device, fwd_table), geo,
                                           ctx.has_b and ctx.needs_input_grad[2], w.dtype)
            if not ctx.needs_input_grad[2]:
                db = None
        if ctx.needs_input_grad[0]:
            gn = geo if geo[0] else geometry(tuple(geo[1:5]), w.shape, ctx.stride, ctx.padding, True)
            if wp is None:
                wp = _ext.ops().conv_pack_weight(w, gn[5])
            ktab, btab = _cached("dgrad", gn, dy.device, dgrad_tables)
            dxp = _ext.ops().conv_dgrad(dy, wp, ktab, btab, gn)   # NHWC [N, H, W, Cp]
            C, Cp = gn[2], gn[5]
            dx = dxp.permute(0, 3, 1, 2) if (C == Cp and ctx.x_cl) else _ext.ops().conv_from_nhwc(dxp, C)
        return dx, dw, db, None, None


def conv2d_igemm(x, weight, bias=None, stride=(1, 1), padding=(0, 0)):
    """bf16 NCHW-logical conv on the implicit-GEMM kernels; returns a channels-last tensor."""
    if not _ext.load():
        raise RuntimeError("conv2d: HIP extension not built")
    if weight.shape[0] % 8:
        raise ValueError(f"conv2d: out channels must be a multiple of 8 (got {weight.shape[0]})")
    return _ConvFn.apply(x, weight, bias, tuple(stride), tuple(padding))
