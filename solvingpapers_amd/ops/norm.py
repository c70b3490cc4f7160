"""RMSNorm / LayerNorm with optional fused residual add (HIP: csrc/kernels/norm.hip).

``rms_norm(x, w, eps, residual=r)`` returns ``(norm(x + r), x + r)`` so a
pre-norm block reads the residual stream once; gradients of the weight go to
``w.main_grad`` when present (see utils/grad.py).
"""
from __future__ import annotations

import torch

from . import _ext, reference
from ..utils.grad import commit_tensor, direct_out as _direct_out


class _NormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, residual, w, b, eps):
        D = x.shape[-1]
        x2 = x.reshape(-1, D)
        r2 = residual.reshape(-1, D) if residual is not None else None
        y, h, rstd, mean = _ext.ops().norm_fwd(x2, r2, w, b, eps)
        hsave = h if residual is not None else x2
        ctx.has_res = residual is not None
        ctx.is_ln = b is not None
        ctx.w, ctx.b = w, b
        ctx.save_for_backward(hsave, rstd, mean if b is not None else rstd)
        ctx.shape = x.shape
        y = y.view(x.shape)
        if residual is not None:
            return y, h.view(x.shape)
        return y

    @staticmethod
    def backward(ctx, dy, dh=None):
        h, rstd, mean = ctx.saved_tensors
        D = ctx.shape[-1]
        dres = dh.reshape(-1, D).contiguous() if (ctx.has_res and dh is not None) else None
        # write dw/db straight into main_grad when this is the param's first commit of the iteration
        dw_out = _direct_out(ctx.w) if ctx.needs_input_grad[2] else None
        db_out = _direct_out(ctx.b) if (ctx.is_ln and ctx.needs_input_grad[3]) else None
        dx, dw, db = _ext.ops().norm_bwd(dy.reshape(-1, D).contiguous(), h, ctx.w, rstd,
                                         mean if ctx.is_ln else None, dres, dw_out, db_out)
        dx = dx.view(ctx.shape)
        gw = gb = None
        if ctx.needs_input_grad[2]:
            gw = None if dw_out is not None else commit_tensor(ctx.w, dw)
        if ctx.is_ln and ctx.needs_input_grad[3]:
            gb = None if db_out is not None else commit_tensor(ctx.b, db)
        if ctx.has_res:
            return dx, dx, gw, gb, None
        return dx, None, gw, gb, None


def _supported(x):
    return x.is_cuda and x.dtype in (torch.bfloat16, torch.float32) and x.shape[-1] % 8 == 0


def rms_norm(x, w, eps=1e-6, residual=None):
    """y = x*rsqrt(mean(x^2)+eps)*w. With ``residual``: returns (norm(x+r), x+r)."""
    if x.is_cuda:
        if not _supported(x):
            raise RuntimeError(f"rms_norm HIP kernel needs bf16/fp32 and D%8==0, got {x.dtype} {tuple(x.shape)}")
        return _NormFn.apply(x.contiguous(), residual.contiguous() if residual is not None else None, w, None, eps)
    y, h = reference.rms_norm(x, w, eps, residual)
    return (y, h) if residual is not None else y


def layer_norm(x, w, b, eps=1e-5, residual=None):
    if x.is_cuda:
        if not _supported(x):
            raise RuntimeError(f"layer_norm HIP kernel needs bf16/fp32 and D%8==0, got {x.dtype} {tuple(x.shape)}")
        return _NormFn.apply(x.contiguous(), residual.contiguous() if residual is not None else None, w, b, eps)
    y, h = reference.layer_norm(x, w, b, eps, residual)
    return (y, h) if residual is not None else y
