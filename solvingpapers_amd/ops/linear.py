"""Linear layer whose weight gradient is written straight into ``main_grad``.

Plain projections are library GEMMs (hipBLASLt through torch.mm); what this
adds is gradient-accumulation fusion: dW = dY^T X is computed directly into
the flat gradient buffer (``torch.mm(out=)`` / ``addmm_``), so backward makes
no per-parameter grad allocation and no extra accumulate pass.
"""
from __future__ import annotations

import os

import torch

from ..utils.grad import commit
from . import _ext
from .layout import wgrad

# decode-time products with <= 4 token rows go to the GEMV kernel; SPA_GEMV=0 -> torch.mm
GEMV = os.environ.get("SPA_GEMV", "1") != "0"
GEMV_MAX_ROWS = 4


class _LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b):
        ctx.w, ctx.b = w, b
        ctx.save_for_backward(x)
        x2 = x.reshape(-1, x.shape[-1])
        if b is not None:
            y = torch.addmm(b, x2, w.t())
        else:
            y = torch.mm(x2, w.t())
        # _unsafe_view: the output is a fresh tensor, not an autograd view, so
        # downstream in-place kernels (packed RoPE) may modify it
        return torch.ops.aten._unsafe_view(y, (*x.shape[:-1], w.shape[0]))

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        w, b = ctx.w, ctx.b
        dy2 = dy.reshape(-1, dy.shape[-1])
        x2 = x.reshape(-1, x.shape[-1])
        dx = torch.mm(dy2, w).view(x.shape) if ctx.needs_input_grad[0] else None
        gw = gb = None
        if ctx.needs_input_grad[1]:
            def _w(out, acc):
                if out is not None and out.dtype != dy2.dtype:
                    g = wgrad(dy2, x2)
                    if acc:
                        out.add_(g)
                    else:
                        out.copy_(g)
                    return None
                return wgrad(dy2, x2, out, acc)
            gw = commit(w, _w)
        if b is not None and ctx.needs_input_grad[2]:
            def _b(out, acc):
                s = dy2.sum(0, dtype=torch.float32)
                if out is None:
                    return s.to(b.dtype)
                if acc:
                    out.add_(s.to(out.dtype))
                else:
                    out.copy_(s)
            gb = commit(b, _b)
        return dx, gw, gb


def _gemv_ok(x, w, b) -> bool:
    """Decode-shaped inference product (<= GEMV_MAX_ROWS token rows, no autograd): routed to
    the weight-streaming GEMV kernel (csrc/kernels/gemv.hip) instead of a library GEMM."""
    if not (GEMV and b is None and x.is_cuda and x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16):
        return False
    if torch.is_grad_enabled() and (x.requires_grad or w.requires_grad):
        return False
    K = x.shape[-1]
    rows = x.numel() // K if K else 0
    return (1 <= rows <= GEMV_MAX_ROWS and K % 8 == 0 and w.dim() == 2 and w.stride(1) == 1
            and w.stride(0) % 8 == 0 and w.data_ptr() % 16 == 0 and x.stride(-1) == 1
            and x.data_ptr() % 16 == 0)


def linear(x, w, b=None):
    if _gemv_ok(x, w, b):
        x2 = x.reshape(-1, x.shape[-1])
        if x2.stride(0) % 8:
            x2 = x2.contiguous()
        return _ext.ops().gemv(x2, w).view(*x.shape[:-1], w.shape[0])
    return _LinearFn.apply(x, w, b)


class Linear(torch.nn.Module):
    """nn.Linear-compatible (weight [out, in]) module using :func:`linear`."""

    def __init__(self, in_features, out_features, bias=True, device=None, dtype=None):
        super().__init__()
        self.in_features, self.out_features = in_features, out_features
        self.weight = torch.nn.Parameter(torch.empty(out_features, in_features, device=device, dtype=dtype))
        self.bias = torch.nn.Parameter(torch.empty(out_features, device=device, dtype=dtype)) if bias else None
        self.reset_parameters()

    def reset_parameters(self):
        torch.nn.init.kaiming_uniform_(self.weight, a=5 ** 0.5)
        if self.bias is not None:
            bound = 1 / self.in_features ** 0.5
            torch.nn.init.uniform_(self.bias, -bound, bound)

    def forward(self, x):
        return linear(x, self.weight, self.bias)

    def extra_repr(self):
        return f"in_features={self.in_features}, out_features={self.out_features}, bias={self.bias is not None}"
