"""Cross-entropy with in-place logit gradients (HIP: csrc/kernels/xent.hip).

``cross_entropy(logits, target)`` = mean CE over non-ignored rows. On the GPU
the gradient (softmax - onehot)/N is computed during the forward pass and
stored over the (dead) logits buffer, so backward is a single scale by the
incoming scalar gradient; the [T, V] logits are never duplicated.
"""
from __future__ import annotations

import torch

from . import _ext
from . import reference
from .layout import wgrad
from ..utils.grad import commit, commit_tensor


class _XentFn(torch.autograd.Function):
    """CE whose gradient is written over the logits during forward. The logits
    buffer is CONSUMED (its producer must not need it for its own backward —
    true for a GEMM output); prefer :func:`linear_cross_entropy`, which never
    lets the logits escape."""

    @staticmethod
    def forward(ctx, logits, target, ignore_index, smoothing):
        V = logits.shape[-1]
        l2 = logits.reshape(-1, V)
        t = target.reshape(-1).contiguous()
        valid = (t != ignore_index).sum().clamp_min(1).float()
        inv = (1.0 / valid).reshape(1)
        loss, _ = _ext.ops().xent_fwd(l2, t, ignore_index, smoothing, True, inv)
        ctx.grad_buf = l2
        ctx.shape = logits.shape
        return loss.sum() * inv[0]

    @staticmethod
    def backward(ctx, g):
        grad = ctx.grad_buf
        ctx.grad_buf = None
        return grad.mul_(g.to(grad.dtype)).view(ctx.shape), None, None, None


class _LinearXentFn(torch.autograd.Function):
    """Fused LM head + cross-entropy: logits = h W^T (+b) -> CE; the logits
    buffer becomes d(loss)/d(logits) in place and is consumed by the two
    backward GEMMs (dh = G W, dW = G^T h written into W.main_grad)."""

    @staticmethod
    def forward(ctx, h, w, b, target, ignore_index, smoothing):
        D = h.shape[-1]
        h2 = h.reshape(-1, D)
        V = w.shape[0]
        # odd vocabularies (GPT-2's 50257) make every GEMM leading dimension misaligned;
        # run the head on a zero-padded copy (multiple of 128 rows: padded logits are exactly
        # 0 and are excluded from the softmax through the row stride), slice the results
        Vp = (V + 127) // 128 * 128 if V % 64 else V
        wp, bp = w, b
        if Vp != V:
            wp = w.new_zeros(Vp, D)
            wp[:V].copy_(w)
            if b is not None:
                bp = b.new_zeros(Vp)
                bp[:V].copy_(b)
        logits = torch.addmm(bp, h2, wp.t()) if bp is not None else torch.mm(h2, wp.t())
        t = target.reshape(-1).contiguous()
        valid = (t != ignore_index).sum().clamp_min(1).float()
        inv = (1.0 / valid).reshape(1)
        loss, _ = _ext.ops().xent_fwd(logits[:, :V], t, ignore_index, smoothing, True, inv)
        ctx.save_for_backward(h2)
        ctx.grad_buf, ctx.w, ctx.wp, ctx.b, ctx.hshape, ctx.V = logits, w, wp, b, h.shape, V
        return loss.sum() * inv[0]

    @staticmethod
    def backward(ctx, g):
        (h2,) = ctx.saved_tensors
        G = ctx.grad_buf
        ctx.grad_buf = None
        G.mul_(g.to(G.dtype))                 # padded columns are exactly 0
        w, b, wp = ctx.w, ctx.b, ctx.wp
        ctx.wp = None
        dh = torch.mm(G, wp).view(ctx.hshape) if ctx.needs_input_grad[0] else None
        G = G[:, :ctx.V]
        gw = gb = None
        if ctx.needs_input_grad[1]:
            def _w(out, acc):
                if out is not None and out.dtype != G.dtype:
                    g = wgrad(G, h2)
                    if acc:
                        out.add_(g)
                    else:
                        out.copy_(g)
                    return None
                return wgrad(G, h2, out, acc)
            gw = commit(w, _w)
        if b is not None and ctx.needs_input_grad[2]:
            gb = commit_tensor(b, G.float().sum(0).to(b.dtype))
        return dh, gw, gb, None, None, None


def linear_cross_entropy(h, w, target, bias=None, ignore_index=-100, label_smoothing=0.0):
    """mean CE(h @ w^T + bias, target) without exposing the [N, V] logits."""
    if h.is_cuda and h.dtype in (torch.bfloat16, torch.float32) and torch.is_grad_enabled() and (
            h.requires_grad or w.requires_grad):
        return _LinearXentFn.apply(h, w, bias, target, ignore_index, float(label_smoothing))
    logits = torch.nn.functional.linear(h, w, bias)
    return cross_entropy(logits, target, ignore_index, label_smoothing)


def cross_entropy(logits, target, ignore_index=-100, label_smoothing=0.0, reduction="mean"):
    """NOTE: on the GPU with grad enabled, ``logits`` is overwritten by its gradient."""
    if logits.is_cuda and logits.dtype in (torch.bfloat16, torch.float32):
        if reduction == "mean" and torch.is_grad_enabled() and logits.requires_grad:
            return _XentFn.apply(logits, target, ignore_index, float(label_smoothing))
        V = logits.shape[-1]
        loss, _ = _ext.ops().xent_fwd(logits.reshape(-1, V), target.reshape(-1).contiguous(), ignore_index,
                                      float(label_smoothing), False, None)
        if reduction == "none":
            return loss.view(target.shape)
        if reduction == "sum":
            return loss.sum()
        return loss.sum() / (target != ignore_index).sum().clamp_min(1)
    return torch.nn.functional.cross_entropy(logits.reshape(-1, logits.shape[-1]).float(), target.reshape(-1),
                                             ignore_index=ignore_index, label_smoothing=label_smoothing,
                                             reduction=reduction)


def per_row_loss(logits, target, ignore_index=-100):
    if logits.is_cuda:
        V = logits.shape[-1]
        return _ext.ops().xent_fwd(logits.reshape(-1, V), target.reshape(-1).contiguous(), ignore_index, 0.0,
                                   False, None)[0]
    return reference.cross_entropy(logits.reshape(-1, logits.shape[-1]), target.reshape(-1), ignore_index)
