"""Direct-to-buffer gradient commits ("main_grad").

Parameters that live in a :class:`~solvingpapers_amd.utils.flat.FlatParams`
carry a ``main_grad`` view into a contiguous gradient buffer. The fused ops
(linear, norms, embedding, ...) write their weight gradient straight into that
view — GEMM ``out=`` on the first write of an iteration, ``addmm_`` afterwards
(tied weights, gradient accumulation) — and return ``None`` to autograd, so no
per-parameter ``.grad`` tensor is ever allocated or copied.
"""
from __future__ import annotations

from typing import Callable, Optional

import torch


class _Gen:
    value = 0


def next_generation():
    """Start a new gradient iteration: the next commit to each param overwrites."""
    _Gen.value += 1


def commit(p: torch.Tensor, compute: Callable[[Optional[torch.Tensor], bool], Optional[torch.Tensor]]):
    """Commit a parameter gradient.

    ``compute(out, accumulate)`` must write into ``out`` (overwriting or adding)
    when ``out`` is given, or return a fresh gradient tensor when ``out`` is None.
    Returns the tensor autograd should receive (None if it went to main_grad).
    """
    mg = getattr(p, "main_grad", None)
    if mg is None:
        return compute(None, False)
    if getattr(p, "_spa_gen", -1) != _Gen.value:
        compute(mg, False)
        p._spa_gen = _Gen.value
    else:
        compute(mg, True)
    return None


def direct_out(p: torch.Tensor):
    """If ``p``'s next commit is an overwrite and the main_grad view is contiguous
    with p's dtype, claim it and return it so a kernel can write the gradient
    straight into it (no temporary + copy). Returns None otherwise."""
    mg = getattr(p, "main_grad", None)
    if mg is None or getattr(p, "_spa_gen", -1) == _Gen.value or mg.dtype != p.dtype or not mg.is_contiguous():
        return None
    p._spa_gen = _Gen.value
    return mg


def claim_main_grad(p: torch.Tensor):
    """For a kernel that writes OR accumulates into the gradient buffer itself: returns
    ``(main_grad, accumulate)`` -- accumulate is False on the first commit of this iteration --
    and marks the commit, or None when ``p`` has no contiguous main_grad of its own dtype."""
    mg = getattr(p, "main_grad", None)
    if mg is None or mg.dtype != p.dtype or not mg.is_contiguous():
        return None
    accumulate = getattr(p, "_spa_gen", -1) == _Gen.value
    p._spa_gen = _Gen.value
    return mg, accumulate


def commit_tensor(p: torch.Tensor, g: torch.Tensor):
    """Commit an already-computed gradient tensor."""
    def _c(out, acc):
        if out is None:
            return g
        if acc:
            out.add_(g.view_as(out))
        else:
            out.copy_(g.view_as(out))
        return None
    return commit(p, _c)


class GradReadyMarker(torch.autograd.Function):
    """Identity whose backward signals that every parameter gradient downstream
    of this point (i.e. of the block it guards) has been committed. Used to launch
    per-layer gradient buckets (all-reduce / reduce-scatter) during backward."""

    @staticmethod
    def forward(ctx, x, callback, key):
        ctx.callback = callback
        ctx.key = key
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        ctx.callback(ctx.key)
        return g, None, None


def mark_ready(x: torch.Tensor, callback, key):
    if callback is None or not torch.is_grad_enabled():
        return x
    return GradReadyMarker.apply(x, callback, key)
