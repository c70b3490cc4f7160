"""Embedding gather / scatter-add (HIP: csrc/kernels/embedding.hip).

Optional fused additive position table (GPT learned pos_embed, DeepSeek
sinusoidal pe) and multiplicative scale (Gemma sqrt(D)). A negative id gives a zero row
and no table gradient (vocab-parallel embedding: tokens of other ranks' shards). The table gradient is
committed to ``W.main_grad`` when present: written in place by ``emb_bwd_into``, which
touches only the rows of the batch's tokens (fp32 scratch + row flags, then a flush of the
flagged rows) instead of materialising a dense [V, D] gradient per call.
"""
from __future__ import annotations

import torch

from . import _ext, reference
from ..utils.grad import claim_main_grad, commit_tensor


class _EmbFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, W, idx, pos, scale):
        ctx.save_for_backward(idx)
        ctx.W, ctx.pos, ctx.scale = W, pos, scale
        return _ext.ops().emb_fwd(W, idx, pos, scale)

    @staticmethod
    def backward(ctx, g):
        (idx,) = ctx.saved_tensors
        W = ctx.W
        gw = gp = None
        if ctx.needs_input_grad[0]:
            claim = claim_main_grad(W)
            if claim is not None and g.dtype == W.dtype:
                # straight into the flat gradient buffer, touching only the batch's rows
                mg, accumulate = claim
                _ext.ops().emb_bwd_into(g.contiguous(), idx, ctx.scale, mg, accumulate)
            else:
                dW = _ext.ops().emb_bwd(g.contiguous(), idx, W.shape[0], ctx.scale, W)
                gw = commit_tensor(W, dW)
        if ctx.pos is not None and ctx.needs_input_grad[2]:
            T = idx.shape[-1]
            D = W.shape[1]
            dpos = g.reshape(-1, T, D).float().sum(0)
            full = torch.zeros(ctx.pos.shape, dtype=torch.float32, device=g.device)
            full.view(-1, D)[:T] = dpos
            gp = commit_tensor(ctx.pos, full.to(ctx.pos.dtype))
        return gw, None, gp, None


def embedding(W, idx, pos=None, scale=1.0):
    if W.is_cuda and W.dtype in (torch.bfloat16, torch.float32) and W.shape[1] % 8 == 0:
        return _EmbFn.apply(W, idx, pos, float(scale))
    return reference.embedding(W, idx, pos, scale)
