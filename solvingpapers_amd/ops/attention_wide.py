"""Wide-head flash attention (HIP: csrc/kernels/attention_wide.hip) for head dims 512 / 768 -- Gemma-ref's two 768-wide query heads over one shared 768-wide K/V head
(gemma/gemma.ipynb:238-249). The head dim is processed in 256-wide chunks: reductions over it
(QK^T, dO V^T) span every chunk, each output (O, dQ, dK, dV) is produced one chunk per
workgroup. O(T) memory, no materialised (T, T) scores."""
from __future__ import annotations

import torch

from . import _ext


class _WideFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, causal, scale):
        out, lse = _ext.ops().attn_wide_fwd(q, k, v, scale, causal)
        ctx.save_for_backward(q, k, v, out, lse)
        ctx.causal, ctx.scale = causal, scale
        return out

    @staticmethod
    def backward(ctx, dout):
        q, k, v, out, lse = ctx.saved_tensors
        dq = torch.empty_like(q, memory_format=torch.contiguous_format)
        dk = torch.empty_like(k, memory_format=torch.contiguous_format)
        dv = torch.empty_like(v, memory_format=torch.contiguous_format)
        _ext.ops().attn_wide_bwd(dout.contiguous(), q, k, v, out, lse, dq, dk, dv, ctx.scale, ctx.causal)
        return dq, dk, dv, None, None


def wide_attention(q, k, v, causal=True, scale=None):
    """q [B,Tq,H,D], k/v [B,Tk,Hkv,D] bf16 on the GPU, D in (512, 768)."""
    import math
    scale = float(scale) if scale is not None else 1.0 / math.sqrt(q.shape[-1])
    return _WideFn.apply(q, k, v, bool(causal), scale)
