"""Flash attention (HIP: csrc/kernels/attention.hip) with GQA/MQA head mapping.

Tensors are [B, T, H, hd] views (hd contiguous); the kernels take (b, t, h)
strides, so q/k/v may be slices of one packed qkv projection output and the
gradients can be written into slices of one dqkv buffer (``attention_packed``).
Head dims 64/128/256 run the MFMA flash kernel; other q/k and v head dims up to
256 (DeepSeek-V3 MLA's 192/128) are zero-padded onto it; wider heads fall back to
a materialised GEMM + softmax path (used only by reference-parity presets such
as Gemma-ref's 768-wide heads).
"""
from __future__ import annotations

import math

import torch

from . import _ext, reference

FLASH_HD = (64, 128, 256)


def _flash_ok(q):
    return q.is_cuda and q.dtype == torch.bfloat16 and (q.dim() == 3 or q.shape[-1] in FLASH_HD)


class _FlashFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, causal, scale):
        out, lse = _ext.ops().attn_fwd(q, k, v, scale, causal)
        ctx.save_for_backward(q, k, v, out, lse)
        ctx.causal, ctx.scale = causal, scale
        return out

    @staticmethod
    def backward(ctx, dout):
        q, k, v, out, lse = ctx.saved_tensors
        dq = torch.empty_like(q, memory_format=torch.contiguous_format)
        dk = torch.empty_like(k, memory_format=torch.contiguous_format)
        dv = torch.empty_like(v, memory_format=torch.contiguous_format)
        _ext.ops().attn_bwd(dout.contiguous(), q, k, v, out, lse, dq, dk, dv, ctx.scale, ctx.causal)
        return dq, dk, dv, None, None


class _PackedFn(torch.autograd.Function):
    """Attention reading q/k/v from one [B, T, (H+2Hkv)*hd] buffer and writing the
    three gradients into one dqkv buffer of the same layout (no cat/split).
    Output is [B, T, H*hd] (a fresh tensor, ready for the output projection)."""

    @staticmethod
    def forward(ctx, qkv, H, Hkv, hd, causal, scale):
        B, T = qkv.shape[0], qkv.shape[1]
        x4 = qkv.view(B, T, H + 2 * Hkv, hd)
        q, k, v = x4[:, :, :H], x4[:, :, H:H + Hkv], x4[:, :, H + Hkv:]
        out, lse = _ext.ops().attn_fwd(q, k, v, scale, causal)
        ctx.save_for_backward(qkv, out, lse)
        ctx.H, ctx.Hkv, ctx.hd, ctx.causal, ctx.scale = H, Hkv, hd, causal, scale
        return torch.ops.aten._unsafe_view(out, (B, T, H * hd))

    @staticmethod
    def backward(ctx, dout):
        qkv, out, lse = ctx.saved_tensors
        H, Hkv, hd = ctx.H, ctx.Hkv, ctx.hd
        B, T = qkv.shape[0], qkv.shape[1]
        dqkv = torch.empty_like(qkv)
        x4 = qkv.view(B, T, H + 2 * Hkv, hd)
        d4 = dqkv.view(B, T, H + 2 * Hkv, hd)
        _ext.ops().attn_bwd(dout.contiguous().view(B, T, H, hd), x4[:, :, :H], x4[:, :, H:H + Hkv],
                            x4[:, :, H + Hkv:], out, lse, d4[:, :, :H], d4[:, :, H:H + Hkv], d4[:, :, H + Hkv:],
                            ctx.scale, ctx.causal)
        return dqkv, None, None, None, None, None


def _materialised(q, k, v, causal, scale):
    """GEMM + softmax path for unsupported head dims (autograd through torch ops)."""
    B, Tq, H, hd = q.shape
    Tk, Hkv = k.shape[1], k.shape[2]
    rep = H // Hkv
    qh = q.transpose(1, 2)
    kh = k.transpose(1, 2).repeat_interleave(rep, dim=1)
    vh = v.transpose(1, 2).repeat_interleave(rep, dim=1)
    s = torch.matmul(qh, kh.transpose(-1, -2)).float() * scale
    if causal:
        i = torch.arange(Tq, device=q.device)[:, None]
        j = torch.arange(Tk, device=q.device)[None, :]
        s = s.masked_fill(j > i + (Tk - Tq), float("-inf"))
    p = torch.softmax(s, dim=-1).to(q.dtype)
    return torch.matmul(p, vh).transpose(1, 2)


def _flash_pad_dim(dqk, dv):
    """Smallest flash head dim that holds both the q/k and the v head dim (None: none does)."""
    return next((h for h in FLASH_HD if h >= max(dqk, dv)), None)


def _pad_last(x, n):
    return x if x.shape[-1] == n else torch.nn.functional.pad(x, (0, n - x.shape[-1]))


def flash_attention(q, k, v, causal=True, scale=None):
    """softmax(q k^T * scale [+causal]) v.  q/k [B,T,H(kv),dqk], v [B,Tk,Hkv,dv].

    dqk == dv in FLASH_HD runs the MFMA kernel directly. Other head dims up to 256
    (DeepSeek-V3 MLA: dqk = 128 nope + 64 rope = 192, dv = 128) are zero-padded to
    the next kernel head dim: zero q/k columns leave every score unchanged, zero v
    columns give zero output columns that are sliced off, and the pad's backward
    slices the gradients. O(T) memory instead of the materialised O(T^2) path."""
    scale = float(scale) if scale is not None else 1.0 / math.sqrt(q.shape[-1])
    if _flash_ok(q) and v.shape[-1] == q.shape[-1]:
        return _FlashFn.apply(q, k, v, causal, scale)
    if q.is_cuda and q.dtype == torch.bfloat16 and q.dim() == 4:
        P = _flash_pad_dim(q.shape[-1], v.shape[-1])
        if P is not None:
            o = _FlashFn.apply(_pad_last(q, P), _pad_last(k, P), _pad_last(v, P), causal, scale)
            return o[..., :v.shape[-1]]
    if q.is_cuda:
        return _materialised(q, k, v, causal, scale)
    if torch.is_grad_enabled() and (q.requires_grad or k.requires_grad or v.requires_grad):
        return _materialised(q, k, v, causal, scale)
    return reference.attention(q, k, v, causal, scale)[0]


def attention_packed(qkv, H, Hkv, causal=True, scale=None, head_dim=None):
    """qkv [B, T, H+2Hkv, hd] (or [B, T, (H+2Hkv)*hd] with head_dim) -> out [B, T, H*hd]."""
    hd = head_dim if head_dim is not None else qkv.shape[-1]
    B, T = qkv.shape[0], qkv.shape[1]
    scale = float(scale) if scale is not None else 1.0 / math.sqrt(hd)
    if qkv.is_cuda and qkv.dtype == torch.bfloat16 and hd in FLASH_HD:
        return _PackedFn.apply(qkv, H, Hkv, hd, causal, scale)
    x4 = qkv.view(B, T, H + 2 * Hkv, hd)
    q, k, v = x4[:, :, :H], x4[:, :, H:H + Hkv], x4[:, :, H + Hkv:]
    return flash_attention(q, k, v, causal, scale).reshape(B, T, H * hd)


def attention_dropout(q, k, v, causal=True, scale=None, p=0.0, training=True, neg=float("-inf")):
    """Materialised attention with dropout on the probability matrix (GPT-ref
    gpt/gpt-jax.ipynb:351 / DeepSeek-ref attention dropout). Used only when a
    reference preset trains with attention-weight dropout; inference and p=0 take
    the flash kernels. q [B,Tq,H,hd], k/v [B,Tk,Hkv,hd]."""
    from .misc import dropout
    if not training or p == 0.0:
        return flash_attention(q, k, v, causal, scale)
    B, Tq, H, hd = q.shape
    Tk, Hkv = k.shape[1], k.shape[2]
    scale = float(scale) if scale is not None else 1.0 / math.sqrt(hd)
    rep = H // Hkv
    qh = q.transpose(1, 2)
    kh = k.transpose(1, 2).repeat_interleave(rep, dim=1)
    vh = v.transpose(1, 2).repeat_interleave(rep, dim=1)
    s = torch.matmul(qh, kh.transpose(-1, -2)).float() * scale
    if causal:
        i = torch.arange(Tq, device=q.device)[:, None]
        j = torch.arange(Tk, device=q.device)[None, :]
        s = s.masked_fill(j > i + (Tk - Tq), neg)
    pr = dropout(torch.softmax(s, dim=-1).to(q.dtype), p, training)
    return torch.matmul(pr, vh).transpose(1, 2)


DECODE_MAX_ROWS = 16


def _decode_ok(q, k, v):
    if not (q.is_cuda and q.dtype == torch.bfloat16 and q.dim() == 4 and q.shape[-1] in FLASH_HD):
        return False
    B, Tq, H, hd = q.shape
    Hkv = k.shape[2]
    if H % Hkv or Tq * (H // Hkv) > DECODE_MAX_ROWS or Tq > k.shape[1]:
        return False
    return all(t.stride(3) == 1 and t.stride(0) % 4 == 0 and t.stride(1) % 4 == 0 and t.stride(2) % 4 == 0
               and t.data_ptr() % 8 == 0 for t in (q, k, v))


def decode_attention(q, k, v, causal=True, scale=None, nsplit=0, kv_len=None):
    """Few new query rows against a KV cache: q [B,Tq,H,hd], k/v [B,Tk,Hkv,hd] (cache views,
    the last Tq cache rows are the query tokens). Split-K HIP kernel (csrc/kernels/decode.hip)
    when Tq * H / Hkv <= 16, else the flash kernel. Inference only (no autograd).

    ``kv_len`` (device int32 [1]): k/v are whole cache buffers and only the first *kv_len
    rows are valid -- the form a captured hipGraph decode step replays at every position."""
    scale = float(scale) if scale is not None else 1.0 / math.sqrt(q.shape[-1])
    if _decode_ok(q, k, v):
        return _ext.ops().attn_decode(q, k, v, scale, causal, int(nsplit), kv_len)[0]
    if kv_len is not None:
        raise ValueError("decode_attention: kv_len needs the decode kernel (Tq * H / Hkv <= 16, bf16 on the GPU)")
    return flash_attention(q.contiguous(), k, v, causal, scale)
