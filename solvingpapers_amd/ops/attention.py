"""Flash attention (HIP: csrc/kernels/attention.hip) with GQA/MQA head mapping.

Tensors are [B, T, H, hd] views (hd contiguous); the kernels take (b, t, h)
strides, so q/k/v may be slices of one packed qkv projection output and the
gradients can be written into slices of one dqkv buffer (``attention_packed``).

Kernel head dims (q/k, v): (64, 64), (128, 128), (256, 256) and DeepSeek-V3 MLA's
(192, 128), all without padding. Other dims up to 256 are zero-padded onto the
smallest kernel pair that holds them; wider heads (Gemma-ref's 768) take the wide-head
kernels (csrc/kernels/attention_wide.hip).

Attention-probability dropout is fused into the kernels (counter-hash mask regenerated
from a per-call seed in the forward and both backward kernels; nothing (T, T) is stored).
``dropout_keep_mask`` reproduces the exact mask on the host for oracles.
"""
from __future__ import annotations

import math

import os

import torch

from . import _ext, reference

FLASH_PAIRS = ((64, 64), (128, 128), (256, 256), (192, 128))
FLASH_HD = (64, 128, 256)


def _pair_for(dqk, dv):
    """Smallest kernel (q/k, v) head-dim pair holding (dqk, dv) (None: none does)."""
    best = None
    for a, b in FLASH_PAIRS:
        if a >= dqk and b >= dv and (best is None or a + b < best[0] + best[1]):
            best = (a, b)
    return best


def _flash_ok(q):
    return q.is_cuda and q.dtype == torch.bfloat16 and (q.dim() == 3 or q.shape[-1] in FLASH_HD)


# ------------------------------------------------------------------ dropout mask (host)
_M32 = 0xFFFFFFFF


def _mix32(x):
    x = x ^ (x >> 16)
    x = (x * 0x7FEB352D) & _M32
    x = x ^ (x >> 15)
    x = (x * 0x846CA68B) & _M32
    return x ^ (x >> 16)


def dropout_keep_mask(seed: int, B: int, H: int, Tq: int, Tk: int, p: float, device="cpu"):
    """Bool [B, H, Tq, Tk]: the keep mask the fused kernels apply for ``seed`` (same 32-bit
    counter hash as csrc/kernels/attention.hip drop_keep)."""
    thr = int(round(p * 16777216.0))
    lo, hi = seed & _M32, (seed >> 32) & _M32
    bh = torch.arange(B * H, device=device, dtype=torch.int64)
    base = _mix32(lo ^ _mix32((hi + bh * 0x9E3779B9) & _M32))             # [B*H]
    q = torch.arange(Tq, device=device, dtype=torch.int64)
    k = torch.arange(Tk, device=device, dtype=torch.int64)
    x = (base[:, None, None] + (q * 0x85EBCA6B)[None, :, None] + (k * 0xC2B2AE35)[None, None, :]) & _M32
    return ((_mix32(x) >> 8) >= thr).view(B, H, Tq, Tk)


def _new_seed() -> int:
    return int(torch.randint(0, 2 ** 62, (1,)).item())   # host generator: no device sync


def _seed_args(seed):
    """(int seed, device seed tensor or None): a tensor seed is read by the kernels on the
    device, so a captured HIP graph draws a fresh mask at every replay."""
    if isinstance(seed, torch.Tensor):
        return 0, seed
    return int(seed or 0), None


class _FlashFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, causal, scale, dropout_p, seed):
        si, st = _seed_args(seed)
        out, lse = _ext.ops().attn_fwd(q, k, v, scale, causal, dropout_p, si, st)
        ctx.save_for_backward(q, k, v, out, lse)
        ctx.causal, ctx.scale, ctx.dropout_p, ctx.seed = causal, scale, dropout_p, seed
        return out

    @staticmethod
    def backward(ctx, dout):
        q, k, v, out, lse = ctx.saved_tensors
        dq = torch.empty_like(q, memory_format=torch.contiguous_format)
        dk = torch.empty_like(k, memory_format=torch.contiguous_format)
        dv = torch.empty_like(v, memory_format=torch.contiguous_format)
        si, st = _seed_args(ctx.seed)
        _ext.ops().attn_bwd(dout.contiguous(), q, k, v, out, lse, dq, dk, dv, ctx.scale, ctx.causal,
                            ctx.dropout_p, si, st)
        return dq, dk, dv, None, None, None, None


class _PackedFn(torch.autograd.Function):
    """Attention reading q/k/v from one [B, T, (H+2Hkv)*hd] buffer and writing the
    three gradients into one dqkv buffer of the same layout (no cat/split).
    Output is [B, T, H*hd] (a fresh tensor, ready for the output projection)."""

    @staticmethod
    def forward(ctx, qkv, H, Hkv, hd, causal, scale, dropout_p=0.0, seed=0):
        B, T = qkv.shape[0], qkv.shape[1]
        x4 = qkv.view(B, T, H + 2 * Hkv, hd)
        q, k, v = x4[:, :, :H], x4[:, :, H:H + Hkv], x4[:, :, H + Hkv:]
        si, st = _seed_args(seed)
        out, lse = _ext.ops().attn_fwd(q, k, v, scale, causal, dropout_p, si, st)
        ctx.save_for_backward(qkv, out, lse)
        ctx.H, ctx.Hkv, ctx.hd, ctx.causal, ctx.scale = H, Hkv, hd, causal, scale
        ctx.dropout_p, ctx.seed = dropout_p, seed
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
                            ctx.scale, ctx.causal, ctx.dropout_p, *_seed_args(ctx.seed))
        return dqkv, None, None, None, None, None, None, None


FLASH_F32_HD = (16, 32, 64, 128, 256)


class _FlashF32Fn(torch.autograd.Function):
    """fp32 flash attention (csrc/kernels/attention_f32.hip, fp32 MFMA): the reference's training
    precision (gpt/gpt-jax.ipynb:344-353, llama3/LLaMA-jax.ipynb:809-829) on a HIP kernel."""

    @staticmethod
    def forward(ctx, q, k, v, causal, scale, dropout_p, seed):
        si, st = _seed_args(seed)
        out, lse = _ext.ops().attn_f32_fwd(q, k, v, scale, causal, dropout_p, si, st)
        ctx.save_for_backward(q, k, v, out, lse)
        ctx.causal, ctx.scale, ctx.dropout_p, ctx.seed = causal, scale, dropout_p, seed
        return out

    @staticmethod
    def backward(ctx, dout):
        q, k, v, out, lse = ctx.saved_tensors
        dq, dk, dv = (torch.empty(t.shape, dtype=t.dtype, device=t.device) for t in (q, k, v))
        si, st = _seed_args(ctx.seed)
        _ext.ops().attn_f32_bwd(dout.contiguous(), q, k, v, out, lse, dq, dk, dv, ctx.scale, ctx.causal,
                                ctx.dropout_p, si, st)
        return dq, dk, dv, None, None, None, None


def _f32_ready(t, hd):
    """t padded to head dim hd, with 16-byte-aligned rows (the fp32 kernel's float4 accesses)."""
    t = _pad_last(t, hd)
    if t.stride(-1) != 1 or any(s % 4 for s in t.stride()[:-1]) or t.data_ptr() % 16:
        t = t.contiguous()
    return t


def _materialised(q, k, v, causal, scale, dropout_p=0.0, seed=0, neg=float("-inf")):
    """GEMM + softmax path (CPU autograd, and the oracle of the fused kernels): with
    ``dropout_p`` it applies exactly the kernels' hash mask for ``seed``."""
    B, Tq, H, hd = q.shape
    Tk, Hkv = k.shape[1], k.shape[2]
    rep = H // Hkv
    qh = q.transpose(1, 2)
    kh = k.transpose(1, 2).repeat_interleave(rep, dim=1)
    vh = v.transpose(1, 2).repeat_interleave(rep, dim=1)
    s = torch.matmul(qh, kh.transpose(-1, -2))
    s = (s if s.dtype == torch.float64 else s.float()) * scale      # fp64 parity tests keep fp64
    if causal:
        i = torch.arange(Tq, device=q.device)[:, None]
        j = torch.arange(Tk, device=q.device)[None, :]
        s = s.masked_fill(j > i + (Tk - Tq), neg)
    p = torch.softmax(s, dim=-1)
    if dropout_p > 0.0:
        keep = dropout_keep_mask(seed, B, H, Tq, Tk, dropout_p, device=q.device)
        p = p * keep / (1.0 - dropout_p)
    return torch.matmul(p.to(q.dtype), vh).transpose(1, 2)


def _pad_last(x, n):
    return x if x.shape[-1] == n else torch.nn.functional.pad(x, (0, n - x.shape[-1]))


def _wide_ok(q, k, v):
    return (q.is_cuda and q.dtype == torch.bfloat16 and q.dim() == 4 and q.shape[-1] == v.shape[-1]
            and q.shape[-1] in (512, 768))


def flash_attention(q, k, v, causal=True, scale=None, dropout_p=0.0, seed=None):
    """softmax(q k^T * scale [+causal]) [dropout] v.  q/k [B,T,H(kv),dqk], v [B,Tk,Hkv,dv].

    (dqk, dv) in FLASH_PAIRS runs the MFMA kernel directly (MLA's 192/128 included). Other
    head dims up to 256 are zero-padded to the smallest kernel pair: zero q/k columns leave
    every score unchanged, zero v columns give zero output columns that are sliced off, and
    the pad's backward slices the gradients. ``dropout_p`` > 0 fuses dropout on P into the
    kernels (``seed`` drawn from torch's host generator when None)."""
    scale = float(scale) if scale is not None else 1.0 / math.sqrt(q.shape[-1])
    dropout_p = float(dropout_p)
    if dropout_p > 0.0 and seed is None:
        # on the GPU a device seed (torch's graph-capture-safe generator): fresh mask per replay
        seed = torch.randint(0, 2 ** 62, (1,), device=q.device, dtype=torch.int64) if q.is_cuda else _new_seed()
    if not isinstance(seed, torch.Tensor):
        seed = int(seed or 0)
    dqk, dv = q.shape[-1], v.shape[-1]
    if q.is_cuda and q.dtype == torch.bfloat16 and q.dim() == 4:
        if (dqk, dv) in FLASH_PAIRS and (dropout_p == 0.0 or dqk == dv):
            return _FlashFn.apply(q, k, v, causal, scale, dropout_p, seed)
        pair = _pair_for(dqk, dv) if dropout_p == 0.0 else _pair_for(max(dqk, dv), max(dqk, dv))
        if pair is not None:
            o = _FlashFn.apply(_pad_last(q, pair[0]), _pad_last(k, pair[0]), _pad_last(v, pair[1]), causal, scale,
                               dropout_p, seed)
            return o[..., :dv]
        if _wide_ok(q, k, v) and dropout_p == 0.0:
            from .attention_wide import wide_attention
            return wide_attention(q, k, v, causal, scale)
    if q.is_cuda and q.dtype == torch.float32 and q.dim() == 4 and max(dqk, dv) <= 256:
        # fp32 (the reference's precision in the parity runs): the fp32-MFMA kernels, head dims
        # zero-padded to the next of 16 / 32 / 64 / 128 / 256 exactly as above
        hd = next(h for h in FLASH_F32_HD if h >= max(dqk, dv))
        o = _FlashF32Fn.apply(_f32_ready(q, hd), _f32_ready(k, hd), _f32_ready(v, hd), causal, scale, dropout_p,
                              seed)
        return o if dv == hd else o[..., :dv]
    if q.is_cuda:
        # no flash kernel for this dtype / head-dim pair (fp16, or wider than 256 in fp32): GEMM +
        # softmax on the GPU
        return _materialised(q, k, v, causal, scale, dropout_p, seed)
    if dropout_p > 0.0 or (torch.is_grad_enabled() and (q.requires_grad or k.requires_grad or v.requires_grad)):
        return _materialised(q, k, v, causal, scale, dropout_p, seed)
    return reference.attention(q, k, v, causal, scale)[0]


class _MLAFn(torch.autograd.Function):
    """DeepSeek-V3 MLA attention core on the (192, 128) (or hd-128) flash kernels with the head assembly
    fused around them (deepseekv3/deepseekv3.ipynb:1152-1189 for the reference's latent heads):

    forward:  q = q_raw with RoPE on its last dr columns (one copy + one in-place rope),
              k = [kv_nope | rope(kr) broadcast over heads] (two strided copies),
              v = the strided view kv[..., dn:] (no copy);
    backward: the flash backward writes dV straight into the dkv buffer's v columns,
              dK's nope columns are copied next to it, dK's rope columns are summed over heads
              in one fp32 reduction, and both rope gradients are rotated back in place.

    The op-by-op form (slices, two torch.cat, out-of-place rope) paid a zero-fill + copy per
    sliced input and an add per reused tensor in the backward."""

    @staticmethod
    def forward(ctx, q_raw, kv, kr, dn, scale, pos_off, theta):
        from .rope import RopeCache
        ops = _ext.ops()
        B, T, H, dqk = q_raw.shape
        dr = dqk - dn
        cos, sin = RopeCache.get(pos_off + T, dr, theta, q_raw.device)
        q = q_raw.contiguous().clone()
        ops.rope_(q[..., dn:], cos, sin, None, H, pos_off, 0, False)
        krr = kr.contiguous().clone()
        ops.rope_(krr, cos, sin, None, 1, pos_off, 0, False)
        k = torch.empty(B, T, H, dqk, device=q.device, dtype=q.dtype)
        k[..., :dn].copy_(kv[..., :dn])
        k[..., dn:].copy_(krr.expand(B, T, H, dr))
        out, lse = ops.attn_fwd(q, k, kv[..., dn:], scale, True, 0.0, 0, None)
        ctx.save_for_backward(q, k, kv, out, lse)
        ctx.args = (dn, scale, pos_off, cos, sin)
        return out

    @staticmethod
    def backward(ctx, do):
        ops = _ext.ops()
        q, k, kv, out, lse = ctx.saved_tensors
        dn, scale, pos_off, cos, sin = ctx.args
        H = q.shape[2]
        dq, dk, dkv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(kv)
        ops.attn_bwd(do.contiguous(), q, k, kv[..., dn:], out, lse, dq, dk, dkv[..., dn:], scale, True, 0.0, 0,
                     None)
        dkv[..., :dn].copy_(dk[..., :dn])
        dkr = dk[..., dn:].sum(2, keepdim=True, dtype=torch.float32).to(q.dtype)
        ops.rope_(dkr, cos, sin, None, 1, pos_off, 0, True)
        ops.rope_(dq[..., dn:], cos, sin, None, H, pos_off, 0, True)
        return dq, dkv, dkr, None, None, None, None


def mla_attention(q_raw, kv, kr, dn, scale, theta, pos_off=0):
    """Causal MLA attention: q_raw [B, T, H, dn+dr] (rope columns not yet rotated), kv
    [B, T, H, dn+dv] (the W_ukv up-projection: k_nope | v per head), kr [B, T, 1, dr] (the shared
    rope key, not yet rotated). Returns o [B, T, H, dv]. RoPE is interleaved (apply_rope's
    default) at positions pos_off.. ."""
    dr = q_raw.shape[-1] - dn
    dv = kv.shape[-1] - dn
    # fused on the (192, 128) kernels (V3 widths) and the hd-128 ones (dsv3_style: 64 nope + 64 rope,
    # v 128); SPA_MLA_FUSED=0 (read per call) keeps the op-by-op composition
    if (q_raw.is_cuda and q_raw.dtype == torch.bfloat16 and (dn + dr, dv) in ((192, 128), (128, 128))
            and kv.stride(-1) == 1 and kr.shape[2] == 1 and os.environ.get("SPA_MLA_FUSED", "1") != "0"):
        return _MLAFn.apply(q_raw, kv, kr, int(dn), float(scale), int(pos_off), float(theta))
    from .rope import apply_rope
    B, T, H, _ = q_raw.shape
    qr = apply_rope(q_raw[..., dn:], theta, pos_off)
    krr = apply_rope(kr, theta, pos_off)
    qf = torch.cat([q_raw[..., :dn], qr], dim=-1)
    k = torch.cat([kv[..., :dn], krr.expand(B, T, H, dr)], dim=-1)
    return flash_attention(qf, k, kv[..., dn:], causal=True, scale=scale)


class _SplitLastFn(torch.autograd.Function):
    """x [..., a + b] -> (x[..., :a], x[..., a:]) as contiguous tensors; the backward writes both
    gradients into one buffer (one cat) instead of two zero-filled slice gradients and an add."""

    @staticmethod
    def forward(ctx, x, a):
        ctx.a, ctx.shape = a, x.shape
        return x[..., :a].contiguous(), x[..., a:].contiguous()

    @staticmethod
    def backward(ctx, ga, gb):
        if ga is None:
            ga = torch.zeros(ctx.shape[:-1] + (ctx.a,), device=gb.device, dtype=gb.dtype)
        if gb is None:
            gb = torch.zeros(ctx.shape[:-1] + (ctx.shape[-1] - ctx.a,), device=ga.device, dtype=ga.dtype)
        return torch.cat([ga, gb], dim=-1), None


def split_last(x, a):
    """(x[..., :a], x[..., a:]) as contiguous tensors with a single-buffer backward."""
    return _SplitLastFn.apply(x, int(a))


def attention_packed(qkv, H, Hkv, causal=True, scale=None, head_dim=None, dropout_p=0.0, seed=None):
    """qkv [B, T, H+2Hkv, hd] (or [B, T, (H+2Hkv)*hd] with head_dim) -> out [B, T, H*hd]."""
    hd = head_dim if head_dim is not None else qkv.shape[-1]
    B, T = qkv.shape[0], qkv.shape[1]
    scale = float(scale) if scale is not None else 1.0 / math.sqrt(hd)
    if dropout_p > 0.0 and seed is None:
        seed = torch.randint(0, 2 ** 62, (1,), device=qkv.device, dtype=torch.int64) if qkv.is_cuda else _new_seed()
    if qkv.is_cuda and qkv.dtype == torch.bfloat16 and hd in FLASH_HD:
        return _PackedFn.apply(qkv, H, Hkv, hd, causal, scale, float(dropout_p),
                               seed if isinstance(seed, torch.Tensor) else int(seed or 0))
    x4 = qkv.view(B, T, H + 2 * Hkv, hd)
    q, k, v = x4[:, :, :H], x4[:, :, H:H + Hkv], x4[:, :, H + Hkv:]
    return flash_attention(q, k, v, causal, scale, dropout_p, seed).reshape(B, T, H * hd)


class _PrefixPackedFn(torch.autograd.Function):
    """Causal attention of a later chunk of the same sequences: queries of ``qkv`` (positions
    [Ta, Ta + Tb)) over the keys of ``qkv_a`` (positions [0, Ta)) and its own. Both operands are
    packed [B, T, (H + 2 Hkv) hd] buffers; their K/V columns are gathered into one [B, Ta + Tb,
    2 Hkv hd] buffer (the kernels read K/V rows at one stride), and the backward hands qkv_a the
    gradient of its K/V columns (its q columns get none from here)."""

    @staticmethod
    def forward(ctx, qkv, qkv_a, H, Hkv, hd, scale):
        B, Tb, Ta = qkv.shape[0], qkv.shape[1], qkv_a.shape[1]
        c = H * hd
        kv = torch.cat([qkv_a[..., c:], qkv[..., c:]], dim=1)
        q4 = qkv.view(B, Tb, H + 2 * Hkv, hd)[:, :, :H]
        kv4 = kv.view(B, Ta + Tb, 2 * Hkv, hd)
        out, lse = _ext.ops().attn_fwd(q4, kv4[:, :, :Hkv], kv4[:, :, Hkv:], scale, True, 0.0, 0, None)
        ctx.save_for_backward(qkv, kv, out, lse)
        ctx.H, ctx.Hkv, ctx.hd, ctx.scale, ctx.Ta, ctx.shape_a = H, Hkv, hd, scale, Ta, qkv_a.shape
        return torch.ops.aten._unsafe_view(out, (B, Tb, H * hd))

    @staticmethod
    def backward(ctx, dout):
        qkv, kv, out, lse = ctx.saved_tensors
        H, Hkv, hd, Ta = ctx.H, ctx.Hkv, ctx.hd, ctx.Ta
        B, Tb = qkv.shape[0], qkv.shape[1]
        c = H * hd
        dqkv = torch.empty_like(qkv)
        dkv = torch.empty_like(kv)
        kv4, dkv4 = kv.view(B, Ta + Tb, 2 * Hkv, hd), dkv.view(B, Ta + Tb, 2 * Hkv, hd)
        _ext.ops().attn_bwd(dout.contiguous().view(B, Tb, H, hd), qkv.view(B, Tb, H + 2 * Hkv, hd)[:, :, :H],
                            kv4[:, :, :Hkv], kv4[:, :, Hkv:], out, lse,
                            dqkv.view(B, Tb, H + 2 * Hkv, hd)[:, :, :H], dkv4[:, :, :Hkv], dkv4[:, :, Hkv:],
                            ctx.scale, True, 0.0, 0, None)
        dqkv[..., c:] = dkv[:, Ta:]
        dqkv_a = torch.zeros(ctx.shape_a, device=dqkv.device, dtype=dqkv.dtype)
        dqkv_a[..., c:] = dkv[:, :Ta]
        return dqkv, dqkv_a, None, None, None, None


def attention_packed_prefix(qkv, qkv_a, H, Hkv, head_dim, scale=None):
    """Causal attention of chunk B of a sequence split in two (models/gemma.py _forward_sp_pair):
    qkv / qkv_a [B, Tb / Ta, (H + 2 Hkv) * head_dim] packed buffers of chunks B / A (RoPE applied),
    chunk B's queries attending to chunk A's keys and its own (causal with offset Ta) -> [B, Tb, H*hd]."""
    hd = head_dim
    B, Tb, Ta = qkv.shape[0], qkv.shape[1], qkv_a.shape[1]
    scale = float(scale) if scale is not None else 1.0 / math.sqrt(hd)
    if qkv.is_cuda and qkv.dtype == torch.bfloat16 and hd in FLASH_HD:
        return _PrefixPackedFn.apply(qkv, qkv_a, H, Hkv, hd, scale)
    xa, xb = qkv_a.view(B, Ta, H + 2 * Hkv, hd), qkv.view(B, Tb, H + 2 * Hkv, hd)
    k = torch.cat([xa[:, :, H:H + Hkv], xb[:, :, H:H + Hkv]], 1)
    v = torch.cat([xa[:, :, H + Hkv:], xb[:, :, H + Hkv:]], 1)
    return flash_attention(xb[:, :, :H], k, v, True, scale).reshape(B, Tb, H * hd)


def attention_dropout(q, k, v, causal=True, scale=None, p=0.0, training=True, neg=float("-inf")):
    """Attention with dropout on the probability matrix (GPT-ref gpt/gpt-jax.ipynb:351,
    Gemma-ref gemma/gemma.ipynb:248, DeepSeek-ref deepseekv3/deepseekv3.ipynb:1186): the fused
    HIP kernels on the GPU. ``neg`` (GPT-ref masks with -1e4 instead of -inf) only changes
    scores of fully masked rows, which causal attention never has; the kernels mask with -inf.
    q [B,Tq,H,hd], k/v [B,Tk,Hkv,hd]."""
    if not training or p == 0.0:
        return flash_attention(q, k, v, causal, scale)
    scale = float(scale) if scale is not None else 1.0 / math.sqrt(q.shape[-1])
    if q.is_cuda:
        return flash_attention(q, k, v, causal, scale, dropout_p=p)
    return _materialised(q, k, v, causal, scale, p, _new_seed(), neg)


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


def mla_decode_attention(q_abs, q_rope, cc, cr, scale, kv_len=0, kv_len_t=None, nsplit=0):
    """DeepSeek MLA decode in latent space (csrc/kernels/mla_decode.hip): q_abs [B,T,H,C]
    (q_nope with W_uk absorbed), q_rope [B,T,H,R]; caches cc [B,Smax,C], cr [B,Smax,R] with
    rows [0, kv_len) valid (``kv_len_t``: device int32 [1], graph mode); query token t sits at
    cache row kv_len - T + t. Returns the latent output [B,T,H,C] (W_uv applied by the caller)."""
    if q_abs.is_cuda:
        return _ext.ops().mla_decode(q_abs, q_rope, cc, cr, float(scale), int(kv_len), kv_len_t, int(nsplit))
    B, T, H, C = q_abs.shape
    S = int(kv_len_t.item()) if kv_len_t is not None else int(kv_len)
    s = (torch.einsum("bthc,bsc->bhts", q_abs.float(), cc[:, :S].float())
         + torch.einsum("bthr,bsr->bhts", q_rope.float(), cr[:, :S].float())) * scale
    i = torch.arange(T, device=s.device)[:, None] + (S - T)
    j = torch.arange(S, device=s.device)[None, :]
    s = s.masked_fill(j > i, float("-inf"))
    return torch.einsum("bhts,bsc->bthc", torch.softmax(s, -1), cc[:, :S].float()).to(q_abs.dtype)
