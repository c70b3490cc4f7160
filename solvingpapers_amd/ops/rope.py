"""Rotary embeddings applied in place on packed q/k heads (HIP: csrc/kernels/rope.hip).

``rope_packed_(qkv, nrot, cos, sin)`` rotates heads [0, nrot) of a
[B, T, NH, hd] buffer in place; its autograd backward applies the inverse
rotation in place on the incoming gradient (no extra buffers).
Reference: llama3/LLaMA-jax.ipynb:563-601 (interleaved pairs, theta 10000).
"""
from __future__ import annotations

import torch

from . import _ext, reference


def _mode(interleaved):
    """interleaved=True -> 0, False (rotate_half) -> 1, "gemma_ref" -> 2."""
    if interleaved == "gemma_ref":
        return 2
    return 0 if interleaved else 1


class RopeCache:
    """Per-(device, hd, theta) cos/sin tables [Tmax, hd/2] fp32, grown on demand."""

    _tables: dict = {}

    @classmethod
    def get(cls, T, hd, theta, device, ref_freqs=False):
        key = (str(device), hd, float(theta), bool(ref_freqs))
        tab = cls._tables.get(key)
        if tab is None or tab[0].shape[0] < T:
            n = max(T, 1 << max(0, (T - 1).bit_length()))
            cos, sin = reference.rope_tables(n, hd, theta, device=device, ref_freqs=ref_freqs)
            tab = (cos.contiguous(), sin.contiguous())
            cls._tables[key] = tab
        return tab


class _RopeFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, nrot, cos, sin, pos_off, interleaved, grad_inplace, hd):
        # x may be [B, T, NH*hd] (packed projection output) or [B, T, NH, hd]
        x4 = x.view(x.shape[0], x.shape[1], -1, hd)
        _ext.ops().rope_(x4, cos, sin, None, nrot, pos_off, _mode(interleaved), False)
        ctx.mark_dirty(x)
        ctx.args = (nrot, cos, sin, pos_off, interleaved, grad_inplace, hd)
        return x

    @staticmethod
    def backward(ctx, g):
        nrot, cos, sin, pos_off, interleaved, grad_inplace, hd = ctx.args
        # grad_inplace: the caller guarantees the incoming gradient buffer is private
        # to this edge (rope_packed_ feeding attention_packed, whose backward returns a
        # fresh dqkv), so the inverse rotation runs in place; otherwise copy first.
        if not (grad_inplace and g.is_contiguous()):
            g = g.contiguous().clone()
        _ext.ops().rope_(g.view(g.shape[0], g.shape[1], -1, hd), cos, sin, None, nrot, pos_off, _mode(interleaved), True)
        return g, None, None, None, None, None, None, None


def rope_packed_(x, nrot, theta=10000.0, pos_off=0, interleaved=True, head_dim=None, ref_freqs=False):
    """In-place rotation of heads [0, nrot) of x ([B, T, NH, hd], or [B, T, NH*hd]
    with ``head_dim``); returns x.

    Only for a buffer consumed by :func:`attention_packed` (its gradient is
    rotated back in place)."""
    hd = head_dim if head_dim is not None else x.shape[-1]
    B, T = x.shape[0], x.shape[1]
    cos, sin = RopeCache.get(pos_off + T, hd, theta, x.device, ref_freqs)
    if x.is_cuda:
        return _RopeFn.apply(x, nrot, cos, sin, pos_off, interleaved, True, hd)
    x4 = x.view(B, T, -1, hd)
    rot = reference.rope(x4[:, :, :nrot], cos, sin, pos_off, interleaved)
    return torch.cat([rot, x4[:, :, nrot:]], dim=2).view(x.shape)


def apply_rope(x, theta=10000.0, pos_off=0, interleaved=True, positions=None, ref_freqs=False, max_len=None):
    """Out-of-place rotation of every head of x [B, T, H, hd]. ``positions`` (int [B, T] on
    the device) with ``max_len`` (table size) is graph-capture safe: no host read."""
    B, T, H, hd = x.shape
    if positions is not None:
        n = max_len if max_len is not None else int(positions.max()) + 1
    else:
        n = pos_off + T
    cos, sin = RopeCache.get(n, hd, theta, x.device, ref_freqs)
    if x.is_cuda and positions is None:
        return _RopeFn.apply(x.clone(), H, cos, sin, pos_off, interleaved, False, hd)
    if x.is_cuda:
        y = x.clone()
        _ext.ops().rope_(y, cos, sin, positions.int().contiguous(), H, 0, _mode(interleaved), False)
        return y
    return reference.rope(x, cos, sin, pos_off, interleaved, positions=positions)


def gemma_ref_tables(T, D, device):
    """gemma/gemma.ipynb:182-200 quirk: angle depends on position only,
    theta_p = 10000^(-2(p-1)/D), angle = p*theta_p; broadcast to [T, D/2]."""
    key = ("gemma_ref", str(device), T, D)
    tab = RopeCache._tables.get(key)
    if tab is None:
        p = torch.arange(T, dtype=torch.float64)
        ang = p * (10000.0 ** (-2.0 * (p - 1) / D))
        cos = ang.cos().float()[:, None].expand(T, D // 2).contiguous().to(device)
        sin = ang.sin().float()[:, None].expand(T, D // 2).contiguous().to(device)
        tab = (cos, sin)
        RopeCache._tables[key] = tab
    return tab


def gemma_ref_rotate(x):
    """Apply the reference's per-position (D x D) 'rotary' matrix (2x2 blocks
    [[cos, cos], [-sin, sin]]) to every head of x [B, T, H, D] without
    materialising the (T, D, D) matrix: y_e = c(x_e + x_o), y_o = s(x_o - x_e)."""
    B, T, H, D = x.shape
    cos, sin = gemma_ref_tables(T, D, x.device)
    if x.is_cuda:
        return _RopeFn.apply(x.contiguous().clone(), H, cos, sin, 0, "gemma_ref", False, D)
    xe, xo = x[..., 0::2].float(), x[..., 1::2].float()
    c, s = cos[None, :, None, :], sin[None, :, None, :]
    return torch.stack([c * (xe + xo), s * (xo - xe)], -1).flatten(-2).to(x.dtype)
