"""Pure-PyTorch fp32 oracles for every HIP op.

These are the numerics reference for the GPU kernel tests and the CPU
execution path (the tiny-GPT CPU plumbing config). They follow the reference
notebooks' math exactly; citations are on each function.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

def _f(t):
    """fp32 compute, or fp64 for fp64 inputs (the CPU numeric-parity tests run whole models in fp64)."""
    return t if t.dtype == torch.float64 else t.float()


ACT_KINDS = {
    "relu": 0, "leaky_relu": 1, "prelu": 2, "elu": 3, "gelu_tanh": 4, "gelu": 5, "gelu_erf": 5,
    "silu": 6, "swish": 6, "sigmoid": 7, "tanh": 8, "identity": 9,
}


def rms_norm(x, w, eps, residual=None):
    """llama3/LLaMA-jax.ipynb:536-538; gemma/gemma.ipynb:139-150 (fp32 compute)."""
    h = x if residual is None else (_f(x) + _f(residual)).to(x.dtype)
    hf = _f(h)
    y = hf * torch.rsqrt(hf.pow(2).mean(-1, keepdim=True) + eps) * _f(w)
    return y.to(x.dtype), h


def layer_norm(x, w, b, eps, residual=None):
    """gpt/gpt-jax.ipynb:414-416 (flax LayerNorm eps 1e-6); ViT.ipynb:205-206."""
    h = x if residual is None else (_f(x) + _f(residual)).to(x.dtype)
    y = F.layer_norm(_f(h), (h.shape[-1],), _f(w), _f(b), eps)
    return y.to(x.dtype), h


def act(x, kind: str, alpha: float = 0.0):
    """activation functions/GELU.ipynb:54-55, ReLU.ipynb:20-54."""
    xf = _f(x)
    if kind == "relu":
        y = F.relu(xf)
    elif kind in ("leaky_relu", "prelu"):
        y = torch.where(xf > 0, xf, alpha * xf)
    elif kind == "elu":
        y = torch.where(xf > 0, xf, alpha * (torch.exp(xf) - 1))
    elif kind == "gelu_tanh":
        y = 0.5 * xf * (1 + torch.tanh(math.sqrt(2 / math.pi) * (xf + 0.044715 * xf ** 3)))
    elif kind in ("gelu", "gelu_erf"):
        y = F.gelu(xf)
    elif kind in ("silu", "swish"):
        y = F.silu(xf)
    elif kind == "sigmoid":
        y = torch.sigmoid(xf)
    elif kind == "tanh":
        y = torch.tanh(xf)
    elif kind == "identity":
        y = xf
    else:
        raise ValueError(kind)
    return y.to(x.dtype)


def glu(gu, kind: str):
    """SwiGLU llama3/LLaMA-jax.ipynb:854-855 (gate=w3 in the ref), GeGLU gemma.ipynb:281-286."""
    g, u = _f(gu).chunk(2, dim=-1)
    return (_f(act(g, kind)) * u).to(gu.dtype)


def rope_tables(T, hd, theta=10000.0, device=None, ref_freqs=False):
    """Angles t*freq_i, i < hd/2. Standard (Meta) freq_i = theta^(-2i/hd);
    ``ref_freqs=True`` reproduces llama3/LLaMA-jax.ipynb:563-567 exactly, whose
    precompute_freqs_cis uses arange(0, dim//2)/dim, i.e. theta^(-i/hd)."""
    expo = torch.arange(0, hd // 2, dtype=torch.float64) / hd if ref_freqs else \
        torch.arange(0, hd, 2, dtype=torch.float64) / hd
    inv = 1.0 / (theta ** expo)
    t = torch.arange(T, dtype=torch.float64)
    ang = torch.outer(t, inv)
    return ang.cos().float().to(device), ang.sin().float().to(device)


def rope(x, cos, sin, pos_off=0, interleaved=True, inverse=False, positions=None):
    """apply_rotary_emb llama3/LLaMA-jax.ipynb:592-601; x [B,T,H,hd]."""
    B, T, H, hd = x.shape
    if positions is None:
        c = cos[pos_off:pos_off + T][None, :, None, :]
        s = sin[pos_off:pos_off + T][None, :, None, :]
    else:
        c = cos[positions.long()][:, :, None, :]
        s = sin[positions.long()][:, :, None, :]
    if inverse:
        s = -s
    xf = _f(x)
    if interleaved:
        x0, x1 = xf[..., 0::2], xf[..., 1::2]
        o0 = x0 * c - x1 * s
        o1 = x0 * s + x1 * c
        out = torch.stack([o0, o1], dim=-1).flatten(-2)
    else:
        x0, x1 = xf[..., : hd // 2], xf[..., hd // 2:]
        out = torch.cat([x0 * c - x1 * s, x0 * s + x1 * c], dim=-1)
    return out.to(x.dtype)


def attention(q, k, v, causal=True, scale=None):
    """Materialised softmax(QK^T*scale + mask) V with GQA head mapping.

    q [B,Tq,H,hd], k/v [B,Tk,Hkv,hd]; causal aligned bottom-right (key j visible
    to query i iff j <= i + Tk - Tq). gpt-jax.ipynb:344-353, LLaMA-jax.ipynb:809-829.
    Returns (out [B,Tq,H,hd], lse [B,H,Tq]).
    """
    B, Tq, H, hd = q.shape
    Tk, Hkv = k.shape[1], k.shape[2]
    scale = scale if scale is not None else 1.0 / math.sqrt(hd)
    rep = H // Hkv
    kf = _f(k).repeat_interleave(rep, dim=2)
    vf = _f(v).repeat_interleave(rep, dim=2)
    s = torch.einsum("bqhd,bkhd->bhqk", _f(q), kf) * scale
    if causal:
        i = torch.arange(Tq, device=q.device)[:, None]
        j = torch.arange(Tk, device=q.device)[None, :]
        s = s.masked_fill(j > i + (Tk - Tq), float("-inf"))
    lse = torch.logsumexp(s, dim=-1)
    p = torch.softmax(s, dim=-1).nan_to_num(0.0)
    o = torch.einsum("bhqk,bkhd->bqhd", p, vf)
    return o.to(q.dtype), lse


def cross_entropy(logits, target, ignore_index=-100, smoothing=0.0):
    """Per-row CE losses (fp32), F.cross_entropy semantics. gpt-jax.ipynb:503."""
    return F.cross_entropy(_f(logits), target, ignore_index=ignore_index, reduction="none",
                           label_smoothing=smoothing)


def embedding(W, idx, pos=None, scale=1.0):
    if bool((idx < 0).any()):       # negative id: a zero row (vocab-parallel foreign tokens)
        keep = (idx >= 0).unsqueeze(-1).to(W.dtype)
        out = W[idx.clamp_min(0)] * keep
        out = out * scale if scale != 1.0 else out
    else:
        out = W[idx] * scale if scale != 1.0 else W[idx]
    if pos is not None:
        T = idx.shape[-1]
        out = out + pos.reshape(-1, W.shape[1])[:T]
    return out


def adamw_(p, master, g, m, v, lr, b1, b2, eps, wd, step, coef=None, adam_l2=False):
    """torch.optim.AdamW / Adam math on flat fp32 state (in place). A NaN ``coef``
    (non-finite global grad norm) skips the update, as the HIP kernel does."""
    if coef is not None and bool(torch.isnan(coef).any()):
        return
    src = master if master is not None else p
    pf = src.float()
    gf = g.float() * (coef.float() if coef is not None else 1.0)
    if adam_l2:
        gf = gf + wd * pf
    mf = m.float().mul_(b1).add_(gf, alpha=1 - b1)      # bf16 moments: update in fp32, store rounded
    vf = v.float().mul_(b2).addcmul_(gf, gf, value=1 - b2)
    m.copy_(mf)
    v.copy_(vf)
    bc1 = 1 - b1 ** step
    bc2 = 1 - b2 ** step
    denom = vf.sqrt() / math.sqrt(bc2) + eps
    if not adam_l2:
        pf = pf * (1 - lr * wd)
    pf = pf - (lr / bc1) * mf / denom
    if master is not None:
        master.copy_(pf)
    p.copy_(pf.to(p.dtype))


def sgd_(p, master, g, buf, lr, momentum, wd, coef=None):
    if coef is not None and bool(torch.isnan(coef).any()):
        return
    src = master if master is not None else p
    pf = src.float()
    gf = g.float() * (coef.float() if coef is not None else 1.0) + wd * pf
    if buf is not None:
        buf.mul_(momentum).add_(gf)
        gf = buf
    pf = pf - lr * gf
    if master is not None:
        master.copy_(pf)
    p.copy_(pf.to(p.dtype))
