"""Autograd wrappers for csrc/kernels/misc.hip (dropout, KD/VAE/MSE losses, LRN,
max-pool, conv-as-GEMM, Luong attention). CPU tensors use PyTorch reference math."""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

from . import _ext
from .linear import linear

_HIP_DT = (torch.bfloat16, torch.float32)


def _hip(x):
    return x.is_cuda and x.dtype in _HIP_DT


def _seed():
    return int(torch.randint(0, 2 ** 62, (1,)).item())


# ------------------------------------------------------------------------------- dropout
def _device_seed(device):
    """Seed drawn by torch's (graph-capture-safe) device generator: inside a captured HIP
    graph every replay gets a fresh seed, so dropout masks differ step to step."""
    return torch.randint(0, 2 ** 62, (1,), device=device, dtype=torch.int64)


def _fmt(x):
    """Storage order the HIP elementwise kernels walk: channels-last conv activations keep it."""
    if x.dim() == 4 and not x.is_contiguous() and x.is_contiguous(memory_format=torch.channels_last):
        return torch.channels_last
    return torch.contiguous_format


class _DropoutFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, p, seed_t):
        ctx.p, ctx.seed_t, ctx.fmt = p, seed_t, _fmt(x)
        return _ext.ops().dropout_apply(x.contiguous(memory_format=ctx.fmt), p, 0, seed_t)

    @staticmethod
    def backward(ctx, g):
        # same mask (regenerated from the seed over the same storage order), same 1/(1-p) scale
        return _ext.ops().dropout_apply(g.contiguous(memory_format=ctx.fmt), ctx.p, 0, ctx.seed_t), None, None


def dropout(x, p=0.1, training=True):
    if not training or p == 0.0:
        return x
    if _hip(x):
        return _DropoutFn.apply(x, float(p), _device_seed(x.device))
    return F.dropout(x, p, training)


# ------------------------------------------------------------------------------- KD loss
class _KDFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, s, t, y, T, alpha):
        hard, soft, gs = _ext.ops().kd_loss_fwd(s, t.detach(), y, T, alpha, True)
        ctx.gs = gs
        B = s.shape[0]
        h = hard.mean()
        so = soft.sum() / B * T * T
        return alpha * h + (1 - alpha) * so, h, so

    @staticmethod
    def backward(ctx, g, gh, gso):
        # gradients w.r.t. the returned hard/soft pieces are not propagated (they are
        # reported for logging, as in the reference's (total, hard, soft) tuple)
        return ctx.gs * g.to(ctx.gs.dtype), None, None, None, None


def distillation_loss(student_logits, teacher_logits, target, temperature, alpha):
    """knowledge distillation/kd.py:48-68 -> (total, hard, soft)."""
    if _hip(student_logits):
        return _KDFn.apply(student_logits, teacher_logits, target, float(temperature), float(alpha))
    slp = F.log_softmax(student_logits / temperature, dim=1)
    tp = F.softmax(teacher_logits / temperature, dim=1)
    hard = F.cross_entropy(student_logits, target)
    soft = F.kl_div(slp, tp, reduction="batchmean") * temperature * temperature
    return alpha * hard + (1.0 - alpha) * soft, hard, soft


# ------------------------------------------------------------------------------- VAE
class _ReparamFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, mu, logvar, seed):
        ctx.save_for_backward(mu, logvar)
        ctx.seed = seed
        return _ext.ops().vae_reparam(mu, logvar, None, seed)

    @staticmethod
    def backward(ctx, dz):
        mu, logvar = ctx.saved_tensors
        dlv = _ext.ops().vae_reparam(mu, logvar, dz.contiguous(), ctx.seed)
        return dz, dlv, None


def reparameterize(mu, logvar):
    """z = mu + eps * exp(0.5 logvar) (variational autoencoder.ipynb:94-97)."""
    if _hip(mu):
        return _ReparamFn.apply(mu, logvar, _seed())
    std = torch.exp(0.5 * logvar)
    return mu + torch.randn_like(std) * std


class _VaeLossFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, r, x, mu, logvar):
        bce, kl, dr, dmu, dlv = _ext.ops().vae_loss_fwd(r, x, mu, logvar)
        ctx.g = (dr, dmu, dlv)
        return (bce + kl).reshape(())

    @staticmethod
    def backward(ctx, g):
        dr, dmu, dlv = ctx.g
        gg = g.to(dr.dtype)
        return dr * gg, None, dmu * gg, dlv * gg


def vae_loss(x_reconstruct, x, mu, logvar):
    """BCE(sum) + KL (variational autoencoder.ipynb:117-120)."""
    if _hip(x_reconstruct):
        return _VaeLossFn.apply(x_reconstruct, x, mu, logvar)
    recon = F.binary_cross_entropy(x_reconstruct, x, reduction="sum")
    kl = -0.5 * torch.sum(1 + logvar - mu.pow(2) - logvar.exp())
    return recon + kl


# ------------------------------------------------------------------------------- MSE
class _MseFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, b):
        ss, ga = _ext.ops().mse_fwd(a, b, True)
        ctx.ga = ga
        return (ss / max(a.numel(), 1)).reshape(())

    @staticmethod
    def backward(ctx, g):
        return ctx.ga * g.to(ctx.ga.dtype), None


def mse_loss(a, b):
    if _hip(a):
        return _MseFn.apply(a, b)
    return F.mse_loss(a, b)


# ------------------------------------------------------------------------------- LRN / maxpool
class _LrnFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, size, alpha, beta, k):
        y, sc = _ext.ops().lrn_fwd(x, size, alpha, beta, k)
        ctx.save_for_backward(x, sc)
        ctx.args = (size, alpha, beta)
        return y

    @staticmethod
    def backward(ctx, g):
        x, sc = ctx.saved_tensors
        size, alpha, beta = ctx.args
        return _ext.ops().lrn_bwd(g, x, sc, size, alpha, beta), None, None, None, None


def local_response_norm(x, size=5, alpha=1e-4, beta=0.75, k=1.0):
    if _hip(x):
        return _LrnFn.apply(x, int(size), float(alpha), float(beta), float(k))
    return F.local_response_norm(x, size, alpha, beta, k)


class _MaxPoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, ks, st):
        y, arg = _ext.ops().maxpool2d_fwd(x, ks, st)
        ctx.save_for_backward(arg)
        ctx.args = (x.shape[2], x.shape[3], ks, st)
        return y

    @staticmethod
    def backward(ctx, g):
        (arg,) = ctx.saved_tensors
        H, W, ks, st = ctx.args
        return _ext.ops().maxpool2d_bwd(g, arg, H, W, ks, st), None, None


def max_pool2d(x, kernel_size=3, stride=2):
    if _hip(x):
        return _MaxPoolFn.apply(x, int(kernel_size), int(stride))
    return F.max_pool2d(x, kernel_size, stride)


# ------------------------------------------------------------------------------- conv2d / patch embed
class _Im2ColFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, kh, kw, sh, sw, ph, pw):
        ctx.args = (x.shape, kh, kw, sh, sw, ph, pw)
        return _ext.ops().im2col(x, kh, kw, sh, sw, ph, pw)

    @staticmethod
    def backward(ctx, g):
        (N, C, H, W), kh, kw, sh, sw, ph, pw = ctx.args
        return _ext.ops().col2im(g, N, C, H, W, kh, kw, sh, sw, ph, pw), None, None, None, None, None, None


def _conv2d_fp32(x, weight, bias, sh, sw, ph, pw):
    """fp32 convs (reference-parity runs) stay exact: HIP im2col + fp32 GEMM. bf16 -- every training
    and benchmark config -- runs the implicit-GEMM MFMA kernels (ops/conv.py)."""
    N, C, H, W = x.shape
    OC, _, KH, KW = weight.shape
    OH, OW = (H + 2 * ph - KH) // sh + 1, (W + 2 * pw - KW) // sw + 1
    cols = _Im2ColFn.apply(x.contiguous(), KH, KW, sh, sw, ph, pw)   # [N*OH*OW, C*KH*KW]
    y = linear(cols, weight.reshape(OC, -1), bias)                  # [N*OH*OW, OC]
    return y.view(N, OH, OW, OC).permute(0, 3, 1, 2)                 # channels-last view


def conv2d(x, weight, bias=None, stride=1, padding=0):
    """2-D convolution, K20 (alexnet/alexnet.py:11-25). bf16 on the GPU: implicit-GEMM MFMA
    kernels, output channels-last (logically NCHW). CPU: torch."""
    sh, sw = (stride, stride) if isinstance(stride, int) else stride
    ph, pw = (padding, padding) if isinstance(padding, int) else padding
    if not _hip(x):
        return F.conv2d(x, weight, bias, (sh, sw), (ph, pw))
    if x.dtype == torch.bfloat16 and weight.dtype == torch.bfloat16:
        from .conv import conv2d_igemm
        return conv2d_igemm(x, weight, bias, (sh, sw), (ph, pw))
    return _conv2d_fp32(x, weight, bias, sh, sw, ph, pw)


def patch_embed(x, weight, bias, patch):
    """Non-overlapping patchify (kernel == stride) + projection -> [N, P, D] tokens
    (vision transformer/ViT.ipynb:182-192: Conv2d(k=s=patch) -> flatten(2).transpose(1,2)).
    bf16: the implicit-GEMM kernel gathers patches straight from the NCHW image (no column
    buffer); its NHWC output IS the [N, P, D] token matrix."""
    if not _hip(x):
        return F.conv2d(x, weight, bias, patch).flatten(2).transpose(1, 2)
    N, C, H, W = x.shape
    OC = weight.shape[0]
    if x.dtype == torch.bfloat16 and weight.dtype == torch.bfloat16:
        from .conv import conv2d_igemm
        y = conv2d_igemm(x, weight, bias, (patch, patch), (0, 0))     # [N, OC, OH, OW] channels-last
        return y.permute(0, 2, 3, 1).reshape(N, -1, OC)
    cols = _Im2ColFn.apply(x.contiguous(), patch, patch, patch, patch, 0, 0)
    y = linear(cols, weight.reshape(OC, -1), bias)
    return y.view(N, (H // patch) * (W // patch), OC)


# ------------------------------------------------------------------------------- Luong attention
class _LuongFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, st, hs):
        ctx_v, w = _ext.ops().luong_fwd(st, hs)
        ctx.save_for_backward(st, hs, w)
        return ctx_v, w

    @staticmethod
    def backward(ctx, dctx, dw):
        st, hs, w = ctx.saved_tensors
        dst, dhs = _ext.ops().luong_bwd(dctx, st, hs, w)
        return dst, dhs


def luong_attention(st, hs):
    """attention/luong.ipynb:22-36: returns (context [B,H], weights [B,S,1])."""
    if st.dim() == 3:
        st = st.squeeze(1)
    if _hip(hs):
        c, w = _LuongFn.apply(st, hs)
        return c, w.to(hs.dtype).unsqueeze(-1)
    dot = torch.sum(st.unsqueeze(1).expand(-1, hs.shape[1], -1) * hs, dim=-1)
    w = torch.softmax(dot, dim=1).unsqueeze(-1)
    return torch.sum(w * hs, dim=1), w
