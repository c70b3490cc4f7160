"""Activations and gated linear units (HIP: csrc/kernels/activation.hip).

Kinds: relu, leaky_relu(alpha=0.01), prelu(alpha), elu(alpha), gelu_tanh,
gelu (exact erf), silu/swish, sigmoid, tanh. GLU: ``glu(gu, kind)`` on a fused
[..., 2F] = [gate | up] GEMM output -> act(gate) * up.
"""
from __future__ import annotations

import torch

from . import _ext, reference
from .reference import ACT_KINDS


def _hip_ok(x):
    return x.is_cuda and x.dtype in (torch.bfloat16, torch.float32)


class _ActFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, kind, alpha):
        ctx.save_for_backward(x)
        ctx.kind, ctx.alpha = kind, alpha
        return _ext.ops().act_fwd(x, kind, alpha)

    @staticmethod
    def backward(ctx, g):
        (x,) = ctx.saved_tensors
        return _ext.ops().act_bwd(g, x, ctx.kind, ctx.alpha), None, None


class _GluFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, gu, kind):
        ctx.save_for_backward(gu)
        ctx.kind = kind
        return _ext.ops().glu_fwd(gu, kind)

    @staticmethod
    def backward(ctx, g):
        (gu,) = ctx.saved_tensors
        return _ext.ops().glu_bwd(g, gu, ctx.kind), None


def act(x, kind="relu", alpha=None):
    if alpha is None:
        alpha = 0.01 if kind == "leaky_relu" else (1.0 if kind == "elu" else 0.0)
    if x.is_cuda:
        if not _hip_ok(x):
            raise RuntimeError(f"activation kernel: unsupported dtype {x.dtype}")
        return _ActFn.apply(x, ACT_KINDS[kind], float(alpha))
    return reference.act(x, kind, alpha)


def glu(gu, kind="silu"):
    if gu.is_cuda:
        if not _hip_ok(gu) or gu.shape[-1] % 16:
            raise RuntimeError(f"glu kernel: unsupported input {gu.dtype} {tuple(gu.shape)}")
        return _GluFn.apply(gu, ACT_KINDS[kind])
    return reference.glu(gu, kind)


def relu(x): return act(x, "relu")
def leaky_relu(x, alpha=0.01): return act(x, "leaky_relu", alpha)
def prelu(x, alpha=0.25): return act(x, "prelu", alpha)
def elu(x, alpha=1.0): return act(x, "elu", alpha)
def gelu(x, approximate="none"): return act(x, "gelu_tanh" if approximate == "tanh" else "gelu")
def silu(x): return act(x, "silu")
def sigmoid(x): return act(x, "sigmoid")
def swiglu(gu): return glu(gu, "silu")
def geglu(gu, approximate="none"): return glu(gu, "gelu_tanh" if approximate == "tanh" else "gelu")
