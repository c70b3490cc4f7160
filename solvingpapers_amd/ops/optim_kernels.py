"""Fused optimizer steps on flat buffers (HIP: csrc/kernels/optim.hip)."""
from __future__ import annotations

import torch

from . import _ext, reference


def adamw_(p, master, g, m, v, lr, b1, b2, eps, wd, step, coef=None, adam_l2=False, hyper=None):
    """``hyper`` (device fp32 [lr, step]) overrides lr/step inside the kernel (HIP-graph replay)."""
    if p.is_cuda:
        _ext.ops().adamw_(p, master, g, m, v, float(lr), float(b1), float(b2), float(eps), float(wd), int(step),
                          coef, bool(adam_l2), hyper)
    else:
        reference.adamw_(p, master, g, m, v, lr, b1, b2, eps, wd, step, coef, adam_l2)


def sgd_(p, master, g, buf, lr, momentum=0.0, wd=0.0, coef=None, hyper=None):
    if p.is_cuda:
        _ext.ops().sgd_(p, master, g, buf, float(lr), float(momentum), float(wd), coef, hyper)
    else:
        reference.sgd_(p, master, g, buf, lr, momentum, wd, coef)


def sqsum(g):
    if g.is_cuda:
        return _ext.ops().sqsum(g)
    return g.float().pow(2).sum().reshape(1)
