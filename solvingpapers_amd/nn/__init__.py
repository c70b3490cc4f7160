"""nn.Module layer over the HIP ops (SURVEY.md §1.2 layer N).

Modules keep PyTorch-compatible parameter names/shapes so the reference
state-dict layouts load directly, while the math runs on the
hand-written gfx950 kernels (CPU tensors fall back to the reference oracles).
"""
from __future__ import annotations

import math

import torch
import torch.nn as tnn

from ..ops import act, embedding, layer_norm, linear, rms_norm
from ..ops.linear import Linear
from ..ops.misc import conv2d, dropout, local_response_norm, max_pool2d


class LayerNorm(tnn.Module):
    def __init__(self, dim, eps=1e-5, device=None, dtype=None):
        super().__init__()
        self.eps = eps
        self.weight = tnn.Parameter(torch.ones(dim, device=device, dtype=dtype))
        self.bias = tnn.Parameter(torch.zeros(dim, device=device, dtype=dtype))

    def forward(self, x, residual=None):
        return layer_norm(x, self.weight, self.bias, self.eps, residual=residual)


class RMSNorm(tnn.Module):
    def __init__(self, dim, eps=1e-6, device=None, dtype=None):
        super().__init__()
        self.eps = eps
        self.weight = tnn.Parameter(torch.ones(dim, device=device, dtype=dtype))

    def forward(self, x, residual=None):
        return rms_norm(x, self.weight, self.eps, residual=residual)


class Dropout(tnn.Module):
    def __init__(self, p=0.1):
        super().__init__()
        self.p = p

    def forward(self, x):
        return dropout(x, self.p, self.training)


class Embedding(tnn.Module):
    def __init__(self, num_embeddings, embedding_dim, device=None, dtype=None):
        super().__init__()
        self.weight = tnn.Parameter(torch.empty(num_embeddings, embedding_dim, device=device, dtype=dtype))
        tnn.init.normal_(self.weight)

    def forward(self, idx, pos=None, scale=1.0):
        return embedding(self.weight, idx, pos, scale)


class Activation(tnn.Module):
    def __init__(self, kind="relu", alpha=None):
        super().__init__()
        self.kind, self.alpha = kind, alpha

    def forward(self, x):
        return act(x, self.kind, self.alpha)

    def extra_repr(self):
        return self.kind


def ReLU(inplace=False):
    return Activation("relu")


def GELU(approximate="none"):
    return Activation("gelu_tanh" if approximate == "tanh" else "gelu")


def Sigmoid():
    return Activation("sigmoid")


class Flatten(tnn.Module):
    def forward(self, x):
        return x.flatten(1)


class Conv2d(tnn.Module):
    def __init__(self, cin, cout, kernel_size, stride=1, padding=0, bias=True, device=None, dtype=None):
        super().__init__()
        k = kernel_size
        self.stride, self.padding = stride, padding
        self.weight = tnn.Parameter(torch.empty(cout, cin, k, k, device=device, dtype=dtype))
        self.bias = tnn.Parameter(torch.empty(cout, device=device, dtype=dtype)) if bias else None
        tnn.init.kaiming_uniform_(self.weight, a=math.sqrt(5))
        if self.bias is not None:
            bound = 1 / math.sqrt(cin * k * k)
            tnn.init.uniform_(self.bias, -bound, bound)

    def forward(self, x):
        return conv2d(x, self.weight, self.bias, self.stride, self.padding)


class MaxPool2d(tnn.Module):
    def __init__(self, kernel_size, stride):
        super().__init__()
        self.k, self.s = kernel_size, stride

    def forward(self, x):
        return max_pool2d(x, self.k, self.s)


class LocalResponseNorm(tnn.Module):
    def __init__(self, size, alpha=1e-4, beta=0.75, k=1.0):
        super().__init__()
        self.size, self.alpha, self.beta, self.k = size, alpha, beta, k

    def forward(self, x):
        return local_response_norm(x, self.size, self.alpha, self.beta, self.k)


__all__ = ["LayerNorm", "RMSNorm", "Dropout", "Embedding", "Activation", "ReLU", "GELU", "Sigmoid", "Flatten",
           "Conv2d", "MaxPool2d", "LocalResponseNorm", "Linear", "linear"]
