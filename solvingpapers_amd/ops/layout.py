"""Layout helpers (HIP: csrc/kernels/layout.hip)."""
from __future__ import annotations

import os

import torch

from . import _ext

# dW = dY^T X through K-contiguous transposed operands + the NT GEMM (see layout.hip);
# SPA_WGRAD_NT=0 restores the direct TN product
WGRAD_NT = os.environ.get("SPA_WGRAD_NT", "1") != "0"
WGRAD_NT_MIN_TOKENS = 2048


def transpose2d(x: torch.Tensor) -> torch.Tensor:
    """[R, C] -> contiguous [C, R] (or batched [Bt, R, C] -> [Bt, C, R])."""
    if x.is_cuda and x.dtype in (torch.bfloat16, torch.float32):
        return _ext.ops().transpose2d(x)
    return x.transpose(-1, -2).contiguous()


def wgrad_nt_ok(dy2: torch.Tensor, x2: torch.Tensor) -> bool:
    # the transpose kernel moves 16-byte units along both axes: token count, N and K all % 8
    # (MTP heads feed T - k tokens, e.g. 8190)
    return (WGRAD_NT and dy2.is_cuda and dy2.dtype == torch.bfloat16 and x2.dtype == torch.bfloat16
            and dy2.shape[0] >= WGRAD_NT_MIN_TOKENS and dy2.shape[0] % 8 == 0
            and dy2.shape[1] % 8 == 0 and x2.shape[1] % 8 == 0
            and dy2.stride(1) == 1 and x2.stride(1) == 1 and dy2.stride(0) % 8 == 0 and x2.stride(0) % 8 == 0)


def wgrad(dy2: torch.Tensor, x2: torch.Tensor, out=None, accumulate=False):
    """dW = dy2^T @ x2 ([N, K] from [T, N] and [T, K]); NT formulation for large T."""
    if wgrad_nt_ok(dy2, x2):
        a, b = transpose2d(dy2), transpose2d(x2).t()
    else:
        a, b = dy2.t(), x2
    if out is None:
        return torch.mm(a, b)
    if accumulate:
        out.addmm_(a, b)
    else:
        torch.mm(a, b, out=out)
    return out
