"""Layout helpers (HIP: csrc/kernels/layout.hip)."""
from __future__ import annotations

import os

import torch

from . import _ext

# dW = dY^T X: hipBLASLt's direct TN form is slow on gfx950 for wide operands, so for those one
# operand is first transposed to token-contiguous rows (layout.hip). Measured with
# tools/bench_wgrad_layouts.py (profiles/r2_wgrad_layouts_vit_llama.txt): at LLaMA3-8B shapes
# (T 8192) transposing only the narrower operand wins (w13 1.450 ms vs 1.517 both-transposed /
# 1.638 direct, w2 0.807 vs 0.811 / 0.899); at ViT-B/16 shapes
# (T 50432, 768-3072 wide) the transposes cost more than they save (fc1 0.392 direct vs 0.514
# both). SPA_WGRAD_NT=0 forces the direct product everywhere.
WGRAD_NT = os.environ.get("SPA_WGRAD_NT", "1") != "0"
WGRAD_NT_MIN_TOKENS = 2048
WGRAD_NT_MIN_WIDTH = 2048
# the narrow-operand / many-token products go to wgrad8 (csrc/kernels/gemm8.hip): token-major
# operands read as they are, split over tokens to fill the chip, fp32 partials; SPA_WGRAD8=0
# keeps them on hipBLASLt's direct form
WGRAD8 = os.environ.get("SPA_WGRAD8", "1") != "0"
WGRAD8_MIN_TOKENS = 4096


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


def wgrad_operand(dy2: torch.Tensor, x2: torch.Tensor):
    """x2 transposed to token-contiguous rows when wgrad(dy2, x2) would transpose it, else None
    (lets a caller issuing several dW products against one x2 transpose it once)."""
    if wgrad_nt_ok(dy2, x2) and min(dy2.shape[1], x2.shape[1]) >= WGRAD_NT_MIN_WIDTH and x2.shape[1] <= dy2.shape[1]:
        return transpose2d(x2)
    return None


def wgrad8_ok(dy2: torch.Tensor, x2: torch.Tensor, out=None) -> bool:
    return (WGRAD8 and dy2.is_cuda and dy2.dtype == torch.bfloat16 and x2.dtype == torch.bfloat16
            and dy2.dim() == 2 and x2.dim() == 2 and dy2.shape[0] >= WGRAD8_MIN_TOKENS
            and min(dy2.shape[1], x2.shape[1]) < WGRAD_NT_MIN_WIDTH
            and dy2.shape[1] % 8 == 0 and x2.shape[1] % 8 == 0 and dy2.stride(1) == 1 and x2.stride(1) == 1
            and dy2.stride(0) % 8 == 0 and x2.stride(0) % 8 == 0
            and dy2.data_ptr() % 16 == 0 and x2.data_ptr() % 16 == 0
            and (out is None or (out.is_contiguous() and out.dtype in (torch.bfloat16, torch.float32))))


def wgrad(dy2: torch.Tensor, x2: torch.Tensor, out=None, accumulate=False, x2t=None, dyt=None):
    """dW = dy2^T @ x2 ([N, K] from [T, N] and [T, K]) into a fresh tensor, or written into /
    added to ``out`` (any float dtype, e.g. an fp32 main_grad). Many tokens with a narrow
    operand: wgrad8; else the narrower operand is transposed to token-contiguous rows first
    when both are wide and T is large (x2t: x2 already transposed). ``dyt``: dy2 already
    transposed by its producer (linear.py linear_glu) -> the both-token-contiguous form."""
    if dyt is None and wgrad8_ok(dy2, x2, out):
        return _ext.ops().wgrad8(dy2, x2, out, accumulate, 0)
    f32out = (out is not None and out.dtype == torch.float32 and dy2.dtype == torch.bfloat16 and dy2.is_cuda
              and out.is_contiguous() and _MM_F32[0] is not False)
    if out is not None and out.dtype != dy2.dtype and not f32out:
        g = wgrad(dy2, x2, x2t=x2t, dyt=dyt)
        out.add_(g) if accumulate else out.copy_(g)
        return out
    N, K = dy2.shape[1], x2.shape[1]
    if dyt is not None:
        a, b = dyt, (x2t if x2t is not None else transpose2d(x2)).t()
    elif wgrad_nt_ok(dy2, x2) and min(N, K) >= WGRAD_NT_MIN_WIDTH:
        if K <= N:
            a, b = dy2.t(), (x2t if x2t is not None else transpose2d(x2)).t()
        else:
            a, b = transpose2d(dy2), x2
    else:
        a, b = dy2.t(), x2
    if out is None:
        return torch.mm(a, b)
    if f32out:
        # fp32 main gradient: hipBLASLt accumulates in fp32 and writes / adds fp32 directly
        # (aten::mm.dtype / addmm.dtype), no bf16 temporary and no separate add pass
        try:
            if accumulate:
                torch.addmm(out, a, b, out_dtype=torch.float32, out=out)
            else:
                torch.mm(a, b, out_dtype=torch.float32, out=out)
            _MM_F32[0] = True
            return out
        except (RuntimeError, TypeError):
            _MM_F32[0] = False
            g = torch.mm(a, b)
            out.add_(g) if accumulate else out.copy_(g)
            return out
    if accumulate:
        out.addmm_(a, b)
    else:
        torch.mm(a, b, out=out)
    return out


_MM_F32 = [None]     # aten::mm.dtype_out / addmm.dtype_out usable (probed on first use)


def bias_grad(dy2: torch.Tensor) -> torch.Tensor:
    """fp32 column sums of [T, N] (the bias gradient): csrc/kernels/norm.hip rowsum_bf16 for bf16
    on the GPU (two-level deterministic sum filling the chip), else torch."""
    if (dy2.is_cuda and dy2.dtype == torch.bfloat16 and dy2.dim() == 2 and dy2.stride(1) == 1
            and dy2.shape[1] % 8 == 0 and dy2.stride(0) % 8 == 0 and dy2.data_ptr() % 16 == 0):
        return _ext.ops().rowsum_bf16(dy2)
    return dy2.sum(0, dtype=torch.float64 if dy2.dtype == torch.float64 else torch.float32)
