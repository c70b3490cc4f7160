"""Mixture-of-Experts ops: router, token permutation, grouped expert GEMMs, combine.

Replaces the reference's Python expert loop (deepseekv3/deepseekv3.ipynb:1059-1079:
per-expert boolean gather + ``mask.any()`` host sync + ``masked_scatter_``) with a
fixed sequence of device kernels whose launch count does not depend on E and which
never synchronise with the host:

    route   -> top-k ids + renormalised softmax weights          (csrc/kernels/moe.hip)
    permute -> stable counting sort of the N*k assignments by expert, device offsets
    gather  -> expert-ordered copy of the token rows
    grouped_linear (x2, + GLU)  -> one MFMA grouped GEMM per projection for all experts
    combine -> weighted gather-sum back to token order (deterministic, no atomics)

Each op has a pure-PyTorch path for CPU tensors with identical semantics (used by
the CPU parity tests and the gloo EP tests).
"""
from __future__ import annotations

from dataclasses import dataclass

import os

import torch

from ..utils.grad import commit
from ._ext import ops


def _gpu(t):
    return t.is_cuda


# --------------------------------------------------------------------------- routing
class _RouteFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, bias, k, bias_in_w):
        logits = logits.float()
        if _gpu(logits):
            idx, w = ops().moe_route(logits, bias, k, bias_in_w)
        else:
            scores = logits + bias if bias is not None else logits
            vals, idx = torch.topk(scores, k, dim=-1)
            sel = vals if bias_in_w else logits.gather(-1, idx)
            w = torch.softmax(sel, dim=-1)
            idx = idx.int()
        ctx.save_for_backward(idx, w)
        ctx.E = logits.shape[-1]
        ctx.mark_non_differentiable(idx)
        return idx, w

    @staticmethod
    def backward(ctx, _didx, dw):
        idx, w = ctx.saved_tensors
        if dw is None:
            return None, None, None, None
        dw = dw.float()
        ds = w * (dw - (w * dw).sum(-1, keepdim=True))
        dl = torch.zeros(w.shape[0], ctx.E, device=w.device, dtype=torch.float32)
        dl.scatter_add_(1, idx.long(), ds)
        return dl, None, None, None


class _RouterLogitsFn(torch.autograd.Function):
    """logits = x2 @ gate^T as one bf16 GEMM with fp32 accumulation AND fp32 output (hipBLASLt
    ``mm(out_dtype=float32)``): the router keeps fp32 logits without the fp32 copies of x2
    ([N, D]) and of the gate that an fp32 GEMM needs, and the backward runs two bf16 GEMMs on
    the bf16-rounded fp32 dlogits."""

    @staticmethod
    def forward(ctx, x2, gate):
        ctx.save_for_backward(x2, gate)
        return torch.mm(x2, gate.t(), out_dtype=torch.float32)

    @staticmethod
    def backward(ctx, dl):
        from ..utils.grad import commit_tensor
        x2, gate = ctx.saved_tensors
        dlb = dl.to(x2.dtype)
        dx = torch.mm(dlb, gate) if ctx.needs_input_grad[0] else None
        dg = commit_tensor(gate, torch.mm(dlb.t(), x2)) if ctx.needs_input_grad[1] else None
        return dx, dg


def router_logits(x2, gate):
    """fp32 router logits [N, E] of x2 [N, D] and gate [E, D]."""
    if x2.is_cuda and x2.dtype == torch.bfloat16 and gate.dtype == torch.bfloat16:
        return _RouterLogitsFn.apply(x2, gate)
    return torch.mm(x2.float(), gate.float().t())


def route(logits, k, bias=None, bias_in_weights=True):
    """Top-k expert choice + softmax over the selected logits.

    ``logits`` [N, E]. ``bias`` (aux-free balancing, [E]) shifts the *selection*; with
    ``bias_in_weights`` the gating weights are softmax(logits + bias) over the top-k
    (reference semantics, deepseekv3.ipynb:1041-1051), else softmax of the raw logits
    (DeepSeek-V3 paper: the bias only steers selection). Returns (idx int32 [N,k], w fp32 [N,k]).
    """
    if bias is not None:
        bias = bias.float()
    return _RouteFn.apply(logits, bias, int(k), bool(bias_in_weights))


# --------------------------------------------------------------------------- permutation
@dataclass
class MoEPlan:
    """Expert-sorted layout of N*k token->expert assignments (a = n*k + j)."""
    perm: torch.Tensor      # [A] int32: sorted position -> assignment
    inv: torch.Tensor       # [A] int32: assignment -> sorted position
    offsets: torch.Tensor   # [E+1] int32 (device): expert e owns rows [off[e], off[e+1])
    counts: torch.Tensor    # [E] int32
    k: int
    n_tokens: int

    @property
    def n_experts(self):
        return self.counts.numel()


def permute(idx, n_experts) -> MoEPlan:
    idx = idx.contiguous().int()
    N, k = idx.shape
    if _gpu(idx):
        perm, inv, offsets, counts = ops().moe_permute(idx, n_experts)
    else:
        flat = idx.reshape(-1).long()
        perm = torch.sort(flat, stable=True).indices
        inv = torch.empty_like(perm)
        inv[perm] = torch.arange(perm.numel())
        counts = torch.bincount(flat, minlength=n_experts)
        offsets = torch.cat([counts.new_zeros(1), counts.cumsum(0)])
        perm, inv, offsets, counts = perm.int(), inv.int(), offsets.int(), counts.int()
    return MoEPlan(perm, inv, offsets, counts, k, N)


class _GatherFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, plan):
        ctx.plan = plan
        if _gpu(x):
            return ops().moe_gather(x.contiguous(), plan.perm, plan.k)
        return x[(plan.perm // plan.k).long()]

    @staticmethod
    def backward(ctx, g):
        p = ctx.plan
        if _gpu(g):
            return ops().moe_combine(g.contiguous(), p.inv, None, p.n_tokens, p.k), None
        return g[p.inv.long()].view(p.n_tokens, p.k, -1).sum(1), None


def gather(x, plan: MoEPlan):
    """x [N, D] -> expert-ordered rows [N*k, D] (row i = x[perm[i] // k])."""
    return _GatherFn.apply(x, plan)


class _CombineFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, yp, w, plan):
        ctx.plan = plan
        ctx.save_for_backward(yp, w)
        if _gpu(yp):
            return ops().moe_combine(yp.contiguous(), plan.inv, w.contiguous(), plan.n_tokens, plan.k)
        rows = yp[plan.inv.long()].view(plan.n_tokens, plan.k, -1)
        return (rows.float() * w[..., None]).sum(1).to(yp.dtype)

    @staticmethod
    def backward(ctx, g):
        yp, w = ctx.saved_tensors
        p = ctx.plan
        if _gpu(g):
            dyp, dw = ops().moe_combine_bwd(g.contiguous(), yp, p.perm, p.inv, w.contiguous(), p.k)
            return dyp, dw, None
        pl = p.perm.long()
        wa = w.reshape(-1)[pl]
        dyp = (g[pl // p.k].float() * wa[:, None]).to(yp.dtype)
        rows = yp[p.inv.long()].view(p.n_tokens, p.k, -1).float()
        dw = (rows * g.float()[:, None, :]).sum(-1)
        return dyp, dw, None


def combine(yp, w, plan: MoEPlan):
    """y[n] = sum_j w[n, j] * yp[inv[n*k + j]] (fp32 accumulation)."""
    return _CombineFn.apply(yp, w, plan)


# --------------------------------------------------------------------------- grouped GEMM
def _cpu_grouped(a, w, offsets, mode):
    off = offsets.tolist()
    if mode == 2:
        out = a.new_zeros(len(off) - 1, a.shape[1], w.shape[1])
        for e in range(len(off) - 1):
            if off[e + 1] > off[e]:
                out[e] = a[off[e]:off[e + 1]].t() @ w[off[e]:off[e + 1]]
        return out
    N = w.shape[1] if mode == 0 else w.shape[2]
    out = a.new_zeros(a.shape[0], N)
    for e in range(len(off) - 1):
        if off[e + 1] > off[e]:
            we = w[e].t() if mode == 0 else w[e]
            out[off[e]:off[e + 1]] = a[off[e]:off[e + 1]] @ we
    return out


GG8 = os.environ.get("SPA_GG8", "1") != "0"
GG8_DW = os.environ.get("SPA_GG8", "1") != "0"


def _gg8_ok(a, w, mode):
    """the 8-phase LDS-DMA kernel (csrc/kernels/gemm8.hip) needs a reduction dim % 64 in modes 0/1
    and output dims % 8. Measured at DeepSeek widths (profiles/r2_grouped_gemm_sweep.txt): fwd
    907 / 870 TF vs 560 / 530, dX 787 / 708 vs 653 / 623, dW 718 / 697 vs 687 / 690 for the
    register-staged moe.hip kernel, which SPA_GG8=0 selects."""
    if mode == 0:
        return w.shape[2] % 64 == 0 and w.shape[1] % 8 == 0
    if mode == 1:
        return w.shape[1] % 64 == 0 and w.shape[2] % 8 == 0
    return GG8_DW and a.shape[1] % 8 == 0 and w.shape[1] % 8 == 0


# the expert weight gradients (mode 2) on gemm4a.hip's register-staged 4-wave kernel (AGPR-resident
# accumulators): 817-820 vs 732-734 TF for gemm8 at dsv3_style widths, same process
# (profiles/r6_gemm4a.txt); fwd / dX stay on gemm8 (987 / 929 vs 939 / 924 TF). SPA_GG_DW=g8 reverts.
GG_DW_G4 = os.environ.get("SPA_GG_DW", "g4r") == "g4r"


def grouped_gemm(a, w, offsets, mode, out=None, accumulate=False):
    """mode 0: a_e @ w_e^T ; mode 1: a_e @ w_e ; mode 2: per-expert a_e^T @ w_e (w = X rows)."""
    if _gpu(a):
        a, w = a.contiguous(), w.contiguous()
        if mode == 2 and GG_DW_G4 and _gg8_ok(a, w, mode) and a.shape[1] % 8 == 0 and w.shape[1] % 8 == 0 \
                and offsets.numel() - 1 <= 256:
            return ops().gemm4a(a, w, offsets, 2, out, accumulate, 1)
        if GG8 and _gg8_ok(a, w, mode):
            return ops().grouped_gemm8(a, w, offsets, mode, out, accumulate)
        return ops().grouped_gemm(a, w, offsets, mode, out, accumulate)
    r = _cpu_grouped(a, w, offsets, mode)
    if out is None:
        return r
    if accumulate:
        out.add_(r.view_as(out))
    else:
        out.copy_(r.view_as(out))
    return out


class _GroupedLinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, xp, W, plan):
        ctx.plan, ctx.W = plan, W
        ctx.save_for_backward(xp)
        return grouped_gemm(xp, W, plan.offsets, 0)

    @staticmethod
    def backward(ctx, dy):
        (xp,) = ctx.saved_tensors
        W, plan = ctx.W, ctx.plan
        dy = dy.contiguous()
        dx = grouped_gemm(dy, W, plan.offsets, 1) if ctx.needs_input_grad[0] else None
        gw = commit_weight_grad(W, dy, xp, plan) if ctx.needs_input_grad[1] else None
        return dx, gw, None


# decode: at most this many expert-sorted rows go to the weight-streaming grouped GEMV
GEMV_MAX_ROWS = 64


def grouped_linear(xp, W, plan: MoEPlan, fp8: bool = False):
    """Per-expert ``xp[rows_e] @ W[e]^T`` for expert-ordered rows; W [E, out, in].
    ``fp8``: forward and dX products in OCP e4m3 on the block-scaled MFMA (per-row scales,
    csrc/kernels/moe_fp8.hip); dW stays bf16. Inference with few rows (decode) streams each
    active expert's weights once (``grouped_gemv``, csrc/kernels/gemv.hip) instead of paying a
    256-row MFMA tile per expert for one or two tokens."""
    if (xp.is_cuda and not torch.is_grad_enabled() and xp.shape[0] <= GEMV_MAX_ROWS
            and xp.dtype == torch.bfloat16 and W.dtype == torch.bfloat16):
        return ops().grouped_gemv(xp.contiguous(), W.contiguous(), plan.offsets)
    if fp8:
        return _GroupedLinearFP8Fn.apply(xp, W, plan)
    return _GroupedLinearFn.apply(xp, W, plan)


# --------------------------------------------------------------------------- fp8 path
def quant_rows_fp8(x):
    """Row-wise e4m3 quantization: (q, scale) with x ~= q * scale[:, None], scale = amax/448."""
    if x.is_cuda:
        q, s = ops().quant_rows_fp8(x.contiguous())
        return q, s
    x2 = x.reshape(-1, x.shape[-1]).float()
    s = (x2.abs().amax(-1) / 448.0).clamp_min(0)
    s = torch.where(s > 0, s, torch.ones_like(s))
    q = (x2 / s[:, None]).to(torch.float8_e4m3fn).view(x.shape)
    return q, s


def grouped_gemm_fp8(xq, sx, wq, sw, offsets):
    if xq.is_cuda:
        return ops().grouped_gemm_fp8(xq, sx, wq, sw.reshape(wq.shape[0], wq.shape[1]), offsets)
    x = xq.float() * sx[:, None]
    w = wq.float() * sw.reshape(wq.shape[0], wq.shape[1], 1)
    return _cpu_grouped(x, w, offsets, 0).to(torch.bfloat16)


def _quant_weight(W):
    E, N, K = W.shape
    q, s = quant_rows_fp8(W.reshape(E * N, K))
    return q.view(E, N, K), s.view(E, N)


# ---- DeepSeek-V3-style block scaling (1 x 128 activation tiles, 128 x 128 weight blocks, E8M0
# scales consumed by the MFMA scale operands: csrc/kernels/moe_fp8.hip)
_WEIGHT_EPOCH = [0]
_WQ_CACHE: dict = {}


def bump_weight_epoch():
    """Called by the optimizers after every parameter update: cached fp8 weight images are
    rebuilt once per step instead of once per forward/backward use."""
    _WEIGHT_EPOCH[0] += 1


def _blk_ok(W):
    return W.shape[1] % 128 == 0 and W.shape[2] % 128 == 0


def quant_act_fp8_blk(x):
    """x [R, K] -> (q e4m3, s uint8 E8M0 [R, K/128]); x ~= q * 2^(s - 127) per 128-wide tile."""
    if x.is_cuda:
        return tuple(ops().quant_act_fp8_blk(x.contiguous()))
    x2 = x.reshape(-1, x.shape[-1]).float()
    t = x2.view(x2.shape[0], -1, 128)
    e = _e8m0(t.abs().amax(-1))
    q = (t * torch.exp2(-e.float())[..., None]).clamp(-448, 448).to(torch.float8_e4m3fn)
    return q.view(x.shape), (e + 127).to(torch.uint8)


def _e8m0(amax):
    """smallest e with amax / 2^e <= 448 (0 for all-zero blocks) -- matches e8m0_exp on the GPU."""
    v = (amax / 448.0).float()
    e = torch.ceil(torch.log2(torch.where(v > 0, v, torch.ones_like(v))))
    e = torch.where(torch.exp2(e - 1) >= v, e - 1, e)          # guard log2 rounding up
    e = torch.where(torch.exp2(e) < v, e + 1, e)
    return torch.where(v > 0, e, torch.zeros_like(e)).clamp(-126, 127).to(torch.int32)


def quant_weight_fp8_blk(W):
    """W [E, N, K] -> (wq [E,N,K], wtq [E,K,N], s [E,N/128,K/128], st [E,K/128,N/128]); cached per
    weight version and optimizer step (never while a HIP graph is being captured)."""
    capturing = W.is_cuda and torch.cuda.is_current_stream_capturing()
    key = ("blk", W.data_ptr(), tuple(W.shape), W._version, _WEIGHT_EPOCH[0])
    hit = None if capturing else _WQ_CACHE.get(key)
    if hit is not None:
        return hit
    if W.is_cuda:
        out = tuple(ops().quant_weight_fp8_blk(W.detach().contiguous()))
    else:
        E, N, K = W.shape
        t = W.detach().float().view(E, N // 128, 128, K // 128, 128)
        e = _e8m0(t.abs().amax(dim=(2, 4)))                       # [E, NB, KB]
        q = (t * torch.exp2(-e.float())[:, :, None, :, None]).clamp(-448, 448).to(torch.float8_e4m3fn)
        q = q.view(E, N, K)
        out = (q, q.transpose(1, 2).contiguous(), (e + 127).to(torch.uint8),
               (e + 127).to(torch.uint8).transpose(1, 2).contiguous())
    if not capturing:
        for k in [k for k in _WQ_CACHE if k[:3] == key[:3]]:
            del _WQ_CACHE[k]
        _WQ_CACHE[key] = out
    return out


def dequant_act_fp8_blk(q, s, dtype=torch.bfloat16):
    """inverse of quant_act_fp8_blk (scale rows may be padded past K/128)."""
    if q.is_cuda:
        return ops().dequant_act_fp8_blk(q.contiguous(), s.contiguous()).to(dtype)
    R, K = q.shape
    return (q.float().view(R, -1, 128) * torch.exp2(s[:, :K // 128].float() - 127)[..., None]).view(R, K).to(dtype)


def commit_weight_grad(W, dy, xp, plan):
    """bf16 dW_e = dy_e^T xp_e (grouped), committed into W's gradient storage."""

    def _w(out, acc):
        if out is None:
            return grouped_gemm(dy, xp, plan.offsets, 2)
        if out.dtype == dy.dtype and out.is_contiguous():
            grouped_gemm(dy, xp, plan.offsets, 2, out=out.view(W.shape), accumulate=acc)
        else:
            g = grouped_gemm(dy, xp, plan.offsets, 2)
            if acc:
                out.add_(g.view_as(out))
            else:
                out.copy_(g.view_as(out))
    return commit(W, _w)


def quant_weight_fp8_rows(W):
    """2-D W [N, K] -> (wq [N,K] e4m3, sw [N], wtq [K,N] e4m3, swt [K]) with one fp32 scale per
    output channel (forward) / per input channel (dX); cached like the block images."""
    capturing = W.is_cuda and torch.cuda.is_current_stream_capturing()
    key = ("rows", W.data_ptr(), tuple(W.shape), W._version, _WEIGHT_EPOCH[0])
    hit = None if capturing else _WQ_CACHE.get(key)
    if hit is not None:
        return hit
    from .layout import transpose2d
    Wd = W.detach().contiguous()
    wq, sw = quant_rows_fp8(Wd)
    wtq, swt = quant_rows_fp8(transpose2d(Wd) if Wd.is_cuda else Wd.t().contiguous())
    out = (wq, sw, wtq, swt)
    if not capturing:
        for k in [k for k in _WQ_CACHE if k[:3] == key[:3]]:
            del _WQ_CACHE[k]
        _WQ_CACHE[key] = out
    return out


# Block-scaled fp8 GEMMs: the register-staged 32x32x64 kernel (moe_fp8.hip) or the 8-phase
# LDS-DMA kernel (csrc/kernels/gemm8_fp8.hip, v_mfma_scale_f32_16x16x128_f8f6f4). Same-process A/B
# at DeepSeek-V3 widths (tools/bench_fp8_g8.py, profiles/r3_fp8_g8_kernel_ab.txt): forward / dX
# within +-5 % of each other (the register kernel ahead at K <= 2048), the token-segment Wgrad 31-37 %
# faster on the 8-phase kernel (1.46-1.59 PF vs 1.07-1.21). SPA_FP8_G8: 1 (default) = 8-phase
# Wgrad, register forward / dX; 2 = 8-phase everywhere; 0 = register kernels everywhere.
FP8_G8 = int(os.environ.get("SPA_FP8_G8", "1"))


def grouped_gemm_fp8_blk(xq, sx, wq, sw, offsets):
    if xq.is_cuda:
        if FP8_G8 >= 2 and xq.shape[1] % 128 == 0:
            return ops().gemm8_fp8_blk(xq, sx, wq, sw, offsets)
        return ops().grouped_gemm_fp8_blk(xq, sx, wq, sw, offsets)
    x = xq.float().view(xq.shape[0], -1, 128) * torch.exp2(sx.float() - 127)[..., None]
    E, N, K = wq.shape
    w = wq.float().view(E, N // 128, 128, K // 128, 128) * torch.exp2(sw.float() - 127)[:, :, None, :, None]
    return _cpu_grouped(x.view(xq.shape), w.view(E, N, K), offsets, 0).to(torch.bfloat16)


# fp8 weight gradient of the routed experts (block-scaled path): dW_e = dY_e^T X_e with both
# operands quantized along the token (reduction) dimension in 128 x 1 tiles -- the DeepSeek-V3
# recipe's Wgrad quantization -- on the block-scaled MFMA (csrc/kernels/moe_fp8.hip
# quant_t_fp8_seg + wgrad_fp8_blk). SPA_FP8_WGRAD=0 keeps the bf16 grouped dW.
FP8_WGRAD = os.environ.get("SPA_FP8_WGRAD", "1") != "0"


def padded_offsets(offsets):
    """[E+1] device offsets -> [E+1] int32 offsets with every expert's segment padded to a
    multiple of 128 tokens (device ops only: no host sync)."""
    cnt = offsets[1:] - offsets[:-1]
    pc = (cnt + 127) // 128 * 128
    return torch.cat([offsets.new_zeros(1), torch.cumsum(pc, 0)]).to(torch.int32)


def quant_t_fp8_seg(x, offsets, poff, ld, rows=False):
    """x [T, C] (rows grouped by expert) -> (q [C, ld] e4m3 transposed, each expert's tokens at its
    128-aligned padded offset, zero-filled; s [C, ld/128] E8M0 per (channel, 128-token block)).
    ``rows``: also return quant_act_fp8_blk(x) (the 1 x 128 row image) from the same read."""
    if x.is_cuda:
        return tuple(ops().quant_t_fp8_seg(x.contiguous(), offsets, poff, int(ld), bool(rows)))
    if rows:
        return quant_t_fp8_seg(x, offsets, poff, ld) + quant_act_fp8_blk(x)
    C = x.shape[1]
    xt = torch.zeros(C, ld, dtype=torch.float32)
    for e in range(offsets.numel() - 1):
        a, b, p0 = int(offsets[e]), int(offsets[e + 1]), int(poff[e])
        xt[:, p0:p0 + (b - a)] = x[a:b].float().t()
    t = xt.view(C, ld // 128, 128)
    ex = _e8m0(t.abs().amax(-1))
    q = (t * torch.exp2(-ex.float())[..., None]).clamp(-448, 448).to(torch.float8_e4m3fn)
    return q.view(C, ld), (ex + 127).to(torch.uint8)


def wgrad_fp8_blk(aq, sa, bq, sb, poff, out=None, accumulate=False):
    """dW_e [M, N] (+)= aq[:, seg_e] bq[:, seg_e]^T on the images of :func:`quant_t_fp8_seg`."""
    if aq.is_cuda:
        if FP8_G8 >= 1:
            return ops().wgrad8_fp8_blk(aq, sa, bq, sb, poff, out, accumulate)
        return ops().wgrad_fp8_blk(aq, sa, bq, sb, poff, out, accumulate)
    M, ld = aq.shape
    a = (aq.float().view(M, ld // 128, 128) * torch.exp2(sa.float() - 127)[..., None]).view(M, ld)
    b = (bq.float().view(bq.shape[0], ld // 128, 128) * torch.exp2(sb.float() - 127)[..., None]).view(-1, ld)
    res = torch.stack([a[:, int(poff[e]):int(poff[e + 1])] @ b[:, int(poff[e]):int(poff[e + 1])].t()
                       for e in range(poff.numel() - 1)])
    if out is None:
        return res.to(torch.bfloat16)
    if accumulate:
        out.add_(res.to(out.dtype).view_as(out))
    else:
        out.copy_(res.view_as(out))
    return out


def _wgrad_fp8_ok(dy, xp, W):
    return FP8_WGRAD and W.shape[1] % 128 == 0 and W.shape[2] % 128 == 0 and dy.shape[0] > 0


def wgrad_ld(T, E):
    """host bound (multiple of 128) on the padded token count of T rows over E experts"""
    return (T + E * 127 + 127) // 128 * 128


def commit_weight_grad_fp8(W, aq, sa, bq, sb, poff):
    """fp8 dW_e = dy_e^T xp_e from the transposed images (aq, sa) of dy and (bq, sb) of xp
    (:func:`quant_t_fp8_seg`), committed into W's gradient storage."""
    def _w(out, acc):
        if out is None:
            return wgrad_fp8_blk(aq, sa, bq, sb, poff).view(W.shape)
        if out.is_contiguous() and out.dtype in (torch.bfloat16, torch.float32):
            wgrad_fp8_blk(aq, sa, bq, sb, poff, out.view(W.shape), acc)
        else:
            g = wgrad_fp8_blk(aq, sa, bq, sb, poff)
            if acc:
                out.add_(g.view_as(out))
            else:
                out.copy_(g.view_as(out))
    return commit(W, _w)


class _GroupedLinearFP8Fn(torch.autograd.Function):
    """fp8 expert projection. Block-scaled path (N, K % 128): X in 1 x 128 tiles, W in 128 x 128
    blocks, W^T for dX from the same quantized bytes; weights quantized once per optimizer step;
    dW on the same MFMA with dY and X quantized in 128 x 1 token tiles (FP8_WGRAD). Otherwise
    per-row scales and a bf16 grouped dW."""

    @staticmethod
    def forward(ctx, xp, W, plan):
        ctx.plan, ctx.W = plan, W
        ctx.blk = _blk_ok(W)
        ctx.wg8 = ctx.blk and _wgrad_fp8_ok(xp, xp, W)
        if ctx.wg8:
            # one read of xp: the 1 x 128 row image for this GEMM and the transposed 128 x 1 image
            # the fp8 dW needs -- saved INSTEAD of xp (half its bytes)
            ctx.poff, ctx.ld = padded_offsets(plan.offsets), wgrad_ld(xp.shape[0], W.shape[0])
            xtq, xts, xq, sx = quant_t_fp8_seg(xp, plan.offsets, ctx.poff, ctx.ld, rows=True)
            ctx.save_for_backward(xtq, xts)
            ctx.xshape = xp.shape
            wq, _, sw, _ = quant_weight_fp8_blk(W)
            return grouped_gemm_fp8_blk(xq, sx, wq, sw, plan.offsets).to(xp.dtype)
        ctx.save_for_backward(xp)
        if ctx.blk:
            xq, sx = quant_act_fp8_blk(xp)
            wq, _, sw, _ = quant_weight_fp8_blk(W)
            return grouped_gemm_fp8_blk(xq, sx, wq, sw, plan.offsets).to(xp.dtype)
        xq, sx = quant_rows_fp8(xp)
        wq, sw = _quant_weight(W)
        return grouped_gemm_fp8(xq, sx, wq, sw, plan.offsets).to(xp.dtype)

    @staticmethod
    def backward(ctx, dy):
        from .layout import transpose2d
        W, plan = ctx.W, ctx.plan
        dy = dy.contiguous()
        if ctx.wg8:
            xtq, xts = ctx.saved_tensors
            dtq, dts, dq, sd = quant_t_fp8_seg(dy, plan.offsets, ctx.poff, ctx.ld, rows=True)
            dx = None
            if ctx.needs_input_grad[0]:
                _, wtq, _, swt = quant_weight_fp8_blk(W)              # [E, in, out], cached
                dx = grouped_gemm_fp8_blk(dq, sd, wtq, swt, plan.offsets).to(dy.dtype)
            gw = commit_weight_grad_fp8(W, dtq, dts, xtq, xts, ctx.poff) if ctx.needs_input_grad[1] else None
            return dx, gw, None
        (xp,) = ctx.saved_tensors
        dx = None
        if ctx.needs_input_grad[0]:
            if ctx.blk:
                dq, sd = quant_act_fp8_blk(dy)
                _, wtq, _, swt = quant_weight_fp8_blk(W)              # [E, in, out], cached
                dx = grouped_gemm_fp8_blk(dq, sd, wtq, swt, plan.offsets).to(xp.dtype)
            else:
                dq, sd = quant_rows_fp8(dy)
                wtq, swt = _quant_weight(transpose2d(W))          # [E, in, out]
                dx = grouped_gemm_fp8(dq, sd, wtq, swt, plan.offsets).to(xp.dtype)
        gw = commit_weight_grad(W, dy, xp, plan) if ctx.needs_input_grad[1] else None
        return dx, gw, None


def moe_ffn(x, idx, w, W13, W2, act="silu", fp8=False):
    """Routed SwiGLU/GeGLU experts: sum_j w[n,j] * E_{idx[n,j]}(x[n]).

    ``W13`` [E, 2F, D] = per-expert [gate; up], ``W2`` [E, D, F].
    """
    from .activation import glu
    plan = permute(idx, W13.shape[0])
    xp = gather(x, plan)
    h = grouped_linear(xp, W13, plan, fp8)
    h = glu(h, act)
    yp = grouped_linear(h, W2, plan, fp8)
    return combine(yp, w, plan), plan


def load_counts(plan: MoEPlan):
    """Tokens routed to each expert (device int32 [E]) - the aux-free balancing signal."""
    return plan.counts
