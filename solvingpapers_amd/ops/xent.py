"""Cross-entropy with in-place logit gradients (HIP: csrc/kernels/xent.hip).

``cross_entropy(logits, target)`` = mean CE over non-ignored rows. On the GPU
the gradient (softmax - onehot)/N is computed during the forward pass and
stored over the (dead) logits buffer, so backward is a single scale by the
incoming scalar gradient; the [T, V] logits are never duplicated.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist

from . import _ext
from . import reference
from .layout import bias_grad, wgrad, wgrad_operand
from .linear import dgrad
from ..utils.grad import commit, commit_tensor


class _XentFn(torch.autograd.Function):
    """CE whose gradient is written over the logits during forward. The logits
    buffer is CONSUMED (its producer must not need it for its own backward —
    true for a GEMM output); prefer :func:`linear_cross_entropy`, which never
    lets the logits escape."""

    @staticmethod
    def forward(ctx, logits, target, ignore_index, smoothing):
        V = logits.shape[-1]
        l2 = logits.reshape(-1, V)
        t = target.reshape(-1).contiguous()
        valid = (t != ignore_index).sum().clamp_min(1).float()
        inv = (1.0 / valid).reshape(1)
        loss, _ = _ext.ops().xent_fwd(l2, t, ignore_index, smoothing, True, inv)
        ctx.grad_buf = l2
        ctx.shape = logits.shape
        return loss.sum() * inv[0]

    @staticmethod
    def backward(ctx, g):
        grad = ctx.grad_buf
        ctx.grad_buf = None
        return grad.mul_(g.to(grad.dtype)).view(ctx.shape), None, None, None


class _LinearXentFn(torch.autograd.Function):
    """Fused LM head + cross-entropy: logits = h W^T (+b) -> CE; the logits
    buffer becomes d(loss)/d(logits) in place and is consumed by the two
    backward GEMMs (dh = G W, dW = G^T h written into W.main_grad)."""

    @staticmethod
    def forward(ctx, h, w, b, target, ignore_index, smoothing):
        D = h.shape[-1]
        h2 = h.reshape(-1, D)
        V = w.shape[0]
        # odd vocabularies (GPT-2's 50257) make every GEMM leading dimension misaligned;
        # run the head on a zero-padded copy (multiple of 128 rows: padded logits are exactly
        # 0 and are excluded from the softmax through the row stride), slice the results
        Vp = (V + 127) // 128 * 128 if V % 64 else V
        wp, bp = w, b
        if Vp != V:
            wp = w.new_zeros(Vp, D)
            wp[:V].copy_(w)
            if b is not None:
                bp = b.new_zeros(Vp)
                bp[:V].copy_(b)
        logits = torch.addmm(bp, h2, wp.t()) if bp is not None else torch.mm(h2, wp.t())
        t = target.reshape(-1).contiguous()
        valid = (t != ignore_index).sum().clamp_min(1).float()
        inv = (1.0 / valid).reshape(1)
        loss, _ = _ext.ops().xent_fwd(logits[:, :V], t, ignore_index, smoothing, True, inv)
        ctx.save_for_backward(h2)
        ctx.grad_buf, ctx.w, ctx.wp, ctx.b, ctx.hshape, ctx.V = logits, w, wp, b, h.shape, V
        return loss.sum() * inv[0]

    @staticmethod
    def backward(ctx, g):
        (h2,) = ctx.saved_tensors
        G = ctx.grad_buf                      # d(loss)/d(logits) for an upstream grad of 1
        ctx.grad_buf = None
        # the upstream grad g (a device scalar: 1 / accum in a gradient-accumulation loop) scales
        # the [N, D] / [N] sides of the products, never the [N, V] buffer: dh = g (G W),
        # dW = G^T (g h) -- a pass over G would stream 2 x N x V x 2 bytes (4.2 GB per LLaMA3-8B
        # micro-batch) through a broadcast-scalar elementwise kernel
        gs = g.to(G.dtype)
        w, b, wp = ctx.w, ctx.b, ctx.wp
        ctx.wp = None
        dh = None
        if ctx.needs_input_grad[0]:   # the cached-W^T form only for the persistent weight (not a padded copy)
            dh = (dgrad(G, wp) if wp is w else torch.mm(G, wp)).mul_(gs).view(ctx.hshape)
        G = G[:, :ctx.V]                      # padded columns are exactly 0
        gw = gb = None
        if ctx.needs_input_grad[1]:
            h2s = h2 * gs

            def _w(out, acc):
                return wgrad(G, h2s, out, acc)
            gw = commit(w, _w)
        if b is not None and ctx.needs_input_grad[2]:
            gb = commit_tensor(b, (bias_grad(G) * g.to(torch.float32)).to(b.dtype))
        return dh, gw, gb, None, None, None


# ----------------------------------------------------------------------------- vocab-chunked
# Logit-chunk budget for the chunked head: heads whose [N, V] logits exceed it run chunked.
XENT_CHUNK_BYTES = int(float(os.environ.get("SPA_XENT_CHUNK_MB", "2048")) * (1 << 20))
# size of one live logits chunk on the chunked path
XENT_CHUNK_BUDGET = int(float(os.environ.get("SPA_XENT_CHUNK_BUDGET_MB", "512")) * (1 << 20))


def _chunk_cols(N, V, elt, budget=None):
    budget = XENT_CHUNK_BUDGET if budget is None else budget
    c = max(256, (budget // max(1, N * elt)) // 256 * 256)
    return min(c, V)


def _stats_chunk(lc, t, v0, m, s, tl, sx):
    if lc.is_cuda:
        _ext.ops().xent_chunk_stats(lc, t, int(v0), m, s, tl, sx)
        return
    x = lc.to(m.dtype)
    cm = x.amax(-1)
    nm = torch.maximum(m, cm)
    s.copy_(torch.where(m == -float("inf"), torch.zeros_like(s), s * torch.exp(m - nm)) +
            torch.exp(x - nm[:, None]).sum(-1))
    m.copy_(nm)
    sx.add_(x.sum(-1))
    inside = (t >= v0) & (t < v0 + x.shape[1])
    idx = torch.where(inside, t - v0, torch.zeros_like(t))
    tl.copy_(torch.where(inside, x.gather(1, idx[:, None]).squeeze(1), tl))


def _grad_chunk_(lc, t, v0, lse, scale, ignore_index, smoothing, Vtot):
    if lc.is_cuda:
        _ext.ops().xent_chunk_grad_(lc, t, int(v0), lse, scale, int(ignore_index), float(smoothing), int(Vtot))
        return lc
    x = lc.to(lse.dtype)
    g = torch.exp(x - lse[:, None]) - smoothing / Vtot
    cols = torch.arange(v0, v0 + x.shape[1], device=x.device)
    g = g - (1.0 - smoothing) * (cols[None, :] == t[:, None]).to(x.dtype)
    sc = scale.to(x.dtype)
    g = g * torch.where(t != ignore_index, sc, torch.zeros_like(sc))[:, None]
    lc.copy_(g.to(lc.dtype))
    return lc


class _ChunkedLinearXent(torch.autograd.Function):
    """mean CE(h W^T + b, target) with the head computed in vocab chunks of ``Vc`` columns:
    forward folds each chunk's logits into per-row running (max, sum-exp, target logit, sum)
    and drops it; backward recomputes each chunk, turns it into d(loss)/d(logits) in place
    (``xent_chunk_grad_``) and feeds it straight into dh += G_c W_c and dW_c = G_c^T h.
    Peak extra memory is one [N, Vc] chunk instead of [N, V] (2.1 GB at 8192 x 128256 bf16).

    With ``group`` (tensor parallelism, W sharded by vocab rows over the group) the running
    statistics are combined across ranks with [N]-float all-reduces only -- never logits --
    and dh, a partial sum over the local vocabulary, is all-reduced in backward."""

    @staticmethod
    def forward(ctx, h, w, b, target, ignore_index, smoothing, group, Vc, reduce_dh=True):
        D = h.shape[-1]
        h2 = h.reshape(-1, D)
        N, Vl = h2.shape[0], w.shape[0]
        from ..parallel import comm
        rank, tp = comm.group_rank_size(group)
        v_off = rank * Vl
        Vtot = Vl * tp
        t = target.reshape(-1).contiguous().long()
        # running statistics in fp32 (fp64 for fp64 inputs: CPU oracle checks)
        f32 = dict(device=h.device, dtype=torch.float64 if h.dtype == torch.float64 else torch.float32)
        m = torch.full((N,), -float("inf"), **f32)
        s, tl, sx = torch.zeros(N, **f32), torch.zeros(N, **f32), torch.zeros(N, **f32)
        for v0 in range(0, Vl, Vc):
            v1 = min(Vl, v0 + Vc)
            lc = torch.mm(h2, w[v0:v1].t()) if b is None else torch.addmm(b[v0:v1], h2, w[v0:v1].t())
            _stats_chunk(lc, t, v_off + v0, m, s, tl, sx)
            del lc
        if tp > 1:
            gm = m.clone()
            comm.all_reduce(gm, group, op=dist.ReduceOp.MAX)
            s = torch.where(m == -float("inf"), torch.zeros_like(s), s * torch.exp(m - gm))
            pack = torch.stack([s, tl, sx])            # tl is 0 on ranks not owning the target
            comm.all_reduce(pack, group)
            s, tl, sx, m = pack[0], pack[1], pack[2], gm
        lse = m + torch.log(s)
        valid = t != ignore_index
        rows = (1.0 - smoothing) * (lse - tl) + smoothing * (lse - sx / Vtot)
        nvalid = valid.sum().clamp_min(1).to(lse.dtype)
        loss = torch.where(valid, rows, torch.zeros_like(rows)).sum() / nvalid
        ctx.save_for_backward(h2, w, t, lse, (1.0 / nvalid).reshape(1))
        ctx.b, ctx.hshape, ctx.cfg = b, h.shape, (ignore_index, smoothing, group, Vc, v_off, Vtot)
        ctx.reduce_dh = reduce_dh
        return loss

    @staticmethod
    def backward(ctx, g):
        h2, w, t, lse, inv = ctx.saved_tensors
        ignore_index, smoothing, group, Vc, v_off, Vtot = ctx.cfg
        b = ctx.b
        scale = (inv * g.to(inv.dtype)).reshape(1)
        Vl = w.shape[0]
        need_h, need_w = ctx.needs_input_grad[0], ctx.needs_input_grad[1]
        need_b = b is not None and ctx.needs_input_grad[2]
        acc_dt = lse.dtype
        dh = torch.zeros(h2.shape, device=h2.device, dtype=acc_dt) if need_h else None
        gb = torch.zeros(Vl, device=h2.device, dtype=acc_dt) if need_b else None
        gw = h2t = None
        for v0 in range(0, Vl, Vc):
            v1 = min(Vl, v0 + Vc)
            wc = w[v0:v1]
            lc = torch.mm(h2, wc.t()) if b is None else torch.addmm(b[v0:v1], h2, wc.t())
            G = _grad_chunk_(lc, t, v_off + v0, lse, scale, ignore_index, smoothing, Vtot)
            if need_h:
                _addmm_f32_(dh, G, wc)
            if need_w:
                if h2t is None:
                    h2t = wgrad_operand(G, h2)      # h2 transposed once for every chunk (or None)
                if getattr(w, "main_grad", None) is None:
                    if gw is None:                  # written chunk by chunk, no per-chunk parts + cat
                        gw = torch.empty(w.shape, device=w.device, dtype=G.dtype)
                    wgrad(G, h2, gw[v0:v1], x2t=h2t)
                else:
                    def _w(out, acc, G=G, v0=v0, v1=v1):
                        wgrad(G, h2, out[v0:v1], acc, x2t=h2t)
                    _commit_rows(w, _w, v0 == 0)
            if need_b:
                gb[v0:v1] = G.to(acc_dt).sum(0)
            del lc, G
        if need_h:
            from ..parallel import comm
            # h is replicated over TP: sum the fp32 vocab partials, then round once (a bf16 sum
            # would round every rank's partial before adding them)
            if ctx.reduce_dh and comm.group_rank_size(group)[1] > 1:
                comm.all_reduce(dh, group)
            dh = dh.to(h2.dtype).view(ctx.hshape)
        if need_b:
            gb = commit_tensor(b, gb.to(b.dtype))
        return dh, gw, gb, None, None, None, None, None, None


_ADDMM_F32 = None


def _addmm_f32_(acc32, a, b):
    """acc32 (fp32) += a @ b for bf16 a/b: hipBLASLt with an fp32 output when available
    (aten::addmm.dtype), else a bf16 product added in fp32."""
    global _ADDMM_F32
    if a.dtype == acc32.dtype:
        acc32.addmm_(a, b)
        return
    if a.is_cuda and _ADDMM_F32 is not False:
        try:
            torch.addmm(acc32, a, b, out_dtype=torch.float32, out=acc32)
            _ADDMM_F32 = True
            return
        except (RuntimeError, TypeError):
            _ADDMM_F32 = False
    acc32.add_(torch.mm(a, b))


def _commit_rows(w, compute, first_chunk):  # w has main_grad
    """commit() for a row slice of w's gradient: the generation bookkeeping happens on the first
    chunk only, so every chunk of one backward overwrites (or, when this backward accumulates,
    adds to) its own rows."""
    from ..utils.grad import _Gen
    mg = w.main_grad
    if first_chunk:
        w._spa_chunk_acc = getattr(w, "_spa_gen", -1) == _Gen.value
        w._spa_gen = _Gen.value
    compute(mg, w._spa_chunk_acc)
    return None


def chunked_linear_cross_entropy(h, w, target, bias=None, ignore_index=-100, label_smoothing=0.0, group=None,
                                 chunk_cols=None, reduce_dh=True):
    """Vocab-chunked fused LM head + CE (never holds [N, V]); ``group``: W is this TP rank's
    vocab shard and the CE is over the full (sharded) vocabulary. ``reduce_dh=False``: return
    this rank's vocab-partial input gradient (the caller all-reduces it, e.g. asynchronously with
    parallel/comm.grad_ar_start / grad_ar_finish around ``h``)."""
    N = h.numel() // h.shape[-1]
    Vc = chunk_cols or _chunk_cols(N, w.shape[0], h.element_size())
    return _ChunkedLinearXent.apply(h, w, bias, target, ignore_index, float(label_smoothing), group, int(Vc),
                                    bool(reduce_dh))


def linear_cross_entropy(h, w, target, bias=None, ignore_index=-100, label_smoothing=0.0):
    """mean CE(h @ w^T + bias, target) without exposing the [N, V] logits. Heads whose logits
    exceed SPA_XENT_CHUNK_MB run vocab-chunked (one [N, Vc] chunk live at a time)."""
    if h.is_cuda and h.dtype in (torch.bfloat16, torch.float32) and torch.is_grad_enabled() and (
            h.requires_grad or w.requires_grad):
        N = h.numel() // h.shape[-1]
        if N * w.shape[0] * h.element_size() > XENT_CHUNK_BYTES:
            return chunked_linear_cross_entropy(h, w, target, bias, ignore_index, label_smoothing)
        return _LinearXentFn.apply(h, w, bias, target, ignore_index, float(label_smoothing))
    logits = torch.nn.functional.linear(h, w, bias)
    return cross_entropy(logits, target, ignore_index, label_smoothing)


def cross_entropy(logits, target, ignore_index=-100, label_smoothing=0.0, reduction="mean"):
    """NOTE: on the GPU with grad enabled, ``logits`` is overwritten by its gradient."""
    if logits.is_cuda and logits.dtype in (torch.bfloat16, torch.float32):
        if reduction == "mean" and torch.is_grad_enabled() and logits.requires_grad:
            return _XentFn.apply(logits, target, ignore_index, float(label_smoothing))
        V = logits.shape[-1]
        loss, _ = _ext.ops().xent_fwd(logits.reshape(-1, V), target.reshape(-1).contiguous(), ignore_index,
                                      float(label_smoothing), False, None)
        if reduction == "none":
            return loss.view(target.shape)
        if reduction == "sum":
            return loss.sum()
        return loss.sum() / (target != ignore_index).sum().clamp_min(1)
    lg = logits.reshape(-1, logits.shape[-1])
    lg = lg if lg.dtype == torch.float64 else lg.float()        # fp64 parity tests keep fp64
    return torch.nn.functional.cross_entropy(lg, target.reshape(-1),
                                             ignore_index=ignore_index, label_smoothing=label_smoothing,
                                             reduction=reduction)


def per_row_loss(logits, target, ignore_index=-100):
    if logits.is_cuda:
        V = logits.shape[-1]
        return _ext.ops().xent_fwd(logits.reshape(-1, V), target.reshape(-1).contiguous(), ignore_index, 0.0,
                                   False, None)[0]
    return reference.cross_entropy(logits.reshape(-1, logits.shape[-1]), target.reshape(-1), ignore_index)
