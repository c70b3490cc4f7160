"""Tensor parallelism (Megatron-style) over RCCL, for the Gemma-7B-shape TP=8 config.

Column-parallel projections (q heads, GeGLU [gate|up]) take a replicated input
through ``copy_to_tp`` (identity fwd, all-reduce bwd); row-parallel projections (o,
down) end in ``reduce_from_tp`` (all-reduce fwd, identity bwd). With MQA (one KV
head < TP degree) the K/V projection is replicated and its activation gradient is
summed over the TP group (``reduce_grad_tp``). The vocabulary is sharded: embedding
rows and the tied LM head, with a vocab-parallel cross-entropy that exchanges only
per-row statistics ([N] floats), never logits.

Message sizing on xGMI: per layer 2 activation all-reduces fwd + 2 bwd of B*T*D bf16
(8192 x 3072 x 2 B = 50 MB), large enough to run near ring bandwidth.
All functions degrade to the single-GPU path when ``group`` is None.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from ..ops import embedding, linear_cross_entropy
from ..ops.xent import chunked_linear_cross_entropy
from . import comm


def tp_rank_size(group):
    """(rank, size) in the TP group: a torch.distributed group, a comm.ProxyGroup, or None."""
    return comm.group_rank_size(group)


def _ar(x, group):
    x = x.contiguous()
    comm.all_reduce(x, group)
    return x


class _CopyToTP(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        return _ar(g, ctx.group), None


class _ReduceFromTP(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, group):
        return _ar(x.clone(), group)

    @staticmethod
    def backward(ctx, g):
        return g, None


def copy_to_tp(x, group):
    return x if tp_rank_size(group)[1] == 1 else _CopyToTP.apply(x, group)


def reduce_from_tp(x, group):
    return x if tp_rank_size(group)[1] == 1 else _ReduceFromTP.apply(x, group)


reduce_grad_tp = copy_to_tp  # identity fwd, sum of activation grads over the TP group bwd


# ----------------------------------------------------------- sequence parallelism
# Megatron sequence parallelism: between the TP regions the residual stream is sharded
# along the sequence ([B, T/tp, D] per rank), so norms, residual adds and their
# activations are computed and stored once per token instead of tp times. Each
# row-parallel all-reduce becomes a reduce-scatter (over T) and each replicated input of
# a column-parallel region an all-gather (over T): same bytes on the wire as one
# all-reduce (RS + AG), split into two calls that bracket the local work.

def _gather_seq_raw(x, group):
    rank, tp = tp_rank_size(group)
    if comm.is_proxy(group):       # stand-in: every rank's shard is this one; wire time modelled
        out = group.gathered(x, 1)
        group._occupy(group.ag_seconds(out.numel() * out.element_size())).wait()
        return out
    if dist.get_backend(group) == "gloo":
        parts = [torch.empty_like(x) for _ in range(tp)]
        dist.all_gather(parts, x.contiguous(), group=group)
        return torch.cat(parts, dim=1)
    xt = x.transpose(0, 1).contiguous()                                 # [T/tp, B, ...]
    out = torch.empty((xt.shape[0] * tp,) + tuple(xt.shape[1:]), dtype=x.dtype, device=x.device)
    dist.all_gather_into_tensor(out, xt, group=group)
    return out.transpose(0, 1).contiguous()


def _reduce_scatter_seq_raw(x, group):
    rank, tp = tp_rank_size(group)
    assert x.shape[1] % tp == 0, "sequence parallelism needs T divisible by the TP size"
    if comm.is_proxy(group):       # stand-in: this rank's rows, unsummed; wire time modelled
        group._occupy(group.ag_seconds(x.numel() * x.element_size())).wait()
        return x.chunk(tp, dim=1)[0].contiguous()
    if dist.get_backend(group) == "gloo":                               # gloo has no reduce-scatter
        y = x.contiguous().clone()
        dist.all_reduce(y, group=group)
        return y.chunk(tp, dim=1)[rank].contiguous()
    xt = x.transpose(0, 1).contiguous()                                 # [T, B, ...]
    out = torch.empty((xt.shape[0] // tp,) + tuple(xt.shape[1:]), dtype=x.dtype, device=x.device)
    dist.reduce_scatter_tensor(out, xt, group=group)
    return out.transpose(0, 1).contiguous()


class _GatherSeq(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        return _gather_seq_raw(x, group)

    @staticmethod
    def backward(ctx, g):
        return _reduce_scatter_seq_raw(g, ctx.group), None


class _ReduceScatterSeq(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        return _reduce_scatter_seq_raw(x, group)

    @staticmethod
    def backward(ctx, g):
        return _gather_seq_raw(g, ctx.group), None


class _ScaleGrad(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, s):
        ctx.s = s
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        return g * ctx.s, None


def gather_seq(x, group):
    """[B, T/tp, ...] -> [B, T, ...]: all-gather fwd, reduce-scatter bwd."""
    return x if tp_rank_size(group)[1] == 1 else _GatherSeq.apply(x, group)


def reduce_scatter_seq(x, group):
    """Partial [B, T, ...] -> summed local shard [B, T/tp, ...]: reduce-scatter fwd, all-gather bwd."""
    return x if tp_rank_size(group)[1] == 1 else _ReduceScatterSeq.apply(x, group)


# ------------------------------------------------ async reduce-scatter -> all-gather
# The sequence-parallel layer boundary as ONE collective pair with no compute between its halves:
# a TP region's partial output (with this rank's residual rows already added, add_owner_rows)
# is reduce-scattered into the new residual shard, and that shard is all-gathered straight away
# into the next region's full-sequence input (whose norm then runs on every rank). Both are
# issued back to back on the communicator, so they can run under other work of the compute
# stream (the other chunk of Gemma._forward_sp_pair) and are waited for only where consumed.
# Backward mirrors it: the gathered input's gradient (with the residual shard's gradient added
# into this rank's rows) is reduce-scattered and all-gathered into the partial output's gradient.

def _rs_ag_launch(x, group):
    """Launch RS(x) -> shard and AG(shard) -> full on ``group``; returns (shard, full, works).
    x [B, T, ...] TP-partial; shard [B, T/tp, ...] = sum over ranks of this rank's rows."""
    rank, tp = tp_rank_size(group)
    B, T = x.shape[0], x.shape[1]
    assert T % tp == 0, "sequence parallelism needs T divisible by the TP size"
    if comm.is_proxy(group):       # stand-in: this rank's rows unsummed / every shard = this one
        shard = x.narrow(1, 0, T // tp).contiguous()
        full = group.gathered(shard, 1)
        w1 = group._occupy(group.ag_seconds(x.numel() * x.element_size()))
        w2 = group._occupy(group.ag_seconds(full.numel() * full.element_size()))
        return shard, full, (w1, w2)
    if dist.get_backend(group) == "gloo":                               # synchronous
        return _reduce_scatter_seq_raw(x, group), None, None
    xt = x.transpose(0, 1).contiguous()                                 # [T, B, ...]
    st = torch.empty((T // tp,) + tuple(xt.shape[1:]), dtype=x.dtype, device=x.device)
    ft = torch.empty_like(xt)
    w1 = dist.reduce_scatter_tensor(st, xt, group=group, async_op=True)
    w2 = dist.all_gather_into_tensor(ft, st, group=group, async_op=True)
    return st.transpose(0, 1), ft.transpose(0, 1), (w1, w2, xt)


def _rs_ag_wait(shard, full, works, group):
    if works is not None:
        for w in works[:2]:
            w.wait()
    if full is None:                                                    # gloo: gather now
        full = _gather_seq_raw(shard, group)
    return shard.contiguous(), full.contiguous()


class _RSAGStart(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, box):
        box.pay = _rs_ag_launch(x, box.group)
        ctx.box = box
        return x.new_empty(0)                # token: the results travel in the box

    @staticmethod
    def backward(ctx, g):
        box = ctx.box
        dx = _rs_ag_wait(*box.bwork, box.group)[1]
        box.bwork = None
        return dx, None


class _RSAGFinish(torch.autograd.Function):
    @staticmethod
    def forward(ctx, token, box):
        shard, full = _rs_ag_wait(*box.pay, box.group)
        box.pay = None
        ctx.box = box
        return shard, full

    @staticmethod
    def backward(ctx, g_shard, g_full):
        box = ctx.box
        rank, tp = tp_rank_size(box.group)
        g = g_full.contiguous().clone() if g_full is not None else None
        if g is None:
            T = g_shard.shape[1] * tp
            g = g_shard.new_zeros((g_shard.shape[0], T) + tuple(g_shard.shape[2:]))
        if g_shard is not None:              # the residual shard's gradient: this rank's rows
            g.narrow(1, rank * (g.shape[1] // tp), g.shape[1] // tp).add_(g_shard)
        box.bwork = _rs_ag_launch(g, box.group)
        return g.new_empty(0), None          # (a defined token gradient: the start node runs)


def rs_ag_start(x, group):
    """Launch the layer-boundary pair on the TP-partial ``x`` [B, T, ...]; finish with
    :func:`rs_ag_finish` where the results are consumed. In backward the reverse pair is launched
    at the finish node and waited for at the start node, so autograd work created between the two
    in the forward runs under it in the backward too."""
    box = comm._Box()
    box.group = group
    return _RSAGStart.apply(x, box), box


def rs_ag_finish(handle):
    """-> (residual shard [B, T/tp, ...], gathered full sequence [B, T, ...])."""
    token, box = handle
    return _RSAGFinish.apply(token, box)


def rs_ag(x, group):
    """Blocking form (start + finish back to back)."""
    return rs_ag_finish(rs_ag_start(x, group))


class _AddOwnerRows(torch.autograd.Function):
    """x[:, rank rows] += h in place (x a fresh TP-partial product, h this rank's residual shard):
    after the reduce-scatter sums the partials the shard holds h + the region's output."""

    @staticmethod
    def forward(ctx, x, h, rank, ts):
        ctx.rank, ctx.ts = rank, ts
        x.narrow(1, rank * ts, ts).add_(h)
        ctx.mark_dirty(x)
        return x

    @staticmethod
    def backward(ctx, g):
        return g, g.narrow(1, ctx.rank * ctx.ts, ctx.ts), None, None


def add_owner_rows(x, h, group):
    rank, tp = tp_rank_size(group)
    if h is None:
        return x
    return _AddOwnerRows.apply(x, h, rank, x.shape[1] // tp)


def scale_grad(x, s):
    """Identity forward, gradient times ``s``: a replicated consumer whose input gradient is
    already complete on every rank, feeding a gather_seq whose backward sums over ranks."""
    return x if s == 1 else _ScaleGrad.apply(x, s)


def sync_sequence_parallel_grads(params, group):
    """Replicated parameters used on sequence shards (norm weights, an MQA K/V projection) see
    only their shard's tokens: sum their gradients over the TP group (main_grad when present,
    else .grad) -- packed per dtype into one all-reduce."""
    if tp_rank_size(group)[1] == 1:
        return
    by_dtype = {}
    for p in params:
        g = getattr(p, "main_grad", None)
        g = g if g is not None else p.grad
        if g is not None:
            by_dtype.setdefault(g.dtype, []).append(g)
    for gs in by_dtype.values():
        flat = torch.cat([g.reshape(-1) for g in gs])
        comm.all_reduce(flat, group)
        torch._foreach_copy_(gs, [f.view_as(g) for f, g in zip(flat.split([g.numel() for g in gs]), gs)])


def vocab_parallel_embedding(w_local, ids, group, scale=1.0, sequence_parallel=False, reduce=True):
    """Rows [r*V/tp, (r+1)*V/tp) live on TP rank r; out-of-shard ids contribute zeros.
    With ``sequence_parallel`` the partial rows are reduce-scattered over T (the output is
    this rank's [B, T/tp, D] shard) instead of all-reduced; ``reduce=False`` returns the
    TP-partial rows (the caller reduces them, e.g. on another stream)."""
    rank, tp = tp_rank_size(group)
    if tp == 1:
        return embedding(w_local, ids, scale=scale)
    vl = w_local.shape[0]
    lo = rank * vl
    mask = (ids >= lo) & (ids < lo + vl)
    # other shards' tokens as -1: zero rows with no gradient (no mask multiply, and the backward's
    # scatter-add does not pile (tp-1)/tp of the tokens onto one row's atomics)
    x = embedding(w_local, torch.where(mask, ids - lo, torch.full_like(ids, -1)), scale=scale)
    if not reduce:
        return x
    return reduce_scatter_seq(x, group) if sequence_parallel else reduce_from_tp(x, group)


def vocab_parallel_cross_entropy(h, w_local, target, group, chunk_cols=None, reduce_dh=True):
    """mean CE(h @ W^T, target) with W sharded by rows (vocab) over the TP group.

    Runs the vocab-chunked fused head (ops/xent.py ``_ChunkedLinearXent``, HIP kernels
    ``xent_chunk_stats`` / ``xent_chunk_grad_``): per rank only a [N, Vc] chunk of its local
    logits is ever live, and the ranks exchange [N]-float statistics (row max, then
    sum-exp / target logit / logit sum in one packed all-reduce) -- never logits. Backward
    recomputes the chunks, writes dlogits in place into the dW / dh GEMMs and all-reduces the
    [N, D] dh partials (h is replicated over TP)."""
    if tp_rank_size(group)[1] == 1:
        return linear_cross_entropy(h, w_local, target)
    return chunked_linear_cross_entropy(h, w_local, target, group=group, chunk_cols=chunk_cols, reduce_dh=reduce_dh)


def gather_vocab_logits(logits_local, group):
    rank, tp = tp_rank_size(group)
    if tp == 1:
        return logits_local
    if comm.is_proxy(group):
        return torch.cat([logits_local] * tp, dim=-1)
    parts = [torch.empty_like(logits_local) for _ in range(tp)]
    dist.all_gather(parts, logits_local.contiguous(), group=group)
    return torch.cat(parts, dim=-1)


def shard_gemma_from_full(full, local, tp_rank, tp):
    """Copy a tp=1 Gemma's weights into a TP-sharded Gemma (tests / checkpoint import)."""
    c = full.c
    hd, F = c.head_dim, c.ffn_hidden
    with torch.no_grad():
        vl = c.vocab_size // tp
        local.embed.copy_(full.embed[tp_rank * vl:(tp_rank + 1) * vl])
        local.norm_f.copy_(full.norm_f)
        for a, b in zip(full.layers, local.layers):
            hl = c.n_heads // tp
            b.attn_norm.copy_(a.attn_norm)
            b.ffn_norm.copy_(a.ffn_norm)
            b.wq.copy_(a.wq[tp_rank * hl * hd:(tp_rank + 1) * hl * hd])
            b.wkv.copy_(a.wkv)
            b.wo.copy_(a.wo[:, tp_rank * hl * hd:(tp_rank + 1) * hl * hd])
            fl = F // tp
            b.w13.copy_(torch.cat([a.w13[tp_rank * fl:(tp_rank + 1) * fl], a.w13[F + tp_rank * fl:F + (tp_rank + 1) * fl]]))
            b.w2.copy_(a.w2[:, tp_rank * fl:(tp_rank + 1) * fl])
    return local
