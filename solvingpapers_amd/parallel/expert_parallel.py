"""Expert parallelism: each rank of an EP group owns E/P experts; tokens travel to
their experts and back with two variable-size all-to-alls over RCCL (xGMI is a full
point-to-point mesh inside a node, so one all-to-all uses all 7 links at once).

The reference keeps all 8 experts on every replica and runs them in a Python loop
(deepseekv3/deepseekv3.ipynb:1018,1059-1079). Dispatch here:

1. local routing + ``permute`` (device counting sort by global expert id);
2. per-expert counts exchanged with one tiny all-to-all; the split sizes are the only
   host sync (one D2H copy of 2*E ints per MoE layer);
3. token rows exchanged (``all_to_all_single`` with uneven splits) — they arrive
   ordered by (source rank, local expert) and are regrouped to (local expert, source)
   by one device kernel (``regroup_rows``, csrc/kernels/ep.hip; no host loop). With fp8
   experts the payload is e4m3 rows + 1 x 128 E8M0 scales (``_Fp8DispatchW13``);
   the combine stays bf16;
4. the local experts run as ONE grouped GEMM per projection (csrc/kernels/moe.hip);
5. the inverse regroup + all-to-all return the rows; ``combine`` applies the gate
   weights in the original token order.

Expert parameters carry ``p.expert_parallel = True``: DataParallel does not
all-reduce them across the EP group (each rank holds different experts) and the
optimizer's grad-norm sums their squares over the EP group.
"""
from __future__ import annotations

from types import SimpleNamespace

import torch

from . import comm
from ..ops._ext import ops
from ..ops.activation import glu
from ..ops.moe import (combine, commit_weight_grad, dequant_act_fp8_blk, gather, grouped_gemm_fp8_blk, grouped_linear,
                       permute, quant_act_fp8_blk, quant_weight_fp8_blk)


def ep_rank_size(group):
    """(rank, size) in the EP group: a torch.distributed group, a comm.ProxyGroup, or None."""
    return comm.group_rank_size(group)


def all_to_all(x, out_splits, in_splits, group):
    """Autograd all-to-all (the reverse exchange in backward) through parallel/comm.py."""
    return comm.a2a(x, out_splits, in_splits, group)


def _em_dest(rc):
    """rc [P, El] rows received from (src, local expert), laid out src-major. Returns, for
    every received row j, its position in the (local expert, src)-major order (CPU path of
    the ``ep_regroup`` kernel; vectorised, no per-segment host loop)."""
    P, El = rc.shape
    flat = rc.reshape(-1).long()
    R = int(flat.sum())
    seg = torch.repeat_interleave(torch.arange(P * El, device=rc.device), flat, output_size=R)
    sm = torch.cumsum(flat, 0) - flat
    emc = rc.t().reshape(-1).long()
    em = (torch.cumsum(emc, 0) - emc).view(El, P).t().reshape(-1)
    return em[seg] + (torch.arange(R, device=rc.device) - sm[seg])


def regroup_rows(x, rc, to_em: bool):
    """(src, expert)-major rows -> (expert, src)-major (``to_em``) or back. One HIP launch
    (csrc/kernels/ep.hip) that builds the segment prefix sums on chip from the device count
    matrix ``rc`` and copies whole rows; CPU tensors use the vectorised index path."""
    P, El = rc.shape
    if x.is_cuda:
        return ops().ep_regroup(x.contiguous(), rc.reshape(-1).long().contiguous(), P, El, bool(to_em))
    dest = _em_dest(rc)
    if to_em:
        y = torch.empty_like(x)
        y[dest] = x
        return y
    return x[dest]


class _Regroup(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, rc, to_em):
        ctx.rc, ctx.to_em = rc, to_em
        return regroup_rows(x, rc, to_em)

    @staticmethod
    def backward(ctx, g):
        return regroup_rows(g.contiguous(), ctx.rc, not ctx.to_em), None, None


class _Fp8DispatchW13(torch.autograd.Function):
    """fp8 dispatch fused with the first expert projection (DeepSeek-V3 sec. 3.3: dispatch in fp8,
    combine in bf16). The sender quantizes its expert-sorted rows once (1 x 128 E8M0 tiles); the
    all-to-all carries e4m3 bytes + scales (~0.52x the bf16 payload); the receiver regroups the
    packed rows and feeds them straight to the block-scaled grouped GEMM. Backward: dX in fp8 on
    the cached W^T bytes, returned in bf16 through the inverse regroup + all-to-all; dW in bf16
    on the dequantized received rows (the same values the forward consumed)."""

    @staticmethod
    def forward(ctx, xp, W13, rc, send_splits, recv_splits, offsets, group):
        D = xp.shape[1]
        KB = D // 128
        q, sx = quant_act_fp8_blk(xp)
        pad = (-KB) % 16
        pay = torch.cat([q.view(torch.uint8), torch.nn.functional.pad(sx, (0, pad))], 1).contiguous()
        pr = pay.new_empty((sum(recv_splits), pay.shape[1]))
        comm.all_to_all_single(pr, pay, recv_splits, send_splits, group)
        pl = regroup_rows(pr, rc, True)
        xq_l = pl[:, :D].contiguous().view(torch.float8_e4m3fn)
        sx_l = pl[:, D:D + KB].contiguous()
        wq, _, sw, _ = quant_weight_fp8_blk(W13)
        ctx.save_for_backward(xq_l, sx_l, rc, offsets)
        ctx.W, ctx.splits, ctx.group = W13, (send_splits, recv_splits), group
        return grouped_gemm_fp8_blk(xq_l, sx_l, wq, sw, offsets).to(xp.dtype)

    @staticmethod
    def backward(ctx, dh):
        xq_l, sx_l, rc, offsets = ctx.saved_tensors
        W, (send_splits, recv_splits) = ctx.W, ctx.splits
        from ..ops import moe as _m
        dh = dh.contiguous()
        lplan = SimpleNamespace(offsets=offsets)
        dxp = None
        wg8 = ctx.needs_input_grad[1] and _m._wgrad_fp8_ok(dh, xq_l, W)
        if wg8:   # fp8 dW (128 x 1 token tiles): dh's transposed image + its dX row image, one read
            poff, ld = _m.padded_offsets(offsets), _m.wgrad_ld(dh.shape[0], W.shape[0])
            dtq, dts, dq, sd = _m.quant_t_fp8_seg(dh, offsets, poff, ld, rows=True)
        if ctx.needs_input_grad[0]:
            if not wg8:
                dq, sd = quant_act_fp8_blk(dh)
            _, wtq, _, swt = quant_weight_fp8_blk(W)
            dxl = grouped_gemm_fp8_blk(dq, sd, wtq, swt, offsets).to(dh.dtype)
            dxr = regroup_rows(dxl, rc, False)
            dxp = dxr.new_empty((sum(send_splits), dxr.shape[1]))
            comm.all_to_all_single(dxp, dxr, send_splits, recv_splits, ctx.group)
        gw = None
        if wg8:   # the received rows are 1 x 128 tiles: dequantize, re-tile along tokens
            xtq, xts = _m.quant_t_fp8_seg(dequant_act_fp8_blk(xq_l, sx_l, dh.dtype), offsets, poff, ld)
            gw = _m.commit_weight_grad_fp8(W, dtq, dts, xtq, xts, poff)
        elif ctx.needs_input_grad[1]:
            gw = commit_weight_grad(W, dh, dequant_act_fp8_blk(xq_l, sx_l, dh.dtype), lplan)
        return dxp, gw, None, None, None, None, None


class EPPrep:
    """Routing plan of one token chunk, with its per-(rank, expert) counts on their way to the
    host (``ep_prepare``); ``ep_run`` reads them after one host sync."""

    def __init__(self, plan, counts=None, recv=None, host=None, ev=None):
        self.plan, self.counts, self.recv, self.host, self.ev = plan, counts, recv, host, ev

    def splits(self, P, El):
        """(send_splits, recv count matrix rc [P, El] on the host); waits for the D2H copy."""
        if self.ev is not None:
            self.ev.synchronize()
        both = self.host
        return both[0].view(P, El).sum(1).tolist(), both[1].view(P, El)


def ep_prepare(idx, n_experts, group):
    """Local permutation + the count exchange of a chunk, all on the device; the counts are
    copied to (pinned) host memory asynchronously. Issue the prepare of every chunk, plus any
    independent work (the shared expert), before the first ``ep_run``: its host sync then
    waits while the GPU is busy."""
    plan = permute(idx, n_experts)
    rank, P = ep_rank_size(group)
    if P == 1:
        return EPPrep(plan)
    counts = plan.counts.to(torch.int64)
    recv = torch.empty_like(counts)
    comm.all_to_all_counts(recv, counts, group)              # recv[(src, e_local)]
    both = torch.stack([counts, recv])
    if both.is_cuda:
        host = torch.empty(both.shape, dtype=both.dtype, pin_memory=True)
        host.copy_(both, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        return EPPrep(plan, counts, recv, host, ev)
    return EPPrep(plan, counts, recv, both.clone())


def ep_run(x, w, prep, W13, W2, n_experts, group, act="silu", fp8=False):
    """Dispatch -> local grouped experts -> combine for a chunk prepared by ``ep_prepare``."""
    plan = prep.plan
    rank, P = ep_rank_size(group)
    if P == 1:
        xp = gather(x, plan)
        h = glu(grouped_linear(xp, W13, plan, fp8), act)
        return combine(grouped_linear(h, W2, plan, fp8), w, plan), plan
    El = n_experts // P
    assert El * P == n_experts and W13.shape[0] == El, "experts must divide evenly over the EP group"
    send_splits, rc = prep.splits(P, El)                     # the single host sync of the chunk
    recv_splits = rc.sum(1).tolist()
    xp = gather(x, plan)                                      # [A, D] sorted by global expert
    per_e = rc.sum(0)
    loff = torch.cat([per_e.new_zeros(1), per_e.cumsum(0)])
    dev = x.device
    rc_dev = prep.recv.view(P, El)                           # device copy of the counts
    lplan = SimpleNamespace(offsets=loff.to(device=dev, dtype=torch.int32))
    D = x.shape[-1]
    if fp8 and D % 128 == 0 and W13.shape[1] % 128 == 0:
        # fp8 dispatch payload (e4m3 rows + E8M0 tile scales), fused with the W13 projection
        h13 = _Fp8DispatchW13.apply(xp, W13, rc_dev, send_splits, recv_splits, lplan.offsets, group)
    else:
        xr = all_to_all(xp, recv_splits, send_splits, group)  # [R, D] (src, e_local) order
        xl = _Regroup.apply(xr, rc_dev, True)                 # (src, e) -> (e, src) rows
        h13 = grouped_linear(xl, W13, lplan, fp8)
    h = glu(h13, act)
    yl = grouped_linear(h, W2, lplan, fp8)
    yr = _Regroup.apply(yl, rc_dev, False)
    yp = all_to_all(yr, send_splits, recv_splits, group)
    return combine(yp, w, plan), plan


def ep_run_interleaved(parts, ws, preps, W13, W2, n_experts, group, act="silu", fp8=False, shared=None):
    """Token chunks of ONE MoE layer on ONE compute stream, their all-to-alls interleaved so
    that each exchange is on the wire while another chunk's experts compute:

        start dispatch(0..n-1), shared(first half) | for c: finish dispatch(c), experts(c),
        start combine(c) | shared(second half) | for c: finish combine(c), combine(c)

    (comm.a2a_start / a2a_finish; autograd replays the same interleave in reverse, each
    reverse exchange launched before the other chunks' backward and waited after it). One
    stream, so chunks never compete for the CUs the way two concurrent grouped GEMMs do.
    ``shared(x_part)`` (the shared expert) covers the first dispatch and the last combine.
    Returns the per-chunk outputs (shared expert added)."""
    from . import comm as _c
    rank, P = ep_rank_size(group)
    El = n_experts // P
    assert El * P == n_experts and W13.shape[0] == El, "experts must divide evenly over the EP group"
    n = len(parts)
    meta, hd = [], []
    for i in range(n):
        send_splits, rc = preps[i].splits(P, El)
        recv_splits = rc.sum(1).tolist()
        per_e = rc.sum(0)
        loff = torch.cat([per_e.new_zeros(1), per_e.cumsum(0)])
        lplan = SimpleNamespace(offsets=loff.to(device=parts[i].device, dtype=torch.int32))
        meta.append((send_splits, recv_splits, preps[i].recv.view(P, El), lplan))
        hd.append(_c.a2a_start(gather(parts[i], preps[i].plan), recv_splits, send_splits, group))
    sh = [None] * n
    if shared is not None:                                   # under the first dispatch
        sh[0] = shared(parts[0])
    hc = []
    for i in range(n):
        send_splits, recv_splits, rc_dev, lplan = meta[i]
        xl = _Regroup.apply(_c.a2a_finish(hd[i]), rc_dev, True)
        h = glu(grouped_linear(xl, W13, lplan, fp8), act)
        yr = _Regroup.apply(grouped_linear(h, W2, lplan, fp8), rc_dev, False)
        hc.append(_c.a2a_start(yr, send_splits, recv_splits, group))
    if shared is not None:                                   # under the last combines
        for i in range(1, n):
            sh[i] = shared(parts[i])
    out = []
    for i in range(n):
        y = combine(_c.a2a_finish(hc[i]), ws[i], preps[i].plan)
        out.append(y + sh[i] if sh[i] is not None else y)
    return out


def ep_moe_ffn(x, idx, w, W13, W2, n_experts, group, act="silu", fp8=False):
    """Routed experts under expert parallelism. ``x`` [N, D] local tokens, ``idx``/``w``
    [N, k] local routing over ``n_experts`` global experts; ``W13`` [E/P, 2F, D] and
    ``W2`` [E/P, D, F] are this rank's experts. Returns (y [N, D], local plan)."""
    return ep_run(x, w, ep_prepare(idx, n_experts, group), W13, W2, n_experts, group, act, fp8)


def shard_experts(full_w, rank, P):
    """Slice [E, ...] expert weights to this EP rank's [E/P, ...] block."""
    El = full_w.shape[0] // P
    return full_w[rank * El:(rank + 1) * El]
