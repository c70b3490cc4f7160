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
   experts the payload is e4m3 rows + 1 x 128 E8M0 scales (``_Fp8DispatchStart`` /
   ``_Fp8DispatchFinish``, on every path); the combine stays bf16;
4. the local experts run as ONE grouped GEMM per projection (csrc/kernels/moe.hip);
5. the inverse regroup + all-to-all return the rows; ``combine`` applies the gate
   weights in the original token order.

Capacity mode (``capacity`` > 0, DSV3Config.ep_capacity): no host sync at all. Every rank
sends every peer a fixed block of C rows (C = capacity x the balanced share A / P, capped at the
exact bound A / k * min(k, El)), so the exchange sizes are host constants; the slot maps (which
expert-sorted row goes to which block slot, which received slot lands in which (local expert,
src) row) are built on the device from the exchanged counts, and the grouped GEMMs take their
offsets from the device (tiles past the last expert exit). A block that would overflow sets a
device flag (max over the EP group, async); the model reads the flags once per forward
(``capacity_overflowed``) -- by then the GPU is still busy with the queued layers -- and re-runs
the forward with every layer's C set from the load it saw (x SPA_EP_CAP_MARGIN >= 1); if that
re-run still overflows (a downstream layer saw perturbed inputs), the next attempt uses the exact
split-size dispatch, so results never depend on C and training never stops on it
(models/deepseekv3.py ``_capacity_run``). Decode / prefill with a cache always takes the exact
path. The price is the padded wire bytes (P*C rows per rank instead of A).

Expert parameters carry ``p.expert_parallel = True``: DataParallel does not
all-reduce them across the EP group (each rank holds different experts) and the
optimizer's grad-norm sums their squares over the EP group.
"""
from __future__ import annotations

import math
import os
from types import SimpleNamespace

import torch
import torch.distributed as dist

from . import comm
from ..ops._ext import ops
from ..ops.activation import glu
from ..ops.moe import (combine, commit_weight_grad, dequant_act_fp8_blk, gather, grouped_gemm_fp8_blk, grouped_linear,
                       permute, quant_act_fp8_blk, quant_weight_fp8_blk)


def ep_rank_size(group):
    """(rank, size) in the EP group: a torch.distributed group, a comm.ProxyGroup, or None."""
    return comm.group_rank_size(group)


def _local(group, P):
    """No exchange: one EP rank -- unless SPA_FORCE_COLLECTIVES drives a real size-1 group."""
    if P > 1:
        return False
    from .dist import force_collectives
    return not (force_collectives() and group is not None and not comm.is_proxy(group))


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


class _Fp8DispatchStart(torch.autograd.Function):
    """fp8 dispatch, first half (DeepSeek-V3 sec. 3.3: dispatch in fp8, combine in bf16). Forward:
    issue the all-to-all of the e4m3 + E8M0 payload the caller quantized from the expert-sorted rows
    (``box.pay``, ~0.52x the bf16 bytes) -- from the launch stream after ``box.ev`` when given -- and
    return an empty token carrying the autograd edge to those rows. Backward: wait for the bf16
    reverse exchange that _Fp8DispatchFinish.backward issued and return it (the rows' gradient)."""

    @staticmethod
    def forward(ctx, xp, box):
        out_splits, in_splits = box.splits
        pay = box.pay
        box.recv = comm.alloc_for_launch((sum(out_splits), pay.shape[1]), pay) if box.ev is not None else \
            pay.new_empty((sum(out_splits), pay.shape[1]))
        box.work = comm.all_to_all_single(box.recv, pay, out_splits, in_splits, box.group, async_op=True, after=box.ev)
        ctx.box = box
        return xp.new_empty(0)

    @staticmethod
    def backward(ctx, g):
        box = ctx.box
        box.bwork.wait()
        dx, box.dx, box.gkeep, box.bwork = box.dx, None, None, None
        if box.cap is not None:                 # [P*C] block slots -> expert-sorted rows
            dx = _map_rows(dx, box.cap.send_back)
        return dx, None


class _Fp8DispatchFinish(torch.autograd.Function):
    """fp8 dispatch, second half, fused with the first expert projection. Forward: wait for the
    payload, regroup the received rows to (local expert, source) order and run the block-scaled W13
    grouped GEMM on them. Backward: dX in fp8 on the cached W^T bytes, regrouped back and sent home
    in bf16 (issued here, waited in _Fp8DispatchStart.backward), then dW13 while it is on the wire
    (fp8 128 x 1 token tiles of dh and of the received rows, or bf16 on the dequantized rows)."""

    @staticmethod
    def forward(ctx, token, W13, rc, offsets, box):
        box.work.wait()
        box.work = None
        D = box.D
        KB = D // 128
        pl = regroup_rows(box.recv, rc, True) if box.cap is None else _map_rows(box.recv, box.cap.recv_to)
        box.recv = box.pay = None
        xq_l = pl[:, :D].contiguous().view(torch.float8_e4m3fn)
        sx_l = pl[:, D:D + KB].contiguous()
        wq, _, sw, _ = quant_weight_fp8_blk(W13)
        ctx.save_for_backward(xq_l, sx_l, rc, offsets)
        ctx.W, ctx.box = W13, box
        return grouped_gemm_fp8_blk(xq_l, sx_l, wq, sw, offsets).to(box.dtype)

    @staticmethod
    def backward(ctx, dh):
        xq_l, sx_l, rc, offsets = ctx.saved_tensors
        W, box = ctx.W, ctx.box
        out_splits, in_splits = box.splits
        from ..ops import moe as _m
        dh = dh.contiguous()
        wg8 = ctx.needs_input_grad[1] and _m._wgrad_fp8_ok(dh, xq_l, W)
        if wg8:   # fp8 dW (128 x 1 token tiles): dh's transposed image + its dX row image, one read
            poff, ld = _m.padded_offsets(offsets), _m.wgrad_ld(dh.shape[0], W.shape[0])
            dtq, dts, dq, sd = _m.quant_t_fp8_seg(dh, offsets, poff, ld, rows=True)
        else:
            dq, sd = quant_act_fp8_blk(dh)
        _, wtq, _, swt = quant_weight_fp8_blk(W)
        dxl = grouped_gemm_fp8_blk(dq, sd, wtq, swt, offsets).to(dh.dtype)
        dxr = regroup_rows(dxl, rc, False) if box.cap is None else _map_rows(dxl, box.cap.recv_back)
        box.dx = dxr.new_empty((sum(in_splits), dxr.shape[1]))
        box.gkeep = dxr                       # the source must live until the exchange is done
        box.bwork = comm.all_to_all_single(box.dx, dxr, in_splits, out_splits, box.group, async_op=True)
        gw = None
        if wg8:   # the received rows are 1 x 128 tiles: dequantize, re-tile along tokens
            xtq, xts = _m.quant_t_fp8_seg(dequant_act_fp8_blk(xq_l, sx_l, dh.dtype), offsets, poff, ld)
            gw = _m.commit_weight_grad_fp8(W, dtq, dts, xtq, xts, poff)
        elif ctx.needs_input_grad[1]:
            gw = commit_weight_grad(W, dh, dequant_act_fp8_blk(xq_l, sx_l, dh.dtype), SimpleNamespace(offsets=offsets))
        return dh.new_empty(0), gw, None, None, None


class EPPrep:
    """Routing plan of one token chunk, with its per-(rank, expert) counts on their way to the
    host (``ep_prepare``); the dispatch reads them after one host sync."""

    def __init__(self, plan, counts=None, recv=None, host=None, ev=None):
        self.plan, self.counts, self.recv, self.host, self.ev = plan, counts, recv, host, ev

    def splits(self, P, El):
        """(send_splits, recv count matrix rc [P, El] on the host); waits for the D2H copy."""
        if self.ev is not None:
            self.ev.synchronize()
        both = self.host
        return both[0].view(P, El).sum(1).tolist(), both[1].view(P, El)


def ep_prepare(idx, n_experts, group, to_host=True):
    """Local permutation + the count exchange of a chunk, all on the device; the counts are
    copied to (pinned) host memory asynchronously (not in capacity mode: ``to_host=False``)."""
    plan = permute(idx, n_experts)
    rank, P = ep_rank_size(group)
    if _local(group, P):
        return EPPrep(plan)
    counts = plan.counts.to(torch.int64)
    recv = torch.empty_like(counts)
    comm.all_to_all_counts(recv, counts, group)              # recv[(src, e_local)]
    if not to_host:
        return EPPrep(plan, counts, recv)
    both = torch.stack([counts, recv])
    if both.is_cuda:
        host = torch.empty(both.shape, dtype=both.dtype, pin_memory=True)
        host.copy_(both, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        return EPPrep(plan, counts, recv, host, ev)
    return EPPrep(plan, counts, recv, both.clone())


# ----------------------------------------------------------------------------- capacity mode
# margin < 1 would size a re-run below the load it just saw (and overflow again): clamped to >= 1
_CAP = {"scale": 1.0, "pending": [], "margin": max(1.0, float(os.environ.get("SPA_EP_CAP_MARGIN", "1.1")))}


def capacity_rows(A, P, El, k, cf):
    """Rows per peer block: cf x the balanced share A / P, rounded up to 16, never above the
    exact bound (a token sends at most min(k, El) rows to one peer) rounded the same way."""
    bound = (A // max(k, 1)) * min(k, El)
    c = min(max(int(math.ceil(cf * A / P)), 1), max(bound, 1))
    return (c + 15) // 16 * 16


def capacity_bound_rows(A, El, k):
    """The exact per-peer bound (a token sends at most min(k, El) of its k rows to one peer),
    rounded up to 16: blocks of this size can never overflow (``capacity`` = inf)."""
    return (max((A // max(k, 1)) * min(k, El), 1) + 15) // 16 * 16


def capacity_scale() -> float:
    """Multiplier on every layer's capacity factor (doubled after each overflow of this process)."""
    return _CAP["scale"]


def capacity_overflowed() -> bool:
    """Read (and clear) the peer-block loads of the capacity dispatches issued since the last call:
    ONE host read of the group-max load of each. Each layer's capacity state then tracks its load
    (rows = max(margin x this load, 0.99 x the previous rows), SPA_EP_CAP_MARGIN default 1.1: a
    slowly decaying max, so alternating micro-batches with different loads do not flip-flop), and
    capacities follow the routing instead of a fixed factor. True if any block of any rank
    overflowed: the caller re-runs the step, which then fits (the same routing against the grown
    capacities)."""
    pend, _CAP["pending"] = _CAP["pending"], []
    if not pend:
        return False
    for work, *_ in pend:
        if work is not None:
            work.wait()
    loads = torch.cat([mx for _, mx, _, _ in pend]).tolist()
    over = False
    for (_, _, C, state), mx in zip(pend, loads):
        over |= mx > C
        if state is not None:
            want = max(mx * _CAP["margin"], mx, 0.99 * (state.rows or 0))
            state.rows = max(16, (int(math.ceil(want)) + 15) // 16 * 16)
        elif mx > C:
            grow_capacity()
    return over


def grow_capacity(factor: float = 2.0):
    _CAP["scale"] *= factor


def _cap_flag(counts, P, El, C, group, state):
    """This rank's largest peer block (rows), max over the group (async); read by
    :func:`capacity_overflowed` against the capacity C it was sent with."""
    mx = counts.view(P, El).sum(1).max().to(torch.int32).reshape(1)
    work = None
    if group is not None and not comm.is_proxy(group):
        work = comm.all_reduce(mx, group, async_op=True, op=dist.ReduceOp.MAX)
    _CAP["pending"].append((work, mx, C, state))


def _cap_send_index(offsets, P, El, C, A):
    """Slot of every expert-sorted row in the [P*C] send blocks (its peer's block, in expert order),
    or the dummy slot P*C for rows past a block's capacity. Device only."""
    starts = offsets.long()[::El].contiguous()          # [P + 1]: first row of each peer's experts, A
    r = torch.arange(A, device=offsets.device)
    p = torch.searchsorted(starts[1:].contiguous(), r, right=True).clamp_(max=P - 1)
    pos = r - starts[p]
    return torch.where(pos < C, p * C + pos, torch.full_like(pos, P * C))


def _cap_recv_dest(rc, C):
    """[P*C] received slots (src-major blocks, each block's rows by local expert) -> row of the
    (local expert, src)-major layout the grouped GEMMs read, or the dummy P*C for empty slots.
    Device only (batched searchsorted over the per-source count prefix sums)."""
    P, El = rc.shape
    rc = rc.long()
    cum = rc.cumsum(1)
    i = torch.arange(C, device=rc.device).expand(P, C).contiguous()
    e = torch.searchsorted(cum.contiguous(), i, right=True)
    valid = i < cum[:, -1:]
    e = e.clamp_(max=El - 1)
    excl = cum - rc
    emc = rc.t().reshape(-1)
    em = (emc.cumsum(0) - emc).view(El, P).t()          # em[s, e]: first row of (e, s)
    dest = em.gather(1, e) + i - excl.gather(1, e)
    valid &= dest < P * C                               # only on an overflowing (discarded) attempt
    return torch.where(valid, dest, torch.full_like(dest, P * C)).reshape(-1)


def _map_rows(x, m):
    """out[j] = x[m[j]], a zero row where m[j] < 0: ONE pass over the rows (csrc/kernels/moe.hip
    gather_rows_kernel, any 16-byte-multiple row width); the CPU path indexes a zero-padded copy."""
    if x.is_cuda:
        return ops().moe_gather(x, m, 1)
    xz = torch.cat([x, x.new_zeros((1,) + tuple(x.shape[1:]))])
    return xz[torch.where(m < 0, torch.full_like(m, x.shape[0]), m).long()]


class _RowMap(torch.autograd.Function):
    """Injective row move ``fwd`` (dest j <- src fwd[j], -1: zero row); its gradient is the move
    back along the inverse map ``inv`` (src i <- dest inv[i], -1: no dest). No atomics, no zero fill."""

    @staticmethod
    def forward(ctx, x, fwd, inv):
        ctx.inv = inv
        return _map_rows(x.contiguous(), fwd)

    @staticmethod
    def backward(ctx, g):
        return _map_rows(g.contiguous(), ctx.inv), None, None


def _cap_maps(slot, n):
    """From slot[i] (row i -> position in an n-row layout, n = dropped): (gather map of the n-row
    layout: position <- row or -1, gather map back: row <- position or -1), int32."""
    A = slot.numel()
    to = torch.full((n + 1,), -1, dtype=torch.int32, device=slot.device)
    to.index_copy_(0, slot, torch.arange(A, dtype=torch.int32, device=slot.device))
    back = torch.where(slot < n, slot, torch.full_like(slot, -1)).to(torch.int32)
    return to[:n].contiguous(), back


class EPStage:
    """One token chunk (e.g. one micro-batch) through an expert-parallel MoE layer, in four calls
    that a caller interleaves with other work (models/deepseekv3.py hidden_pair):

      ep_stage_prepare   routing plan, count exchange (its D2H starts), the expert-sorted rows and,
                         fp8, their e4m3 + E8M0 payload -- all queued on the compute stream; an
                         event marks the payload complete
      ep_stage_dispatch  the ONE host sync of the chunk (split sizes), then the exchange, issued from
                         the launch stream after that event: compute queued after the prepare (the
                         shared expert, another micro-batch's attention) runs while it is on the wire
      ep_stage_experts   wait, regroup, local grouped experts (W13 fused with the fp8 receive), and
                         the combine exchange issued right behind them
      ep_stage_finish    wait, weighted combine in the original token order

    fp8 (default for D, 2F multiples of 128): the dispatch payload is e4m3 + 1 x 128 E8M0 scales,
    the combine bf16. P == 1: no exchange, the same stages run the local experts."""

    def __init__(self):
        self.prep = self.xp = self.w = self.box = self.handle = self.chandle = self.cap = None


def ep_stage_prepare(x, idx, w, n_experts, group, fp8=False, W13=None, capacity=0.0, cap_state=None):
    """``capacity`` > 0: host-sync-free dispatch (module docstring), issued right here -- the
    exchange sizes are host constants, so nothing waits for the counts. ``cap_state``: the layer's
    capacity tracker (``.rows``, set from the loads it has seen; None on first use -> ``capacity``
    x the balanced share)."""
    st = EPStage()
    rank, P = ep_rank_size(group)
    cap = capacity > 0 and not _local(group, P)
    st.prep = ep_prepare(idx, n_experts, group, to_host=not cap)
    st.w = w
    st.group = group
    st.n_experts = n_experts
    st.xp = gather(x, st.prep.plan)                          # [A, D] sorted by global expert
    D = x.shape[-1]
    st.fp8 = bool(fp8)
    rank, P = ep_rank_size(group)
    local = _local(group, P)
    st.fp8_dispatch = st.fp8 and not local and D % 128 == 0 and (W13 is None or W13.shape[1] % 128 == 0)
    if st.fp8_dispatch:
        box = comm._Box()
        KB = D // 128
        q, sx = quant_act_fp8_blk(st.xp.detach())
        pad = (-KB) % 16
        box.pay = torch.cat([q.view(torch.uint8), torch.nn.functional.pad(sx, (0, pad))], 1).contiguous()
        box.D, box.dtype, box.group = D, x.dtype, group
        st.box = box
    st.ev = None
    if cap:
        El = n_experts // P
        A = idx.numel()
        k = idx.shape[-1] if idx.dim() > 1 else 1
        bound = math.isinf(capacity)        # blocks at the exact per-peer bound: cannot overflow
        if bound:
            C = capacity_bound_rows(A, El, k)
        else:
            C = capacity_rows(A, P, El, k, capacity * capacity_scale())
            if cap_state is not None and getattr(cap_state, "rows", None):
                C = cap_state.rows
        st.cap = SimpleNamespace(C=C, P=P, El=El)
        # send: block slot <- expert-sorted row (send_to), and back (send_back); receive: (local
        # expert, src) row <- received slot (recv_to), and back (recv_back)
        st.cap.send_to, st.cap.send_back = _cap_maps(_cap_send_index(st.prep.plan.offsets, P, El, C, A), P * C)
        rc = st.prep.recv.view(P, El)
        st.cap.recv_to, st.cap.recv_back = _cap_maps(_cap_recv_dest(rc, C), P * C)
        if not bound:
            _cap_flag(st.prep.counts, P, El, C, group, cap_state)
        per_e = rc.sum(0)
        st.rc_dev = rc
        # clamped to the P*C rows that exist: an overflowing attempt (re-run by the model) must still
        # never index past the buffers
        st.lplan = SimpleNamespace(offsets=torch.cat([per_e.new_zeros(1), per_e.cumsum(0)]).clamp_(max=P * C)
                                   .to(torch.int32))
        eq = [C] * P
        st.splits = (eq, eq)
        if st.fp8_dispatch:
            st.box.pay = _map_rows(st.box.pay, st.cap.send_to)
            st.box.splits, st.box.cap = (eq, eq), st.cap
        else:
            send = _RowMap.apply(st.xp, st.cap.send_to, st.cap.send_back)
        if x.is_cuda:
            st.ev = torch.cuda.Event()
            st.ev.record()
        if st.fp8_dispatch:
            st.box.ev = st.ev
            st.token = _Fp8DispatchStart.apply(st.xp, st.box)
        else:
            st.handle = comm.a2a_start(send, eq, eq, group, after=st.ev)
        return st
    if not local and x.is_cuda:
        st.ev = torch.cuda.Event()
        st.ev.record()
    return st


def ep_stage_dispatch(st):
    rank, P = ep_rank_size(st.group)
    if _local(st.group, P) or st.cap is not None:   # capacity mode: issued by ep_stage_prepare
        return st
    El = st.n_experts // P
    send_splits, rc = st.prep.splits(P, El)                  # the single host sync of the chunk
    recv_splits = rc.sum(1).tolist()
    per_e = rc.sum(0)
    loff = torch.cat([per_e.new_zeros(1), per_e.cumsum(0)])
    st.splits = (send_splits, recv_splits)
    st.rc_dev = st.prep.recv.view(P, El)                     # device copy of the counts
    st.lplan = SimpleNamespace(offsets=loff.to(device=st.xp.device, dtype=torch.int32))
    if st.fp8_dispatch:
        st.box.splits = (recv_splits, send_splits)
        st.box.ev = st.ev
        st.token = _Fp8DispatchStart.apply(st.xp, st.box)
    else:
        st.handle = comm.a2a_start(st.xp, recv_splits, send_splits, st.group, after=st.ev)
    return st


def ep_stage_experts(st, W13, W2, act="silu"):
    rank, P = ep_rank_size(st.group)
    if _local(st.group, P):
        plan = st.prep.plan
        h = glu(grouped_linear(st.xp, W13, plan, st.fp8), act)
        st.yp = grouped_linear(h, W2, plan, st.fp8)
        return st
    El = st.n_experts // P
    assert El * P == st.n_experts and W13.shape[0] == El, "experts must divide evenly over the EP group"
    send_splits, recv_splits = st.splits
    cap = st.cap
    if st.fp8_dispatch:
        h13 = _Fp8DispatchFinish.apply(st.token, W13, st.rc_dev, st.lplan.offsets, st.box)
    elif cap is not None:
        xl = _RowMap.apply(comm.a2a_finish(st.handle), cap.recv_to, cap.recv_back)
        h13 = grouped_linear(xl, W13, st.lplan, st.fp8)
    else:
        xl = _Regroup.apply(comm.a2a_finish(st.handle), st.rc_dev, True)   # (src, e) -> (e, src) rows
        h13 = grouped_linear(xl, W13, st.lplan, st.fp8)
    h = glu(h13, act)
    yl = grouped_linear(h, W2, st.lplan, st.fp8)
    yr = _RowMap.apply(yl, cap.recv_back, cap.recv_to) if cap is not None else _Regroup.apply(yl, st.rc_dev, False)
    st.chandle = comm.a2a_start(yr, send_splits, recv_splits, st.group)
    return st


def ep_stage_finish(st):
    rank, P = ep_rank_size(st.group)
    yp = st.yp if _local(st.group, P) else comm.a2a_finish(st.chandle)
    if st.cap is not None:                                   # [P*C] block slots -> expert-sorted rows
        yp = _RowMap.apply(yp, st.cap.send_back, st.cap.send_to)
    y = combine(yp, st.w, st.prep.plan)
    st.xp = st.yp = st.handle = st.chandle = st.box = st.token = st.cap = None
    return y


def ep_run(x, idx, w, W13, W2, n_experts, group, act="silu", fp8=False, capacity=0.0, cap_state=None):
    """Dispatch -> local grouped experts -> combine of one chunk, stage after stage (blocking).
    Returns (y, plan)."""
    st = ep_stage_prepare(x, idx, w, n_experts, group, fp8, W13, capacity, cap_state)
    ep_stage_experts(ep_stage_dispatch(st), W13, W2, act)
    plan = st.prep.plan
    return ep_stage_finish(st), plan


def ep_moe_ffn(x, idx, w, W13, W2, n_experts, group, act="silu", fp8=False, capacity=0.0):
    """Routed experts under expert parallelism. ``x`` [N, D] local tokens, ``idx``/``w``
    [N, k] local routing over ``n_experts`` global experts; ``W13`` [E/P, 2F, D] and
    ``W2`` [E/P, D, F] are this rank's experts. ``capacity`` > 0: host-sync-free padded
    dispatch (the caller checks :func:`capacity_overflowed`). Returns (y [N, D], local plan)."""
    return ep_run(x, idx, w, W13, W2, n_experts, group, act, fp8, capacity)


def shard_experts(full_w, rank, P):
    """Slice [E, ...] expert weights to this EP rank's [E/P, ...] block."""
    El = full_w.shape[0] // P
    return full_w[rank * El:(rank + 1) * El]
