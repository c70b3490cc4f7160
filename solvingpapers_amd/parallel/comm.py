"""Collectives for the TP / EP paths, and a one-GPU stand-in group to measure overlap.

Every TP / EP collective of the framework goes through :func:`all_reduce` /
:func:`all_to_all_single` here, so the same model code runs over

* a ``torch.distributed`` process group (RCCL on the GPU, gloo on the CPU), and
* a :class:`ProxyGroup`: ONE GPU standing in for a group of ``size`` ranks. A collective
  returns its input unchanged (all-reduce), copies it straight across (all-to-all:
  every rank sends as much as it receives), or treats every rank's shard as this one
  (all-gather / reduce-scatter over the sequence, parallel/tensor_parallel.py), and meanwhile a streaming kernel occupies the
  proxy's own "comm stream" for the time the real collective would take on xGMI
  (``bytes on the wire / modelled bandwidth``), with ``nwg`` workgroups -- the CU footprint
  of an RCCL ring kernel with that many channels. Ops on the compute stream that do not
  wait for it overlap with it, as they would with RCCL's stream.

The proxy exists because the framework's TP=8 / EP=8 configs cannot be run on the 1-GPU
development boxes; ``tools/overlap_proxy.py`` times layers with collectives (a) modelled
and overlapped, (b) modelled and made blocking, (c) skipped, and reports how much of the
collective time the overlap hides. The modelled bandwidths are inputs, not measurements:
RCCL's large-message all-reduce bus bandwidth and all-to-all per-rank bandwidth over the 7
xGMI links of an MI355X (defaults below; override per run).
"""
from __future__ import annotations

import os
import time
from typing import List

import torch
import torch.distributed as dist

# modelled RCCL rates on one 8x MI355X node (inputs of the proxy, not measured here):
# ring all-reduce bus bandwidth ~ per-link bound x channels; all-to-all uses all 7 links
PROXY_AR_BUSBW_GBPS = 300.0
PROXY_A2A_GBPS = 300.0

# Stream priority of the TP / EP collective streams (RCCL is_high_priority_stream; the proxy's
# comm stream). Measured with round 3's two-stream pipelines on the 1-GPU proxy
# (profiles/r3_overlap_proxy_priorities.jsonl): high priority helped TP (hidden 0.30 -> 0.35) but
# slowed the EP layer's compute 15 %, so it defaults to normal (0); SPA_COMM_PRIO=-1 selects high.
COMM_PRIORITY = int(os.environ.get("SPA_COMM_PRIO", "0"))


class ProxyGroup:
    """A stand-in process group of ``size`` ranks living on one GPU (see module doc).

    mode: ``"overlap"`` -- collectives run on the proxy's comm stream, the caller's stream
    waits only where the result is consumed (``Work.wait``); ``"blocking"`` -- the caller's
    stream waits right away (a collective that overlaps nothing); ``"off"`` -- no stand-in
    kernel at all (compute-only reference)."""

    def __init__(self, size: int, device=None, ar_busbw_gbps: float = PROXY_AR_BUSBW_GBPS,
                 a2a_gbps: float = PROXY_A2A_GBPS, nwg: int = 16, buf_mb: int = 8, mode: str = "overlap",
                 synth_gather: bool = False):
        """``synth_gather``: an all-gather's output is a cached random buffer of the gathered
        shape instead of a compute-stream concatenation of this rank's shard -- a real
        all-gather's output is written by the collective (whose time the stand-in kernel
        models), so timing runs (tools/overlap_proxy.py) should not charge the compute stream
        for it. Off by default: value tests want the replicated shard."""
        self.size, self.rank = int(size), 0
        self.synth_gather = bool(synth_gather)
        self._gcache = {}
        self.device = torch.device(device or "cuda")
        self.ar_bw, self.a2a_bw = ar_busbw_gbps * 1e9, a2a_gbps * 1e9
        self.nwg, self.mode = int(nwg), mode
        self.stream = (torch.cuda.Stream(self.device, priority=COMM_PRIORITY) if self.device.type == "cuda"
                       else None)
        n = buf_mb << 20
        self._src = torch.empty(n, dtype=torch.uint8, device=self.device)
        self._dst = torch.empty_like(self._src)
        self._rep_s = None
        self.modelled_s = 0.0            # sum of modelled collective time issued (for reports)
        self.calls = 0

    # ------------------------------------------------------------------ timing
    def _calibrate(self):
        from ..ops._ext import ops
        o = ops()
        o.stream_copy_wg(self._src, self._dst, self.nwg, 4)
        torch.cuda.synchronize(self.device)
        reps = 32
        t0 = time.perf_counter()
        o.stream_copy_wg(self._src, self._dst, self.nwg, reps)
        torch.cuda.synchronize(self.device)
        self._rep_s = (time.perf_counter() - t0) / reps

    def _occupy(self, seconds: float):
        """Run the stand-in kernel on the comm stream for ~seconds, after the caller's
        stream reaches this point. Returns a Work."""
        self.modelled_s += seconds
        self.calls += 1
        if self.mode == "off" or self.stream is None:
            return _DoneWork()
        from ..ops._ext import ops
        if self._rep_s is None:
            self._calibrate()
        reps = int(round(seconds / self._rep_s))
        cur = torch.cuda.current_stream(self.device)
        if reps == 0:          # below the stand-in's granularity (a few tens of us): latency only
            ev = torch.cuda.Event()
            ev.record(cur)
            return _DoneWork()
        self.stream.wait_stream(cur)
        with torch.cuda.stream(self.stream):
            ops().stream_copy_wg(self._src, self._dst, self.nwg, reps)
            ev = torch.cuda.Event()
            ev.record(self.stream)
        w = _EventWork(ev)
        if self.mode == "blocking":
            w.wait()
            return _DoneWork()
        return w

    def gathered(self, shard, dim: int):
        """The stand-in all-gather output of ``shard`` along ``dim`` (see ``synth_gather``)."""
        if not self.synth_gather:
            return torch.cat([shard] * self.size, dim=dim)
        shape = list(shard.shape)
        shape[dim] *= self.size
        key = (tuple(shape), shard.dtype, shard.device)
        buf = self._gcache.get(key)
        if buf is None:       # random (not constant) data: MFMA power / clocks depend on it
            g = torch.Generator(device=shard.device).manual_seed(len(self._gcache) + 11)
            buf = torch.randn(shape, generator=g, device=shard.device, dtype=torch.float32).to(shard.dtype)
            self._gcache[key] = buf
        return buf

    def ar_seconds(self, nbytes: int) -> float:
        n = self.size
        return 2.0 * (n - 1) / n * nbytes / self.ar_bw

    def ag_seconds(self, nbytes_full: int) -> float:
        """All-gather (or reduce-scatter) whose gathered (unscattered) tensor is nbytes_full:
        half an all-reduce of it at the same bus bandwidth."""
        n = self.size
        return (n - 1) / n * nbytes_full / self.ar_bw

    def a2a_seconds(self, nbytes_sent: int) -> float:
        return (self.size - 1) / self.size * nbytes_sent / self.a2a_bw

    def reset_stats(self):
        self.modelled_s, self.calls = 0.0, 0


class _DoneWork:
    def wait(self):
        return True


class _EventWork:
    def __init__(self, ev):
        self.ev = ev

    def wait(self):
        torch.cuda.current_stream().wait_event(self.ev)
        return True


def is_proxy(group) -> bool:
    return isinstance(group, ProxyGroup)


def group_rank_size(group):
    """(rank, size) of ``group``; (0, 1) when there is no group / no process group."""
    if group is None:
        return 0, 1
    if is_proxy(group):
        return group.rank, group.size
    if not dist.is_initialized():
        return 0, 1
    return dist.get_rank(group), dist.get_world_size(group)


def backend(group) -> str:
    if is_proxy(group):
        return "proxy"
    return dist.get_backend(group)


def all_reduce(t: torch.Tensor, group, async_op: bool = False, op=None):
    """In-place sum (or ``op``) over ``group``. ``async_op``: returns a Work whose ``wait()``
    makes the CURRENT stream wait (RCCL) -- launch early, wait where the result is consumed."""
    if is_proxy(group):
        w = group._occupy(group.ar_seconds(t.numel() * t.element_size()))
        return w if async_op else w.wait()
    if op is None:
        return dist.all_reduce(t, group=group, async_op=async_op)
    return dist.all_reduce(t, op=op, group=group, async_op=async_op)


_LAUNCH = {}


def launch_stream(device):
    """Per-device stream that collectives are ISSUED from when they must start right after an
    earlier point of the compute stream (``after`` event) instead of after everything queued on it
    by the time the host knows the split sizes (work queued meanwhile then overlaps the exchange)."""
    d = torch.device(device)
    key = d.index if d.index is not None else torch.cuda.current_device()
    if key not in _LAUNCH:
        _LAUNCH[key] = torch.cuda.Stream(d)
    return _LAUNCH[key]


def all_to_all_single(out: torch.Tensor, inp: torch.Tensor, out_splits: List[int], in_splits: List[int], group,
                      async_op: bool = False, after=None):
    """Variable-split all-to-all into ``out``. The proxy copies ``inp`` across (sizes must
    match: a balanced exchange) while modelling the time of the bytes that leave the rank.
    ``after`` (a CUDA event recorded when ``inp`` was complete; async only): the exchange is issued
    from :func:`launch_stream` waiting on that event alone, so compute queued on the current stream
    after the event runs beside it. ``out`` must then have been allocated on the launch stream (or
    before the event) -- see :func:`alloc_for_launch`."""
    if after is not None and async_op and inp.is_cuda:
        ls = launch_stream(inp.device)
        ls.wait_event(after)
        # inp was allocated on the compute stream and may be freed there (a temporary) before the
        # exchange on the launch stream has read it: keep its block out of the pool until then
        inp.record_stream(ls)
        with torch.cuda.stream(ls):
            w = all_to_all_single(out, inp, out_splits, in_splits, group, async_op=True)
        return w
    if is_proxy(group):
        assert out.shape == inp.shape, "proxy all-to-all models a balanced exchange"
        out.copy_(inp)
        w = group._occupy(group.a2a_seconds(inp.numel() * inp.element_size()))
        return w if async_op else w.wait()
    return dist.all_to_all_single(out, inp, list(out_splits), list(in_splits), group=group, async_op=async_op)


def alloc_for_launch(shape, like: torch.Tensor):
    """An output buffer for an ``after=`` collective: allocated from the launch stream's pool (a
    block freed by compute-stream work queued after the event can never be handed out here) and
    marked as used by the current stream, where its consumer runs."""
    if not like.is_cuda:
        return like.new_empty(shape)
    ls = launch_stream(like.device)
    with torch.cuda.stream(ls):
        out = like.new_empty(shape)
    out.record_stream(torch.cuda.current_stream(like.device))
    return out


def all_to_all_counts(recv: torch.Tensor, counts: torch.Tensor, group):
    """Exchange of per-(rank, expert) counts (tiny). The proxy returns the counts unchanged:
    every rank sends the same histogram it receives."""
    if is_proxy(group):
        recv.copy_(counts)
        return
    dist.all_to_all_single(recv, counts, group=group)


# ----------------------------------------------------------------- autograd pieces
class _Box:
    """Hand-off between a collective's start and finish nodes (forward and backward)."""
    __slots__ = ("work", "bwork", "splits", "group", "dx", "gkeep", "ev", "pay", "recv", "D", "dtype", "cap")

    def __init__(self):
        self.work = self.bwork = self.dx = self.gkeep = self.ev = self.pay = self.recv = self.cap = None


class _A2AStart(torch.autograd.Function):
    """Forward: launch the all-to-all of x into a fresh buffer (not yet valid) and return the
    buffer; backward: wait for the reverse all-to-all launched by _A2AFinish.backward and
    return its result (the gradient of x)."""

    @staticmethod
    def forward(ctx, x, box):
        out_splits, in_splits = box.splits
        shape = (sum(out_splits),) + tuple(x.shape[1:])
        out = alloc_for_launch(shape, x) if box.ev is not None else x.new_empty(shape)
        box.work = all_to_all_single(out, x.contiguous(), out_splits, in_splits, box.group, async_op=True,
                                     after=box.ev)
        ctx.box = box
        return out

    @staticmethod
    def backward(ctx, g):
        box = ctx.box
        box.bwork.wait()
        # drop the Work too: it holds the exchange's input and output until it is destroyed
        dx, box.dx, box.gkeep, box.bwork = box.dx, None, None, None
        return dx, None


class _A2AFinish(torch.autograd.Function):
    """Forward: wait for the all-to-all (the buffer becomes valid here); backward: launch the
    reverse all-to-all of the gradient into a pending buffer kept in the box."""

    @staticmethod
    def forward(ctx, buf, box):
        box.work.wait()
        box.work = None
        ctx.box = box
        return buf.view_as(buf)

    @staticmethod
    def backward(ctx, g):
        box = ctx.box
        out_splits, in_splits = box.splits
        gc = g.contiguous()
        box.dx = g.new_empty((sum(in_splits),) + tuple(g.shape[1:]))
        box.gkeep = gc                       # the source must live until the exchange is done
        box.bwork = all_to_all_single(box.dx, gc, in_splits, out_splits, box.group, async_op=True)
        return gc, None


def a2a_start(x, out_splits, in_splits, group, after=None):
    """Start an overlappable all-to-all. Returns a handle for :func:`a2a_finish`; ops issued
    between the two (forward) -- and, in reverse, between their backward nodes -- run while
    the rows are on the wire. Autograd runs backward nodes in reverse creation order, so
    work created between start and finish in the forward lands between the reverse
    all-to-all's launch and its wait in the backward. ``after``: an event recorded when ``x``
    was complete -- the exchange then starts there, not behind work queued since
    (see :func:`all_to_all_single`)."""
    box = _Box()
    box.splits, box.group, box.ev = (list(out_splits), list(in_splits)), group, after
    return _A2AStart.apply(x, box), box


def a2a_finish(handle):
    buf, box = handle
    return _A2AFinish.apply(buf, box)


def a2a(x, out_splits, in_splits, group):
    """Blocking (start + finish back to back) all-to-all with autograd."""
    return a2a_finish(a2a_start(x, out_splits, in_splits, group))


class _ARStart(torch.autograd.Function):
    """Row-parallel output: forward launches the all-reduce (async) of x; backward identity."""

    @staticmethod
    def forward(ctx, x, box):
        y = x.contiguous().clone()
        box.work = all_reduce(y, box.group, async_op=True)
        return y

    @staticmethod
    def backward(ctx, g):
        return g, None


class _ARFinish(torch.autograd.Function):
    @staticmethod
    def forward(ctx, y, box):
        box.work.wait()
        box.work = None
        return y.view_as(y)

    @staticmethod
    def backward(ctx, g):
        return g, None


def ar_start(x, group):
    """Start the forward all-reduce of a row-parallel output; finish with :func:`ar_finish`
    where the sum is consumed (identity backward, Megatron's g)."""
    box = _Box()
    box.group = group
    return _ARStart.apply(x, box), box


def ar_finish(handle):
    y, box = handle
    return _ARFinish.apply(y, box)


class _GradARStart(torch.autograd.Function):
    """Identity forward; backward waits for the gradient all-reduce launched by
    _GradARFinish.backward and returns its result."""

    @staticmethod
    def forward(ctx, x, box):
        ctx.box = box
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        box = ctx.box
        box.bwork.wait()
        dx, box.dx, box.bwork = box.dx, None, None
        return dx, None


class _GradARFinish(torch.autograd.Function):
    """Identity forward; backward launches the all-reduce of the incoming gradient (in place,
    async) and hands it to _GradARStart.backward."""

    @staticmethod
    def forward(ctx, x, box):
        ctx.box = box
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        box = ctx.box
        box.dx = g.contiguous()
        box.bwork = all_reduce(box.dx, box.group, async_op=True)
        return g, None


def grad_ar_start(x, group):
    """Megatron's f operator (identity forward, all-reduce of the gradient backward) split in
    two: ops created between ``grad_ar_start`` and :func:`grad_ar_finish` in the forward run, in
    the backward, while the gradient all-reduce is on the wire (it is launched at the finish
    node's backward and waited at the start node's)."""
    box = _Box()
    box.group = group
    return _GradARStart.apply(x, box), box


def grad_ar_finish(handle):
    y, box = handle
    return _GradARFinish.apply(y, box)


__all__ = ["launch_stream", "alloc_for_launch", "grad_ar_start", "grad_ar_finish", "ProxyGroup", "COMM_PRIORITY", "is_proxy", "group_rank_size", "backend", "all_reduce", "all_to_all_single",
           "all_to_all_counts", "a2a_start", "a2a_finish", "a2a", "ar_start", "ar_finish"]
