"""Data parallelism over RCCL with per-layer gradient buckets overlapped with backward.

Replaces the reference's single-process ``nn.DataParallel`` over 2xT4
(deepseekv3/deepseekv3.ipynb:1709-1711, 2345-2346), which broadcast all
parameters every forward (~578 MB), gathered logits onto cuda:0 (~206 MB) and
reduced gradients onto cuda:0. Here:

* one process per GPU; parameters stay resident (no per-step broadcast);
* loss is local; only gradients move;
* gradient buckets are contiguous slices of the FlatParams gradient buffer, one
  per transformer layer (LLaMA3-8B: ~436 MB bf16 each — large messages that run
  RCCL near its xGMI ring bandwidth), launched asynchronously from a
  GradReadyMarker the moment the layer's backward finishes, so all-reduce of
  layer i overlaps the backward GEMMs of layers i-1..0;
* ``zero1=True`` switches each bucket to reduce-scatter, shards AdamW state
  across ranks (optimizer memory/compute / N) and all-gathers updated params;
* ``reduce="a2a"`` (default for bf16 gradient buffers; SPA_DP_REDUCE=ring|a2a): a bucket's
  reduce-scatter is ONE all-to-all -- every rank receives the N bf16 copies of its shard straight
  from the N-1 peers, which on the xGMI full mesh uses all 7 links at once -- followed by an fp32
  sum of the copies on the device (``spa::shard_sum_``, one bf16 rounding) and, without ZeRO-1, an
  all-gather. The wire bytes equal a ring all-reduce's (2(N-1)/N of the bucket per rank), but a
  ring's reduce-scatter rounds its running bf16 partial at every hop: N-1 = 7 roundings at N = 8,
  2.2x one bf16 rounding of the exact average on LLaMA-8B gradients vs 1.0x here
  (tools/grad_precision.py --mode ring, profiles/r6_dp_reduce_numerics.txt). The reference
  reduces fp32 gradients (deepseekv3/deepseekv3.ipynb:2427). ``reduce="ring"``: RCCL all-reduce /
  reduce-scatter (ReduceOp.AVG);
* expert-parallel buckets (every param tagged ``expert_parallel``) hold different
  experts on each EP rank and already contain the gradient contributions of every
  rank's tokens (the all-to-all backward brought them home): they are summed only
  over ``expert_dp_group`` (ranks holding the same experts, None = no replicas) and
  scaled by 1/world so the objective is the same mean-over-ranks as dense params.
"""
from __future__ import annotations

import os
from contextlib import contextmanager
from typing import List, Optional

import torch
import torch.distributed as dist

from ..utils.flat import FlatParams


class DataParallel:
    def __init__(self, model: torch.nn.Module, flat: FlatParams, group=None, zero1: bool = False,
                 expert_dp_group=None, reduce: Optional[str] = None):
        self.model = model
        self.expert_dp_group = expert_dp_group
        self.expert_buckets = {b.index for b in flat.buckets
                               if b.params and all(getattr(p, "expert_parallel", False) for p in b.params)}
        assert not (zero1 and self.expert_buckets), "ZeRO-1 with expert-parallel buckets is not supported"
        self.flat = flat
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.zero1 = zero1
        self.backend = dist.get_backend(group) if dist.is_initialized() else "none"
        self._sync = True
        self._launched = set()
        self._works: List = []
        self._avg_after: List[torch.Tensor] = []
        from .dist import force_collectives
        # the collective paths run at world > 1, or at world 1 under SPA_FORCE_COLLECTIVES (tests)
        self.active = self.world > 1 or (dist.is_initialized() and force_collectives())
        if reduce is None:
            reduce = os.environ.get("SPA_DP_REDUCE") or ("a2a" if flat.grad.dtype == torch.bfloat16 else "ring")
        assert reduce in ("a2a", "ring"), reduce
        self.reduce = reduce
        self._keep: List[torch.Tensor] = []       # a2a receive buffers (CPU / gloo path)
        self._rstream = torch.cuda.Stream(device=flat.grad.device) \
            if (self.active and reduce == "a2a" and flat.grad.is_cuda) else None
        if self.active:
            model.grad_ready_cb = self._on_ready
            for b in flat.buckets:
                assert b.numel % self.world == 0, "FlatParams align must be a multiple of world size"

    # ---------------------------------------------------------------- sharding
    def shard_ranges(self):
        """This rank's ZeRO-1 slice of every bucket."""
        out = []
        for b in self.flat.buckets:
            n = b.numel // self.world
            out.append((b.start + self.rank * n, b.start + (self.rank + 1) * n))
        return out

    # ------------------------------------------------------------------ comms
    def _reduce_bucket(self, idx: int):
        if idx in self._launched or idx >= len(self.flat.buckets):
            return
        self._launched.add(idx)
        b = self.flat.buckets[idx]
        g = self.flat.grad[b.start:b.end]
        if idx in self.expert_buckets:
            grp = self.expert_dp_group
            if grp is not None and dist.get_world_size(grp) > 1:
                self._works.append(dist.all_reduce(g, group=grp, async_op=True))
            self._avg_after.append((g, self.world))
            return
        group, world = self.group, self.world
        if self.reduce == "a2a":
            self._works.append(self._a2a_reduce(g, b.numel // world))
            return
        use_avg = self.backend == "nccl"
        op = dist.ReduceOp.AVG if use_avg else dist.ReduceOp.SUM
        if self.zero1:
            n = b.numel // self.world
            out = g[self.rank * n:(self.rank + 1) * n]
            w = dist.reduce_scatter_tensor(out, g, op=op, group=self.group, async_op=True)
            if not use_avg:
                self._avg_after.append((out, world))
        else:
            w = dist.all_reduce(g, op=op, group=group, async_op=True)
            if not use_avg:
                self._avg_after.append((g, world))
        self._works.append(w)

    def _a2a_reduce(self, g: torch.Tensor, n: int):
        """Reduce-scatter of bucket ``g`` as one all-to-all + an fp32 device sum of the N received
        shard copies (one rounding), then (no ZeRO-1) the in-place all-gather. On the GPU the three
        run on a side stream that first waits for the compute stream (the bucket's gradients are
        complete there); returns a handle whose wait() orders the caller's stream after them."""
        shard = g[self.rank * n:(self.rank + 1) * n]
        scale = 1.0 / self.world
        if self._rstream is None:                  # CPU / gloo
            recv = torch.empty_like(g)
            dist.all_to_all_single(recv, g, group=self.group)
            shard.copy_((recv.view(self.world, n).float().sum(0) * scale).to(g.dtype))
            if self.zero1:
                return _Done()
            return dist.all_gather_into_tensor(g, shard.clone(), group=self.group, async_op=True)
        from ..ops._ext import ops
        s = self._rstream
        s.wait_stream(torch.cuda.current_stream(g.device))
        with torch.cuda.stream(s):
            recv = torch.empty_like(g)             # allocated on s: reused only after s passes here
            w = dist.all_to_all_single(recv, g, group=self.group, async_op=True)
            w.wait()                               # s waits for the RCCL stream (no host block)
            ops().shard_sum_(shard, recv, self.world, scale)
            del recv
            if self.zero1:
                ev = torch.cuda.Event()
                ev.record(s)
                return _EventWork(ev)
            # in place: the input is this rank's slice of the output (RCCL's in-place all-gather)
            return dist.all_gather_into_tensor(g, shard, group=self.group, async_op=True)

    def _on_ready(self, key):
        if self._sync and self.active:
            self._reduce_bucket(int(key))

    @contextmanager
    def no_sync(self):
        """Gradient accumulation: skip communication for inner micro-batches."""
        prev = self._sync
        self._sync = False
        try:
            yield
        finally:
            self._sync = prev

    def finish_grad_sync(self):
        """Launch any bucket not yet launched (e.g. the embedding) and wait for all."""
        if not self.active:
            return
        for i in range(len(self.flat.buckets) - 1, -1, -1):
            self._reduce_bucket(i)
        for w in self._works:
            w.wait()
        for t, n in self._avg_after:
            t.div_(n)
        self._works.clear()
        self._avg_after.clear()
        self._launched.clear()

    def gather_params(self):
        """ZeRO-1: all-gather each bucket's updated parameter shards."""
        if not self.zero1 or not self.active:
            return
        works = []
        for b in self.flat.buckets:
            p = self.flat.param[b.start:b.end]
            n = b.numel // self.world
            works.append(dist.all_gather_into_tensor(p, p[self.rank * n:(self.rank + 1) * n].clone(),
                                                     group=self.group, async_op=True))
        for w in works:
            w.wait()
        _invalidate()

    def broadcast_params(self, src: int = 0):
        """Make every replica start from the same parameters: dense buckets from rank ``src``
        of the DP group (a group-local rank), expert-parallel buckets only over
        ``expert_dp_group`` -- each EP rank holds DIFFERENT experts, so broadcasting those
        over the whole DP group would overwrite every rank's experts with rank 0's."""
        if not self.active:
            return
        gsrc = dist.get_global_rank(self.group, src) if self.group is not None else src
        dense = [b for b in self.flat.buckets if b.index not in self.expert_buckets]
        if not self.expert_buckets:
            dist.broadcast(self.flat.param, src=gsrc, group=self.group)
        else:
            for b in dense:
                dist.broadcast(self.flat.param[b.start:b.end], src=gsrc, group=self.group)
            grp = self.expert_dp_group
            if grp is not None and dist.get_world_size(grp) > 1:
                esrc = dist.get_global_rank(grp, 0)
                for b in self.flat.buckets:
                    if b.index in self.expert_buckets:
                        dist.broadcast(self.flat.param[b.start:b.end], src=esrc, group=grp)
        _invalidate()


class _Done:
    def wait(self):
        return True


class _EventWork:
    """wait(): the current stream waits for the event (no host block), like an RCCL work's wait."""

    def __init__(self, ev):
        self.ev = ev

    def wait(self):
        torch.cuda.current_stream().wait_event(self.ev)
        return True


def _invalidate():
    """params were rewritten through the flat buffer: cached W^T / fp8 images are stale
    (ops/linear.py CONTRACT)."""
    from ..ops.linear import invalidate_weight_caches
    invalidate_weight_caches()
