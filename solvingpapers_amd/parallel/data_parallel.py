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
* expert-parallel buckets (every param tagged ``expert_parallel``) hold different
  experts on each EP rank and already contain the gradient contributions of every
  rank's tokens (the all-to-all backward brought them home): they are summed only
  over ``expert_dp_group`` (ranks holding the same experts, None = no replicas) and
  scaled by 1/world so the objective is the same mean-over-ranks as dense params.
"""
from __future__ import annotations

from contextlib import contextmanager
from typing import List, Optional

import torch
import torch.distributed as dist

from ..utils.flat import FlatParams


class DataParallel:
    def __init__(self, model: torch.nn.Module, flat: FlatParams, group=None, zero1: bool = False,
                 expert_dp_group=None):
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


def _invalidate():
    """params were rewritten through the flat buffer: cached W^T / fp8 images are stale
    (ops/linear.py CONTRACT)."""
    from ..ops.linear import invalidate_weight_caches
    invalidate_weight_caches()
