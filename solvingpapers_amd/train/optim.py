"""Optimizers over :class:`~solvingpapers_amd.utils.flat.FlatParams`.

AdamW/Adam/SGD with bf16 params + fp32 master copy + fp32 moments, grad-norm
clipping via a device-resident coefficient (no host sync), optional ZeRO-1
(each rank updates only its shard of every bucket; see parallel/data_parallel.py).
Reference optimizers: gpt/gpt-jax.ipynb:600 (optax.adamw 3e-4, wd 0.01),
deepseekv3/deepseekv3.ipynb:2350-2356 (AdamW betas .9/.95 wd .1 eps 1e-8, clip 1.0),
llama3/LLaMA-jax.ipynb:993-1001 (plain SGD 3e-4).
"""
from __future__ import annotations

import math
from typing import List, Optional, Tuple

import torch

from ..ops import optim_kernels as K
from ..utils.flat import FlatParams

# priority of the overlapped optimizer's side stream (torch: 0 default, -1 high). SPA_OPT_PRIO
OPT_STREAM_PRIORITY = int(__import__("os").environ.get("SPA_OPT_PRIO", "0"))


class FlatOptimizer:
    def __init__(self, flat: FlatParams, lr: float, weight_decay: float = 0.0, max_grad_norm: Optional[float] = None,
                 shard: Optional[Tuple[List[Tuple[int, int]], object]] = None, ep_group=None, tp_group=None,
                 graph_safe: bool = False, skip_nonfinite: bool = True):
        self.flat = flat
        # skip_nonfinite: compute the global grad norm even without clipping so a non-finite
        # gradient skips the update on every rank alike (clip_coef). Cost: one extra
        # memory-bound pass over the gradients (sqsum, ~2 bytes/param) plus the norm's
        # all-reduces per optimizer step when no clipping was asked for.
        self.skip_nonfinite = skip_nonfinite
        # On the GPU lr and step live on the device ([lr, step] fp32): a skipped step (NaN
        # coefficient) then does not advance Adam's bias correction -- the step counter moves by
        # isfinite(coef) without a host sync -- and a captured HIP graph of the whole training
        # step replays with the right bias correction / schedule (set_lr). ``graph_safe`` is
        # kept for API compatibility; the device form is always used on the GPU.
        self.graph_safe = graph_safe
        self.hyper = (torch.tensor([lr, 0.0], dtype=torch.float32, device=flat.device)
                      if flat.device.type == "cuda" else None)
        self._host_steps = 0          # CPU: applied (finite) steps
        # tensor parallelism: params tagged ``tp_replicated`` are identical on every TP rank and
        # counted once; the squared norm of everything else is summed over the TP group
        self.tp_group = tp_group
        self.tp_rep_ranges = sorted((flat.offsets[id(p)], flat.offsets[id(p)] + p.numel())
                                    for b in flat.buckets for p in b.params if getattr(p, "tp_replicated", False))
        # expert-parallel buckets: their squared-norm partial is summed over the EP group
        self.ep_group = ep_group
        self.expert_ranges = [(b.start, b.end) for b in flat.buckets
                              if b.params and all(getattr(p, "expert_parallel", False) for p in b.params)]
        self.lr = lr
        self.weight_decay = weight_decay
        self.max_grad_norm = max_grad_norm
        self.step_count = 0
        # ranges of the flat buffer this optimizer owns (all, or this rank's ZeRO shard)
        self.ranges = shard[0] if shard else [(0, flat.numel)]
        self.sharded = shard is not None          # ZeRO-1: grad-norm partials summed over the DP group
        self.norm_group = shard[1] if shard else None
        self.use_master = flat.param_dtype != torch.float32
        self.last_grad_norm: Optional[torch.Tensor] = None
        # owned element count and per-range state offsets
        self.state_off = []
        o = 0
        for a, b in self.ranges:
            self.state_off.append(o)
            o += b - a
        self.state_numel = o
        self.master = None
        if self.use_master:
            self.master = torch.empty(o, dtype=torch.float32, device=flat.device)
            for (a, b), so in zip(self.ranges, self.state_off):
                self.master[so:so + b - a].copy_(flat.param[a:b].float())

    def _segments(self):
        """(flat_a, flat_b, state_a, decay, bucket) pieces = owned ranges x decay segments,
        in bucket (= forward) order."""
        out = []
        for (a, b), so in zip(self.ranges, self.state_off):
            for sa, sb, dec in self.flat.decay_segments:
                lo, hi = max(a, sa), min(b, sb)
                # split at bucket boundaries: one update (and one ready event) per bucket, so
                # an overlapped optimizer releases layer i's params as soon as they are done
                for bi, bk in enumerate(self.flat.buckets):
                    l2, h2 = max(lo, bk.start), min(hi, bk.end)
                    if l2 < h2:
                        out.append((l2, h2, so + l2 - a, dec, bi))
        out.sort(key=lambda x: x[0])
        return out

    def _run(self, lr, overlap: bool):
        """Apply self._update to every owned segment. With ``overlap`` (GPU), the
        updates run on a low-priority side stream, one event per bucket, so the
        memory-bound optimizer overlaps the compute-bound forward of the next
        step (see FlatParams.wait_bucket)."""
        self.step_count += 1
        from ..ops.moe import bump_weight_epoch
        bump_weight_epoch()                  # cached fp8 / W^T weight images go stale now
        coef = self.clip_coef()
        if self.hyper is not None:
            if not torch.cuda.is_current_stream_capturing():
                self.hyper[0].fill_(lr)
            if coef is None:
                self.hyper[1].add_(1.0)
            else:                            # a skipped (non-finite) step does not count
                self.hyper[1].add_(torch.isfinite(coef).to(torch.float32)[0])
        elif coef is None or bool(torch.isfinite(coef).all()):
            self._host_steps += 1
        segs = self._segments()
        if overlap and self.flat.device.type == "cuda":
            main = torch.cuda.current_stream(self.flat.device)
            if not hasattr(self, "_side"):
                self._side = torch.cuda.Stream(self.flat.device, priority=OPT_STREAM_PRIORITY)
            side = self._side
            side.wait_stream(main)
            if coef is not None:
                coef.record_stream(side)
            with torch.cuda.stream(side):
                last = None
                for a, b, so, dec, bi in segs:
                    if last is not None and bi != last:
                        ev = torch.cuda.Event()
                        ev.record(side)
                        self.flat.set_ready_event(last, ev)
                    self._update(a, b, so, dec, lr, coef)
                    last = bi
                if last is not None:
                    ev = torch.cuda.Event()
                    ev.record(side)
                    self.flat.set_ready_event(last, ev)
                # anything the model does not wait on explicitly (e.g. checkpoint
                # reads) is ordered by wait_all()
        else:
            for a, b, so, dec, bi in segs:
                self._update(a, b, so, dec, lr, coef)

    def grad_norm(self) -> torch.Tensor:
        """Global L2 norm of the (already reduced) gradient, on the device."""
        import torch.distributed as dist
        tot = None
        ex = None
        for a, b in self.ranges:
            if self.ep_group is not None and self.expert_ranges:
                # split the owned range into replicated / expert pieces
                for ea, eb in self.expert_ranges:
                    lo, hi = max(a, ea), min(b, eb)
                    if lo < hi:
                        s = K.sqsum(self.flat.grad[lo:hi])
                        ex = s if ex is None else ex + s
                pieces = _subtract([(a, b)], self.expert_ranges)
            else:
                pieces = [(a, b)]
            for lo, hi in pieces:
                s = K.sqsum(self.flat.grad[lo:hi])
                tot = s if tot is None else tot + s
        if tot is None:
            tot = torch.zeros((), dtype=torch.float32, device=self.flat.device)
        if self.tp_group is not None and dist.is_initialized() and dist.get_world_size(self.tp_group) > 1:
            rep = None
            for a, b in self.ranges:
                for ra, rb in self.tp_rep_ranges:
                    lo, hi = max(a, ra), min(b, rb)
                    if lo < hi:
                        s = K.sqsum(self.flat.grad[lo:hi])
                        rep = s if rep is None else rep + s
            sharded = tot - rep if rep is not None else tot
            dist.all_reduce(sharded, group=self.tp_group)
            tot = sharded + rep if rep is not None else sharded
        if self.sharded and dist.is_initialized():
            dist.all_reduce(tot, group=self.norm_group)
        if ex is not None:
            if dist.is_initialized():
                dist.all_reduce(ex, group=self.ep_group)
            tot = tot + ex
        return tot.sqrt()

    def clip_coef(self):
        """Device-resident update coefficient: the clip factor, or NaN when the global grad
        norm is not finite -- the fused kernels then skip the update. The norm is already
        reduced over every DP/ZeRO/TP/EP group, so every rank reaches the same skip decision
        with no host sync and no mismatched collectives (a rank-local loss check would
        desynchronise the ranks)."""
        if self.max_grad_norm is None and not self.skip_nonfinite:
            self.last_grad_norm = None
            return None
        n = self.grad_norm()
        self.last_grad_norm = n
        nan = torch.full_like(n, float("nan"))
        if self.max_grad_norm is None:
            c = torch.where(torch.isfinite(n), torch.ones_like(n), nan)
        else:
            c = torch.where(torch.isfinite(n), torch.clamp(self.max_grad_norm / (n + 1e-6), max=1.0), nan)
        return c.float().reshape(1)

    def last_step_ok(self):
        """Device bool: did the last step apply an update (finite global grad norm)?"""
        if self.last_grad_norm is None:
            return None
        return torch.isfinite(self.last_grad_norm)

    def zero_grad(self):
        from ..utils.grad import next_generation
        next_generation()

    def set_lr(self, lr: float):
        """Update the learning rate (also for an already captured graph_safe step)."""
        self.lr = lr
        if self.hyper is not None:
            self.hyper[0].fill_(lr)

    def device_step(self) -> int:
        """Applied optimizer steps (skipped non-finite steps excluded)."""
        return int(self.hyper[1].item()) if self.hyper is not None else self._host_steps

    def _kstep(self) -> int:
        """host step handed to the kernels (ignored on the GPU, where hyper[1] is used)."""
        return self.step_count if self.hyper is not None else max(1, self._host_steps)


def _subtract(ranges, holes):
    out = []
    for a, b in ranges:
        cur = a
        for ha, hb in sorted(holes):
            if hb <= cur or ha >= b:
                continue
            if ha > cur:
                out.append((cur, ha))
            cur = max(cur, hb)
        if cur < b:
            out.append((cur, b))
    return out


class FlatAdamW(FlatOptimizer):
    def __init__(self, flat, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.01, max_grad_norm=None,
                 adam_l2=False, shard=None, ep_group=None, tp_group=None, graph_safe=False,
                 moment_dtype=torch.float32):
        """moment_dtype bf16: the DeepSeek-V3 recipe (moments in BF16, fp32 master weights;
        arXiv 2412.19437 sec. 3.3.2) -- needs an fp32 master (low-precision params)."""
        super().__init__(flat, lr, weight_decay, max_grad_norm, shard, ep_group, tp_group, graph_safe)
        self.b1, self.b2 = betas
        self.eps = eps
        self.adam_l2 = adam_l2
        if moment_dtype != torch.float32 and self.master is None:
            moment_dtype = torch.float32      # fp32 params: keep the moments at their precision
        self.m = torch.zeros(self.state_numel, dtype=moment_dtype, device=flat.device)
        self.v = torch.zeros(self.state_numel, dtype=moment_dtype, device=flat.device)

    @torch.no_grad()
    def step(self, lr: Optional[float] = None, overlap: bool = False):
        self._run(self.lr if lr is None else lr, overlap)

    def _update(self, a, b, so, dec, lr, coef):
        f = self.flat
        n = b - a
        K.adamw_(f.param[a:b], self.master[so:so + n] if self.master is not None else None, f.grad[a:b],
                 self.m[so:so + n], self.v[so:so + n], lr, self.b1, self.b2, self.eps,
                 self.weight_decay if dec else 0.0, self._kstep(), coef, self.adam_l2, self.hyper)

    def state_dict(self):
        return {"step": self.device_step(), "m": self.m, "v": self.v, "master": self.master, "lr": self.lr}

    def load_state_dict(self, sd):
        self.step_count = self._host_steps = int(sd["step"])
        if self.hyper is not None:
            self.hyper[1].fill_(float(self.step_count))
        self.m.copy_(sd["m"])
        self.v.copy_(sd["v"])
        if self.master is not None and sd.get("master") is not None:
            self.master.copy_(sd["master"])


def FlatAdam(flat, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, max_grad_norm=None, shard=None):
    """torch.optim.Adam semantics (L2 weight decay folded into the gradient)."""
    return FlatAdamW(flat, lr, betas, eps, weight_decay, max_grad_norm, adam_l2=True, shard=shard)


class FlatSGD(FlatOptimizer):
    def __init__(self, flat, lr=1e-3, momentum=0.0, weight_decay=0.0, max_grad_norm=None, shard=None,
                 graph_safe=False, ep_group=None, tp_group=None):
        super().__init__(flat, lr, weight_decay, max_grad_norm, shard, ep_group, tp_group, graph_safe=graph_safe)
        self.momentum = momentum
        self.buf = torch.zeros(self.state_numel, dtype=torch.float32, device=flat.device) if momentum else None

    @torch.no_grad()
    def step(self, lr: Optional[float] = None, overlap: bool = False):
        self._run(self.lr if lr is None else lr, overlap)

    def _update(self, a, b, so, dec, lr, coef):
        f = self.flat
        n = b - a
        K.sgd_(f.param[a:b], self.master[so:so + n] if self.master is not None else None, f.grad[a:b],
               self.buf[so:so + n] if self.buf is not None else None, lr, self.momentum,
               self.weight_decay if dec else 0.0, coef, self.hyper)

    def state_dict(self):
        return {"step": self.device_step(), "buf": self.buf, "master": self.master, "lr": self.lr}

    def load_state_dict(self, sd):
        self.step_count = self._host_steps = int(sd["step"])
        if self.hyper is not None:
            self.hyper[1].fill_(float(self.step_count))
        if self.buf is not None and sd.get("buf") is not None:
            self.buf.copy_(sd["buf"])
        if self.master is not None and sd.get("master") is not None:
            self.master.copy_(sd["master"])


def cosine_lr(step, max_lr, warmup, total, min_lr):
    """deepseekv3/deepseekv3.ipynb:1976-1986: linear warmup max_lr*(s+1)/(warmup+1) -> cosine -> min_lr."""
    if step < warmup:
        return max_lr * (step + 1) / (warmup + 1)
    if step > total:
        return min_lr
    r = (step - warmup) / max(1, total - warmup)
    return min_lr + 0.5 * (1.0 + math.cos(math.pi * r)) * (max_lr - min_lr)
