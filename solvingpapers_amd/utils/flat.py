"""Flat, resident parameter / gradient / optimizer-state buffers.

MI355X-first memory layout: all trainable parameters of a model live in ONE
contiguous buffer (in bucket order = reverse-backward order friendly layer
blocks), gradients in a second buffer with identical offsets. Consequences:

* the fused optimizer is one kernel launch per contiguous weight-decay segment;
* a DP gradient bucket is a contiguous slice -> one RCCL all-reduce / reduce-scatter
  per bucket with no packing copies;
* ZeRO-1 shards are contiguous slices of every bucket;
* checkpoints are a handful of large tensors.

Sized for 288 GB HBM3E: LLaMA3-8B keeps 16 GB bf16 params + 16 GB bf16 grads +
32 GB fp32 master + 64 GB Adam moments resident on every GPU.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Callable, Iterable, List, Optional, Sequence

import torch


@dataclass
class Bucket:
    index: int
    start: int
    end: int
    params: List[torch.nn.Parameter] = field(default_factory=list)

    @property
    def numel(self):
        return self.end - self.start


class FlatParams:
    """Owns the flat param/grad buffers of ``module``.

    ``groups``: optional list of lists of parameters giving the bucket order
    (e.g. [[embedding], [layer0 params], ..., [final norm, lm_head]]); any
    parameter not listed goes to a trailing bucket. ``align`` pads every bucket
    to a multiple of ``align`` elements (for equal ZeRO shards / 16-byte vectors).
    """

    def __init__(self, module: torch.nn.Module, groups: Optional[Sequence[Sequence[torch.nn.Parameter]]] = None,
                 param_dtype: Optional[torch.dtype] = None, grad_dtype: Optional[torch.dtype] = None,
                 device=None, align: int = 64, no_decay: Optional[Callable[[str, torch.nn.Parameter], bool]] = None,
                 hook_autograd: bool = True):
        params = [p for p in module.parameters() if p.requires_grad]
        names = {id(p): n for n, p in module.named_parameters()}
        seen = set()
        ordered: List[List[torch.nn.Parameter]] = []
        for g in (groups or []):
            lst = []
            for p in g:
                if p.requires_grad and id(p) not in seen:
                    seen.add(id(p))
                    lst.append(p)
            if lst:
                ordered.append(lst)
        rest = [p for p in params if id(p) not in seen]
        if rest:
            ordered.append(rest)
        if not ordered:
            raise ValueError("FlatParams: module has no trainable parameters")
        dev = device if device is not None else params[0].device
        pdt = param_dtype or params[0].dtype
        gdt = grad_dtype or pdt
        self.device, self.param_dtype, self.grad_dtype = torch.device(dev), pdt, gdt
        self.buckets: List[Bucket] = []
        self.offsets = {}
        off = 0
        for bi, lst in enumerate(ordered):
            start = off
            for p in lst:
                self.offsets[id(p)] = off
                off += p.numel()
                off = (off + 7) // 8 * 8  # 16-byte aligned starts for vector kernels
            off = (off + align - 1) // align * align
            self.buckets.append(Bucket(bi, start, off, lst))
        self.numel = off
        self.params = [p for lst in ordered for p in lst]
        self.names = [names.get(id(p), f"param{i}") for i, p in enumerate(self.params)]
        self.param = torch.zeros(off, dtype=pdt, device=dev)
        self.grad = torch.zeros(off, dtype=gdt, device=dev)
        for p in self.params:
            o = self.offsets[id(p)]
            n = p.numel()
            view = self.param[o:o + n].view(p.shape)
            view.copy_(p.data.to(dev, pdt))
            p.data = view
            p.main_grad = self.grad[o:o + n].view(p.shape)
            p._spa_gen = -1
        # weight-decay segments: maximal runs of params with equal decay flag
        nd = no_decay or (lambda n, p: False)
        segs = []
        for name, p in zip(self.names, self.params):
            o = self.offsets[id(p)]
            flag = not nd(name, p)
            if segs and segs[-1][2] == flag:
                segs[-1][1] = o + p.numel()
            else:
                segs.append([o, o + p.numel(), flag])
        self.decay_segments = [(a, b, f) for a, b, f in segs]
        if hook_autograd:
            attach_autograd_grads(self)

    # ---- overlap of the optimizer step with the next forward -----------------
    # The optimizer may update buckets on a side stream, recording one event per
    # bucket; the model calls wait_bucket(i) right before it first reads bucket
    # i's parameters, so the update of layer i overlaps the forward of layers < i.
    def set_ready_event(self, idx: int, ev):
        if not hasattr(self, "_ready"):
            self._ready = {}
        self._ready[idx] = ev

    def wait_bucket(self, idx: int):
        r = getattr(self, "_ready", None)
        if r:
            ev = r.pop(idx, None)
            if ev is not None:
                torch.cuda.current_stream(self.device).wait_event(ev)

    def wait_all(self):
        r = getattr(self, "_ready", None)
        if r:
            for idx in list(r):
                self.wait_bucket(idx)

    def group_waiter(self, groups: Sequence[Sequence[torch.nn.Parameter]]) -> Callable[[int], None]:
        """``wait(i)`` for a model that numbers its waits by its param_groups() index i: waits for
        the bucket that holds group i's parameters. FlatParams drops empty / frozen groups and
        appends a trailing bucket for unlisted params, so group index != bucket index in general;
        the map is taken from where each group's parameters actually landed."""
        table = []
        for g in groups:
            bs = sorted({self.bucket_of(p).index for p in g if id(p) in self.offsets})
            table.append(bs)

        def wait(i: int):
            if 0 <= i < len(table):
                for b in table[i]:
                    self.wait_bucket(b)
        wait.table = table
        return wait

    def bucket_of(self, p) -> Bucket:
        o = self.offsets[id(p)]
        for b in self.buckets:
            if b.start <= o < b.end:
                return b
        raise KeyError

    def zero_grad(self):
        self.grad.zero_()

    def param_view(self, p):
        o = self.offsets[id(p)]
        return self.param[o:o + p.numel()]

    def state_dict(self):
        return {"param": self.param, "names": self.names,
                "offsets": [self.offsets[id(p)] for p in self.params],
                "shapes": [tuple(p.shape) for p in self.params]}


def attach_autograd_grads(flat: "FlatParams"):
    """Route gradients that arrive through plain autograd (parameters used by
    non-fused torch ops) into ``main_grad`` as soon as they are accumulated, then
    drop ``.grad`` so no second copy stays alive. Idempotent."""
    from .grad import commit_tensor

    def _hook(p):
        if p.grad is not None:
            commit_tensor(p, p.grad)
            p.grad = None

    for p in flat.params:
        if not getattr(p, "_spa_hooked", False):
            p.register_post_accumulate_grad_hook(_hook)
            p._spa_hooked = True
