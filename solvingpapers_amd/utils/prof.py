"""Profiling hooks (SURVEY §5 'Tracing / profiling'; the reference has only tqdm bars).

* :func:`annotate` -- a roctx range (``torch.cuda.nvtx`` is roctx on ROCm builds) around a
  step phase, so ``rocprofv3 --marker-trace --kernel-trace`` attributes kernels to
  forward / backward / optimizer / comm. Off unless ``SPA_ROCTX=1`` or
  :func:`enable_markers` (a push/pop pair costs ~1 us of host time).
* :class:`PhaseTimer` -- device-side phase timing with HIP events (no host sync until
  :meth:`PhaseTimer.summary`), averaged over steps.
* Kernel counters (MFMA utilisation, LDS bank conflicts, HBM bytes) come from
  ``rocprofv3 --pmc`` runs: tools/gpu_tasks.sh (headline-pmc, kernels-pmc), summarised by tools/prof_summary.py.
"""
from __future__ import annotations

import contextlib
import os
from collections import defaultdict
from typing import Dict, List

import torch

_MARKERS = os.environ.get("SPA_ROCTX") == "1"


def enable_markers(on: bool = True):
    global _MARKERS
    _MARKERS = on


@contextlib.contextmanager
def annotate(name: str):
    if not _MARKERS or not torch.cuda.is_available():
        yield
        return
    torch.cuda.nvtx.range_push(name)
    try:
        yield
    finally:
        torch.cuda.nvtx.range_pop()


class PhaseTimer:
    """``with timer.phase("fwd"): ...`` records HIP events around the phase on the current
    stream; ``summary()`` synchronises once and returns mean milliseconds per phase."""

    def __init__(self, enabled: bool = True):
        self.enabled = enabled and torch.cuda.is_available()
        self._ev: Dict[str, List] = defaultdict(list)

    @contextlib.contextmanager
    def phase(self, name: str):
        with annotate(name):
            if not self.enabled:
                yield
                return
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            try:
                yield
            finally:
                b.record()
                self._ev[name].append((a, b))

    def summary(self) -> Dict[str, float]:
        if not self.enabled or not self._ev:
            return {}
        torch.cuda.synchronize()
        out = {k: sum(a.elapsed_time(b) for a, b in v) / len(v) for k, v in self._ev.items()}
        self._ev.clear()
        return out
