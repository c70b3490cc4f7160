"""HIP-graph capture of a whole training (or decode) step.

Small configs (the reference presets: 2-8 layers, d256-512, T128-256) are launch
bound: a step is hundreds of short kernels. ``StepGraph(step_fn)`` warms the step up
on a side stream (so lazy allocations / autotuning happen outside the capture),
captures one invocation with ``torch.cuda.graph`` (hipGraph under ROCm) and replays it
with a single launch per step.

Requirements the framework meets for capture: no host synchronisation inside the step
(device-resident grad-norm clip coefficient, MoE offsets on the device), optimizer lr /
step read from a device tensor (``FlatOptimizer(graph_safe=True)`` + ``set_lr``),
dropout seeds drawn by torch's capture-aware device generator, and static input
buffers (refill them in place between replays).
"""
from __future__ import annotations

from typing import Callable

import torch


class StepGraph:
    def __init__(self, fn: Callable[[], None], warmup: int = 2, pool=None):
        self.fn = fn
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(warmup):
                fn()
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph, pool=pool):
            fn()
        self.replays = 0

    def replay(self):
        self.graph.replay()
        self.replays += 1

    __call__ = replay
