"""Shared timing harness for the per-model benchmarks under bench/ (same contract as the
root bench.py: W untimed warmup steps, K timed steps bracketed by barrier + device
sync on both sides, max elapsed over ranks, one JSON line from rank 0)."""
from __future__ import annotations

import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from solvingpapers_amd.parallel import dist as sdist  # noqa: E402

PEAK_BF16 = 2.5e15


def timed(step, steps, warmup):
    for _ in range(warmup):
        step()
    sdist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    sdist.barrier()
    return sdist.all_reduce_max(time.perf_counter() - t0)


def report(metric, value, unit, steps, warmup, elapsed, config, **extra):
    info = sdist.info()
    if info.is_main:
        out = {"metric": metric, "value": round(value, 2), "unit": unit, "n_gpus": info.world_size,
               "steps": steps, "warmup": warmup, "ms_per_step": round(elapsed / steps * 1e3, 3),
               "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "bf16",
               "data": "synthetic (random token ids / images, random-init weights)", "config": config}
        out.update(extra)
        if torch.cuda.is_available():
            out["mem_gb"] = round(torch.cuda.max_memory_allocated() / 1e9, 1)
            free, total = torch.cuda.mem_get_info()     # device-wide: RCCL / hipBLASLt buffers included
            out["dev_mem_used_gb"] = round((total - free) / 1e9, 1)
        print(json.dumps(out), flush=True)
