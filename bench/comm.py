#!/usr/bin/env python
"""RCCL collective bandwidth over xGMI: all-reduce, reduce-scatter, all-gather, all-to-all
for 1 MiB .. 1 GiB bf16 messages (nccl-tests conventions: algbw = bytes / time,
busbw = algbw x 2(n-1)/n for all-reduce, (n-1)/n for the others). One JSON line per
(op, size) from rank 0. ``torchrun --nproc-per-node N --master-addr 127.0.0.1 bench/comm.py``"""
from __future__ import annotations

import argparse
import json
import time

import torch
import torch.distributed as dist

from common import sdist


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--min-mb", type=float, default=1)
    ap.add_argument("--max-mb", type=float, default=1024)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    info = sdist.init_distributed()
    n, dev = info.world_size, info.device
    mb = a.min_mb
    while mb <= a.max_mb:
        numel = int(mb * 2 ** 20 // 2) // n * n
        x = torch.randn(numel, device=dev, dtype=torch.bfloat16)
        out_full = torch.empty_like(x)
        shard = torch.empty(numel // n, device=dev, dtype=torch.bfloat16)
        ops = {
            "all_reduce": (lambda: dist.all_reduce(x), 2 * (n - 1) / n),
            "reduce_scatter": (lambda: dist.reduce_scatter_tensor(shard, x), (n - 1) / n),
            "all_gather": (lambda: dist.all_gather_into_tensor(out_full, shard), (n - 1) / n),
            "all_to_all": (lambda: dist.all_to_all_single(out_full, x), (n - 1) / n),
        }
        for name, (fn, f) in ops.items():
            if n == 1:
                break
            fn()
            torch.cuda.synchronize()
            dist.barrier()
            t0 = time.perf_counter()
            for _ in range(a.iters):
                fn()
            torch.cuda.synchronize()
            dt = sdist.all_reduce_max((time.perf_counter() - t0) / a.iters)
            if info.is_main:
                alg = numel * 2 / dt / 1e9
                print(json.dumps({"op": name, "bytes": numel * 2, "n_gpus": n, "ms": round(dt * 1e3, 3),
                                  "algbw_GBs": round(alg, 1), "busbw_GBs": round(alg * f, 1)}), flush=True)
        mb *= 4
    sdist.cleanup()


if __name__ == "__main__":
    main()
