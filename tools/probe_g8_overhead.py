"""Fixed per-tile cost of the 8-phase GEMM (gemm8.hip): one dense product with exactly one tile per
CU (M = N = 4096 -> 256 tiles of 256 x 256) timed at growing reduction depth K, so that
time(K) = fixed + K / 64 * per-K-tile; the intercept is what a tile pays besides its K-loop
(tile mapping, prologue DMA latency, epilogue, block launch). Modes 0 (fwd), 1 (dX), 2 (dW).
    python tools/probe_g8_overhead.py [--iters N]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from solvingpapers_amd.ops import _ext

ap = argparse.ArgumentParser()
ap.add_argument("--iters", type=int, default=30)
ap.add_argument("--mn", type=int, default=4096)
a = ap.parse_args()
ops = _ext.ops()
dev = "cuda"


def tm(fn):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(a.iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / a.iters * 1e3   # us


MN = a.mn
for mode in (0, 1, 2):
    xs, ys = [], []
    for K in (128, 256, 512, 1024, 2048, 4096):
        if mode == 2:   # dW [MN, MN] over K tokens
            A = torch.randn(K, MN, device=dev).bfloat16()
            Bm = torch.randn(K, MN, device=dev).bfloat16()
            off = torch.tensor([0, K], dtype=torch.int32, device=dev)
            fn = lambda: ops.grouped_gemm8(A, Bm, off, 2, None, False)
        else:
            A = torch.randn(MN, K, device=dev).bfloat16()
            W = torch.randn(1, MN, K, device=dev).bfloat16() if mode == 0 else torch.randn(1, K, MN, device=dev).bfloat16()
            off = torch.tensor([0, MN], dtype=torch.int32, device=dev)
            fn = lambda: ops.grouped_gemm8(A, W, off, mode, None, False)
        us = tm(fn)
        xs.append(K / 64)
        ys.append(us)
        print(f"mode {mode} MN {MN} K {K:5d}: {us:8.1f} us  {2 * MN * MN * K / us / 1e6:6.0f} TF", flush=True)
    n = len(xs)
    mx, my = sum(xs) / n, sum(ys) / n
    slope = sum((x - mx) * (y - my) for x, y in zip(xs, ys)) / sum((x - mx) ** 2 for x in xs)
    icpt = my - slope * mx
    print(f"mode {mode}: fixed {icpt:.2f} us per tile wave + {slope:.3f} us per K-tile "
          f"(steady {2 * MN * MN * 64 / slope / 1e6:.0f} TF)", flush=True)

# per-tile-wave cost at a fixed, dW-like depth (K = 768 tokens): waves = (MN / 256)^2 / 256
print("-- fixed K 768, growing tile count (slope = cost of one more wave of 256 tiles)", flush=True)
for mode in (0, 2):
    xs, ys = [], []
    for MN in (4096, 5888, 8192, 11520):
        K = 768
        if mode == 2:
            A = torch.randn(K, MN, device=dev).bfloat16()
            Bm = torch.randn(K, MN, device=dev).bfloat16()
            off = torch.tensor([0, K], dtype=torch.int32, device=dev)
            fn = lambda: ops.grouped_gemm8(A, Bm, off, 2, None, False)
        else:
            A = torch.randn(MN, K, device=dev).bfloat16()
            W = torch.randn(1, MN, K, device=dev).bfloat16()
            off = torch.tensor([0, MN], dtype=torch.int32, device=dev)
            fn = lambda: ops.grouped_gemm8(A, W, off, 0, None, False)
        us = tm(fn)
        waves = (MN // 256) ** 2 / 256
        xs.append(waves)
        ys.append(us)
        print(f"mode {mode} MN {MN:5d} K 768 waves {waves:5.2f}: {us:8.1f} us  {2 * MN * MN * K / us / 1e6:6.0f} TF", flush=True)
    n = len(xs)
    mx, my = sum(xs) / n, sum(ys) / n
    slope = sum((x - mx) * (y - my) for x, y in zip(xs, ys)) / sum((x - mx) ** 2 for x in xs)
    print(f"mode {mode}: {slope:.2f} us per wave of 256 tiles at K 768 (intercept {my - slope * mx:.2f} us)", flush=True)
