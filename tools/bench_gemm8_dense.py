"""The 8-phase bf16 kernel (gemm8.hip) as ONE dense GEMM (E = 1) against hipBLASLt, on random
operands: separates the core loop from grouping overheads, and gives rocprofv3 --pmc a short
program whose dispatches are just these GEMMs.
    python tools/bench_gemm8_dense.py [S] [--iters N] [--modes 0,1,2]"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from solvingpapers_amd.ops import _ext

ap = argparse.ArgumentParser()
ap.add_argument("S", type=int, nargs="?", default=8192)
ap.add_argument("--iters", type=int, default=20)
ap.add_argument("--modes", default="0,1,2")
ap.add_argument("--no-blas", action="store_true")
a = ap.parse_args()
ops = _ext.ops()
S = a.S
dev = "cuda"
off1 = torch.tensor([0, S], dtype=torch.int32, device=dev)
xa = torch.rand(S, S, device=dev).sub_(0.5).bfloat16()
wb = torch.rand(1, S, S, device=dev).sub_(0.5).bfloat16()
fl = 2.0 * S ** 3


def tm(fn):
    w0 = time.perf_counter()
    while time.perf_counter() - w0 < 0.3:        # clock ramp
        fn()
        torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(a.iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / a.iters


ref = torch.mm(xa, wb[0].t()).float()
for mode in [int(m) for m in a.modes.split(",")]:
    bb = wb if mode < 2 else xa
    out = ops.grouped_gemm8(xa, bb, off1, mode, None, False)
    r = {0: ref, 1: None, 2: None}[mode]
    err = ((out.float() - r).norm() / r.norm()).item() if r is not None else float("nan")
    ms = tm(lambda: ops.grouped_gemm8(xa, bb, off1, mode, None, False))
    print(f"gemm8 mode{mode} {S}^3: {ms:.3f} ms {fl / ms / 1e9:.0f} TF (rel err vs hipBLASLt {err:.1e})", flush=True)
if not a.no_blas:
    ms = tm(lambda: torch.mm(xa, wb[0].t()))
    print(f"hipBLASLt NT {S}^3: {ms:.3f} ms {fl / ms / 1e9:.0f} TF", flush=True)
