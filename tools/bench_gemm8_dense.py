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
ap.add_argument("--ab", type=int, default=None, help="also run SPA_GG8_ABLATE=<v> (ABBA, same process) and "
                "the dsv3_style grouped shapes")
ap.add_argument("--abenv", default=None, help="NAME=VALUE: the ABBA arm sets this variable instead (e.g. SPA_G8W=0)")
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


def arm(v):
    if a.abenv:
        k, val = a.abenv.split("=")
        if v == 0:
            os.environ.pop(k, None)
        else:
            os.environ[k] = val
    else:
        os.environ["SPA_GG8_ABLATE"] = str(v)


if a.abenv and a.ab is None:
    a.ab = 1
if a.ab is not None:
    from solvingpapers_amd.ops import moe as M
    torch.manual_seed(0)
    T, E, k, D, F = 8192, 64, 6, 2048, 1408
    idx, _ = M.route(torch.randn(T, E, device=dev), k)
    plan = M.permute(idx, E)
    A = T * k
    x = torch.randn(A, D, device=dev, dtype=torch.bfloat16)
    W13 = torch.randn(E, 2 * F, D, device=dev, dtype=torch.bfloat16) * 0.02
    W2 = torch.randn(E, D, F, device=dev, dtype=torch.bfloat16) * 0.02
    h = torch.randn(A, F, device=dev, dtype=torch.bfloat16)
    dy13 = torch.randn(A, 2 * F, device=dev, dtype=torch.bfloat16)
    dy2 = torch.randn(A, D, device=dev, dtype=torch.bfloat16)
    # skewed routing (per-expert logit offsets, as an untrained router produces): a few hot experts
    idx_s, _ = M.route(torch.randn(T, E, device=dev) + 1.5 * torch.randn(E, device=dev), k)
    plan_s = M.permute(idx_s, E)
    cnt = plan_s.counts.float()
    print(f"skewed routing: max/mean tokens per expert {cnt.max().item() / cnt.mean().item():.2f}", flush=True)
    cases = {"dense mode0": (lambda: ops.grouped_gemm8(xa, wb, off1, 0, None, False), fl),
             "dense mode1": (lambda: ops.grouped_gemm8(xa, wb, off1, 1, None, False), fl),
             "dense mode2": (lambda: ops.grouped_gemm8(xa, xa, off1, 2, None, False), fl),
             "fwd W13": (lambda: ops.grouped_gemm8(x, W13, plan.offsets, 0, None, False), 2 * A * 2 * F * D),
             "fwd W2": (lambda: ops.grouped_gemm8(h, W2, plan.offsets, 0, None, False), 2 * A * D * F),
             "dX W13": (lambda: ops.grouped_gemm8(dy13, W13, plan.offsets, 1, None, False), 2 * A * 2 * F * D),
             "dX W2": (lambda: ops.grouped_gemm8(dy2, W2, plan.offsets, 1, None, False), 2 * A * D * F),
             "dW W13": (lambda: ops.grouped_gemm8(dy13, x, plan.offsets, 2, None, False), 2 * A * 2 * F * D),
             "dW W2": (lambda: ops.grouped_gemm8(dy2, h, plan.offsets, 2, None, False), 2 * A * D * F),
             "dW W13 skew": (lambda: ops.grouped_gemm8(dy13, x, plan_s.offsets, 2, None, False), 2 * A * 2 * F * D),
             "dW W2 skew": (lambda: ops.grouped_gemm8(dy2, h, plan_s.offsets, 2, None, False), 2 * A * D * F),
             "dX W13 skew": (lambda: ops.grouped_gemm8(dy13, W13, plan_s.offsets, 1, None, False), 2 * A * 2 * F * D)}
    for name, (fn, f) in cases.items():
        arm(0); r0 = fn().float()
        arm(a.ab); r1 = fn().float()
        same = torch.equal(r0, r1)
        t = {0: [], a.ab: []}
        for v in (0, a.ab, a.ab, 0):
            arm(v)
            t[v].append(tm(fn))
        m0, m1 = sum(t[0]) / 2, sum(t[a.ab]) / 2
        rel = ((r0 - r1).norm() / r1.norm().clamp_min(1e-30)).item()
        print(f"{name:12s} default {f / m0 / 1e9:6.0f} TF | {a.abenv or 'sched %d' % a.ab} {f / m1 / 1e9:6.0f} TF "
              f"({m0 / m1:.3f}x) bitwise-equal {same} rel {rel:.1e}", flush=True)
    arm(0)
    sys.exit(0)
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
