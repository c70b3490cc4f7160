"""Grouped GEMM time vs the per-expert row counts at dsv3_style widths (E 64, 8192 x 6 rows, D 2048 ->
2F 2816): the routed counts of M.route, perfectly balanced counts (768 = 3 x 256 each), and counts whose
remainders past a multiple of 256 are all tiny. A 256-row tile is paid in full for a 3-row remainder.
    python tools/bench_gg_counts.py [--iters N]"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from solvingpapers_amd.ops import _ext
from solvingpapers_amd.ops import moe as M

ap = argparse.ArgumentParser()
ap.add_argument("--iters", type=int, default=20)
ap.add_argument("--env", default="", help="NAME=V: a second arm with this env var set (read at op call)")
a = ap.parse_args()
ops = _ext.ops()
dev = "cuda"


def tm(fn):
    w0 = time.perf_counter()
    while time.perf_counter() - w0 < 0.2:
        fn()
        torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(a.iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / a.iters


def rel(x, y):
    return ((x.float() - y.float()).norm() / y.float().norm()).item()


torch.manual_seed(0)
T, E, k, D, F = 8192, 64, 6, 2048, 1408
A = T * k
idx, _ = M.route(torch.randn(T, E, device=dev), k)
routed = torch.bincount(idx.reshape(-1).long(), minlength=E).cpu()
g = torch.Generator().manual_seed(1)
tiny = torch.full((E,), 768)
tiny[:32] += torch.randint(1, 48, (32,), generator=g)           # half the experts 1-47 rows past 768
tiny[32:] -= (tiny[:32].sum() - 768 * 32) // 32 + 1
tiny[-1] += A - int(tiny.sum())
sets = {"routed": routed, "balanced": torch.full((E,), 768), "tiny-rem": tiny}
xg = torch.randn(A, D, device=dev, dtype=torch.bfloat16)
dy = torch.randn(A, 2 * F, device=dev, dtype=torch.bfloat16)
W13 = torch.randn(E, 2 * F, D, device=dev, dtype=torch.bfloat16) * 0.02
fl = 2.0 * A * 2 * F * D
for name, c in sets.items():
    assert int(c.sum()) == A and int(c.min()) >= 0, name
    off = torch.cat([torch.zeros(1, dtype=torch.long), c.cumsum(0)]).to(torch.int32).to(dev)
    oc = off.tolist()
    rem = [x % 256 for x in c.tolist() if x % 256]
    tiles = sum((x + 255) // 256 for x in c.tolist())
    y = ops.grouped_gemm8(xg, W13, off, 0, None, False)
    ref = torch.cat([xg[oc[e]:oc[e + 1]].float() @ W13[e].float().t() for e in range(E)])
    dx = ops.grouped_gemm8(dy, W13, off, 1, None, False)
    refx = torch.cat([dy[oc[e]:oc[e + 1]].float() @ W13[e].float() for e in range(E)])
    line = (f"{name:9s} row tiles {tiles} (ideal {A / 256:.1f}), remainders <=64 rows: {sum(r <= 64 for r in rem)}, "
            f"rel fwd {rel(y, ref):.1e} dX {rel(dx, refx):.1e}")
    arms = [("", None)] + ([(a.env, a.env.split("=", 1))] if a.env else [])
    for lab, kv in arms:
        old = None
        if kv:
            old = os.environ.get(kv[0])
            os.environ[kv[0]] = kv[1]
        tf = tm(lambda: ops.grouped_gemm8(xg, W13, off, 0, None, False))
        tx = tm(lambda: ops.grouped_gemm8(dy, W13, off, 1, None, False))
        if kv:
            y2 = ops.grouped_gemm8(xg, W13, off, 0, None, False)
            x2 = ops.grouped_gemm8(dy, W13, off, 1, None, False)
            line += f" | {lab}: fwd rel {rel(y2, ref):.1e} dX rel {rel(x2, refx):.1e}"
            if old is None:
                del os.environ[kv[0]]
            else:
                os.environ[kv[0]] = old
        line += f" | {lab or 'default'} fwd {tf:.3f} ms {fl / tf / 1e9:.0f} TF, dX {tx:.3f} ms {fl / tx / 1e9:.0f} TF"
    print(line, flush=True)
