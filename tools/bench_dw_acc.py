"""Expert dW (grouped mode 2, gemm4r by default) at dsv3_style widths with routed token counts, with
and without accumulation into the existing gradient (the accum > 1 micro-batches), one process per
extension build: run it once per SPA_EXT_SO in B N N B order to A/B an epilogue change.
    python tools/bench_dw_acc.py [--iters N]"""
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


torch.manual_seed(0)
T, E, k, D, F = 8192, 64, 6, 2048, 1408
idx, _ = M.route(torch.randn(T, E, device=dev), k)
offs = M.permute(idx, E).offsets.to(torch.int32)
A = T * k
oc = offs.tolist()
xg = torch.randn(A, D, device=dev, dtype=torch.bfloat16)
h = torch.randn(A, F, device=dev, dtype=torch.bfloat16)
dy13 = torch.randn(A, 2 * F, device=dev, dtype=torch.bfloat16)
dy2 = torch.randn(A, D, device=dev, dtype=torch.bfloat16)
res = []
for name, dy, xx in (("W13 dW [64 x 2816 x 2048]", dy13, xg), ("W2 dW [64 x 2048 x 1408]", dy2, h)):
    ref = torch.stack([dy[oc[e]:oc[e + 1]].float().t() @ xx[oc[e]:oc[e + 1]].float() for e in range(E)])
    g = torch.randn(ref.shape, device=dev).bfloat16()
    g0 = g.clone()
    ops.gemm4a(dy, xx, offs, 2, g, True)
    err = ((g.float() - g0.float() - ref).norm() / ref.norm()).item()
    assert err < 1e-2, err
    fl = 2.0 * A * dy.shape[1] * xx.shape[1]
    t0 = tm(lambda: ops.gemm4a(dy, xx, offs, 2, g, False))
    t1 = tm(lambda: ops.gemm4a(dy, xx, offs, 2, g, True))
    res.append(f"{name}: write {t0:.3f} ms {fl / t0 / 1e9:.0f} TF | accumulate {t1:.3f} ms {fl / t1 / 1e9:.0f} TF (rel {err:.1e})")
print(f"[{os.environ.get('SPA_EXT_SO', 'tree')}] " + " || ".join(res), flush=True)
