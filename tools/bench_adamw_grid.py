"""AdamW / grad-norm launch grid A/B in ONE process (same buffers, interleaved arms, several rounds):
the block count of the grid-stride optimizer kernels is read per call from SPA_ADAMW_GRID /
SPA_SQSUM_GRID, so arms differ only in the grid (separate processes also differ in where the
buffers land, which moved the fp32 case by 15 % between runs).
    python tools/bench_adamw_grid.py [--n 268435456] [--rounds 3] [--grids 256,512,1024,4096]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from solvingpapers_amd.ops import optim_kernels

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=1 << 28)
ap.add_argument("--rounds", type=int, default=3)
ap.add_argument("--iters", type=int, default=20)
ap.add_argument("--grids", default="256,512,1024,4096")
a = ap.parse_args()
dev = "cuda"
n = a.n
p = torch.zeros(n, device=dev, dtype=torch.bfloat16)
mst = torch.zeros(n, device=dev)
m32, v32 = torch.zeros(n, device=dev), torch.zeros(n, device=dev)
m16, v16 = torch.zeros(n, device=dev, dtype=torch.bfloat16), torch.zeros(n, device=dev, dtype=torch.bfloat16)
g = torch.full((n,), 1e-3, device=dev, dtype=torch.bfloat16)
cases = {
    "adamw_fp32mom": (lambda: optim_kernels.adamw_(p, mst, g, m32, v32, 3e-4, 0.9, 0.95, 1e-8, 0.1, 1), n * (2 + 2 + 24), "SPA_ADAMW_GRID"),
    "adamw_bf16mom": (lambda: optim_kernels.adamw_(p, mst, g, m16, v16, 3e-4, 0.9, 0.95, 1e-8, 0.1, 1), n * (2 + 2 + 8 + 8), "SPA_ADAMW_GRID"),
    "sqsum_bf16": (lambda: optim_kernels.sqsum(g), n * 2, "SPA_SQSUM_GRID"),
}


def tm(fn):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(a.iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / a.iters


grids = [int(x) for x in a.grids.split(",")]
res = {}
for r in range(a.rounds):
    for name, (fn, nbytes, env) in cases.items():
        line = []
        for gr in grids:
            os.environ[env] = str(gr)
            ms = tm(fn)
            res.setdefault((name, gr), []).append(nbytes / ms / 1e9)
            line.append(f"grid {gr}: {ms:.3f} ms {nbytes / ms / 1e9:.2f} TB/s")
        print(f"round {r} {name}: " + " | ".join(line), flush=True)
for (name, gr), v in sorted(res.items()):
    print(f"{name} grid {gr}: mean {sum(v) / len(v):.2f} TB/s over {len(v)} rounds", flush=True)
