"""ViT-B/16 step GEMMs (T = 256 x 197 = 50432 tokens, D 768, MLP 3072): hipBLASLt with the ViT table
(tuning/tunableop_vit_b16.csv) against our gemm4a (dense = one-expert grouped GEMM, gemm4d pipeline)
and gemm8, forward (X W^T) and data-gradient (dY W) forms, same process, interleaved rounds.
    python tools/bench_vit_gemms.py [--iters N] [--rounds R]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from solvingpapers_amd.ops import _ext
from solvingpapers_amd.utils.tuning import load_gemm_tuning

ap = argparse.ArgumentParser()
ap.add_argument("--iters", type=int, default=20)
ap.add_argument("--rounds", type=int, default=2)
a = ap.parse_args()
dev = "cuda"
ops = _ext.ops()
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
print("vit table loaded:", load_gemm_tuning(os.path.join(root, "tuning", "tunableop_vit_b16.csv")), flush=True)


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


T = 256 * 197
shapes = [("qkv", 768, 2304), ("proj", 768, 768), ("fc1", 768, 3072), ("fc2", 3072, 768)]
off = torch.tensor([0, T], dtype=torch.int32, device=dev)
cases = []
for name, K, N in shapes:
    x = torch.randn(T, K, device=dev, dtype=torch.bfloat16)
    w = torch.randn(1, N, K, device=dev, dtype=torch.bfloat16) * K ** -0.5
    dy = torch.randn(T, N, device=dev, dtype=torch.bfloat16)
    fl = 2.0 * T * N * K
    ref = torch.mm(x, w[0].t())
    y4 = ops.gemm4a(x, w, off, 0, None)
    y8 = ops.grouped_gemm8(x, w, off, 0, None, False)
    r4 = ((y4.float() - ref.float()).norm() / ref.float().norm()).item()
    r8 = ((y8.float() - ref.float()).norm() / ref.float().norm()).item()
    print(f"{name}: rel gemm4a {r4:.1e} gemm8 {r8:.1e}", flush=True)
    cases.append((f"{name} fwd [{T}x{K}]x[{K}x{N}]", fl, {
        "hipBLASLt": lambda x=x, w=w: torch.mm(x, w[0].t()),
        "gemm4a": lambda x=x, w=w: ops.gemm4a(x, w, off, 0, None),
        "gemm8": lambda x=x, w=w: ops.grouped_gemm8(x, w, off, 0, None, False)}))
    if N % 64 == 0:
        cases.append((f"{name} dX [{T}x{N}]x[{N}x{K}]", fl, {
            "hipBLASLt": lambda dy=dy, w=w: torch.mm(dy, w[0]),
            "gemm4a": lambda dy=dy, w=w: ops.gemm4a(dy, w, off, 1, None),
            "gemm8": lambda dy=dy, w=w: ops.grouped_gemm8(dy, w, off, 1, None, False)}))
for r in range(a.rounds):
    for name, fl, arms in cases:
        line = []
        for arm, fn in arms.items():
            ms = tm(fn)
            line.append(f"{arm} {ms:.3f} ms {fl / ms / 1e9:.0f} TF")
        print(f"round {r} {name}: " + " | ".join(line), flush=True)
