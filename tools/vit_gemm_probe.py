"""ViT-B/16 projection GEMMs (T = 256 x 197 tokens): the 8-phase kernel (gemm8.hip, one dense group)
against hipBLASLt (torch.mm / addmm with the tuned table if present), forward X W^T and data grad
dY W, same operands, interleaved timing.
    python tools/vit_gemm_probe.py [--iters N]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from solvingpapers_amd.ops import _ext  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--iters", type=int, default=30)
a = ap.parse_args()
ops = _ext.ops()
dev = "cuda"
T = 256 * 197
off = torch.tensor([0, T], dtype=torch.int32, device=dev)


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
    return s.elapsed_time(e) / a.iters


for name, (N, K) in {"qkv": (2304, 768), "proj": (768, 768), "fc1": (3072, 768), "fc2": (768, 3072)}.items():
    x = torch.randn(T, K, device=dev, dtype=torch.bfloat16)
    w = torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.03
    b = torch.randn(N, device=dev, dtype=torch.bfloat16)
    dy = torch.randn(T, N, device=dev, dtype=torch.bfloat16)
    fl = 2.0 * T * N * K
    g_f = tm(lambda: ops.grouped_gemm8(x, w[None], off, 0, None, False))
    h_f = tm(lambda: torch.addmm(b, x, w.t()))
    g_d = tm(lambda: ops.grouped_gemm8(dy, w[None], off, 1, None, False))
    wt = w.t().contiguous()
    h_d = tm(lambda: torch.mm(dy, wt.t()))
    g_f2 = tm(lambda: ops.grouped_gemm8(x, w[None], off, 0, None, False))
    h_f2 = tm(lambda: torch.addmm(b, x, w.t()))
    rel = ((ops.grouped_gemm8(x, w[None], off, 0, None, False).float() - torch.mm(x, w.t()).float()).norm()
           / torch.mm(x, w.t()).float().norm()).item()
    print(f"{name:5s} N {N} K {K}: fwd gemm8 {fl / min(g_f, g_f2) / 1e9:6.0f} TF vs hipBLASLt+bias "
          f"{fl / min(h_f, h_f2) / 1e9:6.0f} TF | dgrad gemm8 {fl / g_d / 1e9:6.0f} vs hipBLASLt {fl / h_d / 1e9:6.0f} TF"
          f" (rel {rel:.1e})", flush=True)
