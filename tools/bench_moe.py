"""Grouped-GEMM tile-config sweep at DeepSeek-style MoE shapes vs a dense hipBLASLt GEMM
of the same FLOPs. usage: python tools/bench_moe.py [tokens] [E] [k] [D] [F]"""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from solvingpapers_amd.ops import _ext, moe as M

T = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
E = int(sys.argv[2]) if len(sys.argv) > 2 else 64
k = int(sys.argv[3]) if len(sys.argv) > 3 else 6
D = int(sys.argv[4]) if len(sys.argv) > 4 else 2048
F = int(sys.argv[5]) if len(sys.argv) > 5 else 1408
ops = _ext.ops()
dev = "cuda"
torch.manual_seed(0)
logits = torch.randn(T, E, device=dev)
idx, w = M.route(logits, k)
plan = M.permute(idx, E)
A = T * k
x = torch.randn(A, D, device=dev, dtype=torch.bfloat16)
W13 = torch.randn(E, 2 * F, D, device=dev, dtype=torch.bfloat16) * 0.02
W2 = torch.randn(E, D, F, device=dev, dtype=torch.bfloat16) * 0.02
h = torch.randn(A, F, device=dev, dtype=torch.bfloat16)
dy13 = torch.randn(A, 2 * F, device=dev, dtype=torch.bfloat16)
dy2 = torch.randn(A, D, device=dev, dtype=torch.bfloat16)
cases = {
    "fwd W13": (lambda c: ops.grouped_gemm(x, W13, plan.offsets, 0, None, False, c), 2 * A * 2 * F * D),
    "fwd W2": (lambda c: ops.grouped_gemm(h, W2, plan.offsets, 0, None, False, c), 2 * A * D * F),
    "dX W13": (lambda c: ops.grouped_gemm(dy13, W13, plan.offsets, 1, None, False, c), 2 * A * 2 * F * D),
    "dX W2": (lambda c: ops.grouped_gemm(dy2, W2, plan.offsets, 1, None, False, c), 2 * A * D * F),
    "dW W13": (lambda c: ops.grouped_gemm(dy13, x, plan.offsets, 2, None, False, c), 2 * A * 2 * F * D),
    "dW W2": (lambda c: ops.grouped_gemm(dy2, h, plan.offsets, 2, None, False, c), 2 * A * D * F),
}


def tm(fn, it=10):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it


print(f"tokens {T} E {E} k {k} D {D} F {F}; assignments {A}")
for name, (fn, fl) in cases.items():
    ref = fn(0).float()
    row = []
    for c in range(6):
        out = fn(c).float()
        err = ((out - ref).norm() / ref.norm()).item()
        ms = tm(lambda: fn(c))
        row.append(f"c{c}:{fl / ms / 1e9:6.0f}TF{'' if err < 1e-2 else ' ERR%.2e' % err}")
    print(f"{name:8s} " + " ".join(row))
xq, sx = M.quant_rows_fp8(x)
wq, sw = M.quant_rows_fp8(W13.view(E * 2 * F, D))
wq = wq.view(E, 2 * F, D)
ms = tm(lambda: ops.grouped_gemm_fp8(xq, sx, wq, sw.view(E, 2 * F), plan.offsets))
print(f"fp8 fwd W13 grouped GEMM: {2 * A * 2 * F * D / ms / 1e9:.0f} TF (e4m3, block-scaled MFMA)")
msq = tm(lambda: M.quant_rows_fp8(x))
print(f"quant_rows_fp8 [{A}x{D}]: {msq:.3f} ms = {A * D * 3 / msq / 1e6:.0f} GB/s")
a = torch.randn(A, D, device=dev, dtype=torch.bfloat16)
b = torch.randn(2 * F, D, device=dev, dtype=torch.bfloat16)
ms = tm(lambda: torch.mm(a, b.t()))
print(f"dense hipBLASLt [{A}x{D}]x[{D}x{2*F}]: {2 * A * 2 * F * D / ms / 1e9:.0f} TF")
