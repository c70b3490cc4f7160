"""dsv3_style expert GEMM cases on the 8-phase kernel (gemm8.hip), one process, TF per case: for
B N N B comparisons of two builds (SPA_EXT_SO=<other .so> for the B arms).
    python tools/g8_cases.py [--iters N]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from solvingpapers_amd.ops import _ext  # noqa: E402
from solvingpapers_amd.ops import moe as M  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--iters", type=int, default=20)
a = ap.parse_args()
ops = _ext.ops()
dev = "cuda"
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
g13 = torch.zeros(E, 2 * F, D, device=dev, dtype=torch.bfloat16)
g2 = torch.zeros(E, D, F, device=dev, dtype=torch.bfloat16)
cases = {"fwd W13": (lambda: ops.grouped_gemm8(x, W13, plan.offsets, 0, None, False), 2 * A * 2 * F * D),
         "fwd W2": (lambda: ops.grouped_gemm8(h, W2, plan.offsets, 0, None, False), 2 * A * D * F),
         "dX W13": (lambda: ops.grouped_gemm8(dy13, W13, plan.offsets, 1, None, False), 2 * A * 2 * F * D),
         "dX W2": (lambda: ops.grouped_gemm8(dy2, W2, plan.offsets, 1, None, False), 2 * A * D * F),
         "dW W13": (lambda: ops.grouped_gemm8(dy13, x, plan.offsets, 2, None, False), 2 * A * 2 * F * D),
         "dW W2": (lambda: ops.grouped_gemm8(dy2, h, plan.offsets, 2, None, False), 2 * A * D * F),
         "dW W13 acc": (lambda: ops.grouped_gemm8(dy13, x, plan.offsets, 2, g13, True), 2 * A * 2 * F * D),
         "dW W2 acc": (lambda: ops.grouped_gemm8(dy2, h, plan.offsets, 2, g2, True), 2 * A * D * F)}
res = {}
for name, (fn, fl) in cases.items():
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(a.iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / a.iters
    res[name] = fl / ms / 1e9
print(" ".join(f"{n.replace(' ', '_')}={v:.0f}" for n, v in res.items()), flush=True)
