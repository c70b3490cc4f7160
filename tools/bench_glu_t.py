"""LLaMA3-8B w13 backward pieces (T 8192, D 4096, F 14336): glu_bwd vs glu_bwd_t (GLU backward that also
writes dH^T), and the dW products they feed (x-transposed form vs both-transposed form), same process.
    python tools/bench_glu_t.py [--iters N]"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from solvingpapers_amd.ops import _ext
from solvingpapers_amd.ops.layout import transpose2d
from solvingpapers_amd.utils.tuning import load_gemm_tuning

ap = argparse.ArgumentParser()
ap.add_argument("--iters", type=int, default=20)
a = ap.parse_args()
print("table loaded:", load_gemm_tuning(), flush=True)
ops = _ext.ops()


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


T, D, F = 8192, 4096, 14336
h = torch.randn(T, 2 * F, device="cuda").bfloat16()
df = torch.randn(T, F, device="cuda").bfloat16()
x = torch.randn(T, D, device="cuda").bfloat16()
out = torch.zeros(2 * F, D, device="cuda").bfloat16()
dh, dht = ops.glu_bwd_t(df, h, 6)
xt = transpose2d(x)
w13 = (torch.randn(2 * F, D, device="cuda") * 0.01).bfloat16()
w13t = transpose2d(w13)
for r in range(2):
    t_b = tm(lambda: ops.glu_bwd(df, h, 6))
    t_bt = tm(lambda: ops.glu_bwd_t(df, h, 6))
    t_tr = tm(lambda: transpose2d(dh))
    t_x = tm(lambda: out.addmm_(dh.t(), xt.t()))
    t_both = tm(lambda: out.addmm_(dht, xt.t()))
    t_dg = tm(lambda: torch.mm(dh, w13t.t()))
    t_dgt = tm(lambda: torch.mm(dht.t(), w13t.t()))
    t_dgt2 = tm(lambda: torch.mm(dht.t(), w13))
    print(f"round {r}: dX from dH {t_dg:.3f} ms | from dH^T (on W^T) {t_dgt:.3f} ms | from dH^T (on W) {t_dgt2:.3f} ms", flush=True)
    t_f = tm(lambda: ops.glu_fwd(h, 6))
    t_ft = tm(lambda: ops.glu_fwd_t(h, 6))
    print(f"round {r}: glu_fwd {t_f:.3f} ms | glu_fwd_t {t_ft:.3f} ms", flush=True)
    print(f"round {r}: glu_bwd {t_b:.3f} ms | glu_bwd_t {t_bt:.3f} ms | transpose dH {t_tr:.3f} ms | "
          f"dW x-form {t_x:.3f} ms | dW both-form {t_both:.3f} ms | plain {t_b + t_x:.3f} vs glu_t {t_bt + t_both:.3f}",
          flush=True)
