"""Attention kernel micro-benchmark (LLaMA3-8B shape by default): TFLOP/s fwd / bwd.

--ab ENV=VAL[,ENV=VAL...]: also time the backward with those env settings in the same
process (the dK/dV kernel choice is read per call), since MI355X devices differ by up to
~10 % and cross-box comparisons are noise."""
import argparse, math, time, sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from solvingpapers_amd.ops import _ext

ap = argparse.ArgumentParser()
ap.add_argument("--B", type=int, default=1); ap.add_argument("--T", type=int, default=8192)
ap.add_argument("--H", type=int, default=32); ap.add_argument("--Hkv", type=int, default=8)
ap.add_argument("--hd", type=int, default=128); ap.add_argument("--noncausal", action="store_true")
ap.add_argument("--iters", type=int, default=10)
ap.add_argument("--ab", default="")
a = ap.parse_args()
ops = _ext.ops()
B, T, H, Hkv, hd = a.B, a.T, a.H, a.Hkv, a.hd
causal = not a.noncausal
q = torch.randn(B, T, H, hd, device="cuda", dtype=torch.bfloat16)
k = torch.randn(B, T, Hkv, hd, device="cuda", dtype=torch.bfloat16)
v = torch.randn(B, T, Hkv, hd, device="cuda", dtype=torch.bfloat16)
sc = 1 / math.sqrt(hd)
out, lse = ops.attn_fwd(q, k, v, sc, causal)
do = torch.randn_like(out)
dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
def t(fn):
    for _ in range(2): fn()
    torch.cuda.synchronize(); s = time.perf_counter()
    for _ in range(a.iters): fn()
    torch.cuda.synchronize(); return (time.perf_counter() - s) / a.iters
fl = 4 * B * H * T * T * hd * (0.5 if causal else 1.0)
tf = t(lambda: ops.attn_fwd(q, k, v, sc, causal))
tb = t(lambda: ops.attn_bwd(do, q, k, v, out, lse, dq, dk, dv, sc, causal))
print(f"attn B{B} T{T} H{H}/{Hkv} hd{hd} causal={causal}: fwd {tf*1e3:.3f} ms {fl/tf/1e12:.0f} TF | bwd {tb*1e3:.3f} ms {2.5*fl/tb/1e12:.0f} TF(2.5x)", flush=True)
for setting in filter(None, a.ab.split(",")):
    key, val = setting.split("=")
    old = os.environ.get(key)
    os.environ[key] = val
    tb2 = t(lambda: ops.attn_bwd(do, q, k, v, out, lse, dq, dk, dv, sc, causal))
    if old is None: os.environ.pop(key)
    else: os.environ[key] = old
    tb3 = t(lambda: ops.attn_bwd(do, q, k, v, out, lse, dq, dk, dv, sc, causal))
    print(f"   bwd with {key}={val}: {tb2*1e3:.3f} ms ({2.5*fl/tb2/1e12:.0f} TF) vs default again {tb3*1e3:.3f} ms", flush=True)
