"""gemm4a (csrc/kernels/gemm4a.hip: 4 waves x 128x128, AGPR-pinned accumulators) against gemm8 and
hipBLASLt on random operands, same process, interleaved rounds: dense 8192^3 / 4096^3 and the
dsv3_style grouped forward (E 64, top-6 over 8192 tokens, D 2048 -> 2F 2816). Checks every
result against an fp32 torch reference first.
    python tools/bench_gemm4a.py [--iters N] [--rounds R] [--env NAME=V1,V2]"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from solvingpapers_amd.ops import _ext

ap = argparse.ArgumentParser()
ap.add_argument("--iters", type=int, default=20)
ap.add_argument("--rounds", type=int, default=2)
ap.add_argument("--env", action="append", default=[], help="NAME=V1,V2,...: extra gemm4a arms with NAME set to each value (repeatable)")
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


cases = []
for S in (8192, 4096):
    x = torch.rand(S, S, device=dev).sub_(0.5).bfloat16()
    w = torch.rand(1, S, S, device=dev).sub_(0.5).bfloat16()
    off = torch.tensor([0, S], dtype=torch.int32, device=dev)
    ref = torch.mm(x.float(), w[0].float().t())
    cases.append((f"dense {S}^3", x, w, off, ref, 2.0 * S ** 3, lambda x=x, w=w: torch.mm(x, w[0].t())))
from solvingpapers_amd.ops import moe as M
torch.manual_seed(0)
T, E, k, D, F = 8192, 64, 6, 2048, 1408
idx, _ = M.route(torch.randn(T, E, device=dev), k)
plan = M.permute(idx, E)
A = T * k
xg = torch.randn(A, D, device=dev, dtype=torch.bfloat16)
W13 = torch.randn(E, 2 * F, D, device=dev, dtype=torch.bfloat16) * 0.02
offs = plan.offsets.to(torch.int32)
oc = offs.tolist()
ref = torch.cat([xg[oc[e]:oc[e + 1]].float() @ W13[e].float().t() for e in range(E)])
cases.append(("grouped fwd dsv3_style", xg, W13, offs, ref, 2.0 * A * 2 * F * D, None))
# ragged: experts with 0, 1, 255, 257 rows
cnt = torch.tensor([0, 1, 255, 257, 0, 513, 3, 64], dtype=torch.int32)
offr = torch.cat([torch.zeros(1, dtype=torch.int32), cnt.cumsum(0).to(torch.int32)]).to(dev)
xr = torch.randn(int(cnt.sum()), 256, device=dev, dtype=torch.bfloat16)
wr = torch.randn(8, 192, 256, device=dev, dtype=torch.bfloat16)
o = offr.tolist()
refr = torch.cat([xr[o[e]:o[e + 1]].float() @ wr[e].float().t() for e in range(8)])
cases.append(("ragged E8 N192 K256", xr, wr, offr, refr, 1.0, None))

for name, x, w, off, ref, fl, blas in cases:
    y4 = ops.gemm4a(x, w, off, 0, None)
    y8 = ops.grouped_gemm8(x, w, off, 0, None, False)
    torch.cuda.synchronize()
    print(f"{name}: gemm4a rel {rel(y4, ref):.2e}  gemm8 rel {rel(y8, ref):.2e}  gemm4a==gemm8 {torch.equal(y4, y8)}",
          flush=True)
    assert rel(y4, ref) < 1e-2, name

# modes 1 (dX = dY W_e) and 2 (dW_e = dY_e^T X_e), dsv3_style widths and ragged experts, + accumulate
dy13 = torch.randn(A, 2 * F, device=dev, dtype=torch.bfloat16)
mcases = [("grouped dX dsv3_style", dy13, W13, offs, oc, 2.0 * A * 2 * F * D),
          ("ragged dX", torch.randn(xr.shape[0], 192, device=dev, dtype=torch.bfloat16), wr, offr, o, 1.0)]
for name, dy, w, off, oo, fl in mcases:
    y4 = ops.gemm4a(dy, w, off, 1, None)
    y8 = ops.grouped_gemm8(dy, w, off, 1, None, False)
    ref = torch.cat([dy[oo[e]:oo[e + 1]].float() @ w[e].float() for e in range(len(oo) - 1)])
    print(f"{name}: gemm4a rel {rel(y4, ref):.2e}  gemm8 rel {rel(y8, ref):.2e}", flush=True)
    assert rel(y4, ref) < 1e-2, name
wcases = [("grouped dW dsv3_style", dy13, xg, offs, oc, 2.0 * A * 2 * F * D),
          ("ragged dW", torch.randn(xr.shape[0], 192, device=dev, dtype=torch.bfloat16), xr, offr, o, 1.0)]
for name, dy, xx, off, oo, fl in wcases:
    y4 = ops.gemm4a(dy, xx, off, 2, None)
    ref = torch.stack([dy[oo[e]:oo[e + 1]].float().t() @ xx[oo[e]:oo[e + 1]].float() for e in range(len(oo) - 1)])
    acc0 = torch.randn_like(y4)
    y4a = ops.gemm4a(dy, xx, off, 2, acc0.clone(), True)
    print(f"{name}: gemm4a rel {rel(y4, ref):.2e}  accumulate rel {rel(y4a, ref + acc0.float()):.2e}", flush=True)
    assert rel(y4, ref) < 1e-2 and rel(y4a, ref + acc0.float()) < 1e-2, name
timed_mw = [("grouped dX dsv3_style", lambda: ops.gemm4a(dy13, W13, offs, 1, None), lambda: ops.grouped_gemm8(dy13, W13, offs, 1, None, False), 2.0 * A * 2 * F * D),
            ("grouped dW dsv3_style", lambda: ops.gemm4a(dy13, xg, offs, 2, None), lambda: ops.grouped_gemm8(dy13, xg, offs, 2, None, False), 2.0 * A * 2 * F * D)]

arms = [("gemm4a", None)]
for ev_ in a.env:
    k_, vs = ev_.split("=")
    arms += [(f"{k_}={v}", (k_, v)) for v in vs.split(",")]
for r in range(a.rounds):
    for name, x, w, off, ref, fl, blas in cases[:3]:
        res = []
        for lab, ev in arms:
            if ev:
                os.environ[ev[0]] = ev[1]
            res.append((lab, tm(lambda: ops.gemm4a(x, w, off, 0, None))))
            if ev:
                os.environ.pop(ev[0])
        res.append(("gemm8", tm(lambda: ops.grouped_gemm8(x, w, off, 0, None, False))))
        if blas is not None:
            res.append(("hipBLASLt", tm(blas)))
        print(f"round {r} {name}: " + "  ".join(f"{lab} {ms:.3f} ms {fl / ms / 1e9:.0f} TF" for lab, ms in res),
              flush=True)
    for name, f4, f8, fl in timed_mw:
        res = []
        for lab, ev in arms:
            if ev:
                os.environ[ev[0]] = ev[1]
            res.append((lab, tm(f4)))
            if ev:
                os.environ.pop(ev[0])
        res.append(("gemm8", tm(f8)))
        print(f"round {r} {name}: " + "  ".join(f"{lab} {ms:.3f} ms {fl / ms / 1e9:.0f} TF" for lab, ms in res), flush=True)
