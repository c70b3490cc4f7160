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


def gg(a, b, mode, c):
    """c = 0..5: register-staged tile configs of moe.hip; c = 6: the 8-phase LDS-DMA kernel (gemm8.hip)"""
    if c == 6:
        return ops.grouped_gemm8(a, b, plan.offsets, mode, None, False)
    return ops.grouped_gemm(a, b, plan.offsets, mode, None, False, c)


cases = {
    "fwd W13": (lambda c: gg(x, W13, 0, c), 2 * A * 2 * F * D),
    "fwd W2": (lambda c: gg(h, W2, 0, c), 2 * A * D * F),
    "dX W13": (lambda c: gg(dy13, W13, 1, c), 2 * A * 2 * F * D),
    "dX W2": (lambda c: gg(dy2, W2, 1, c), 2 * A * D * F),
    "dW W13": (lambda c: gg(dy13, x, 2, c), 2 * A * 2 * F * D),
    "dW W2": (lambda c: gg(dy2, h, 2, c), 2 * A * D * F),
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
    for c in (0, 2, 3, 6):
        out = fn(c).float()
        err = ((out - ref).norm() / ref.norm()).item()
        ms = tm(lambda: fn(c))
        row.append(f"{'g8' if c == 6 else 'c%d' % c}:{fl / ms / 1e9:6.0f}TF{'' if err < 1e-2 else ' ERR%.2e' % err}")
    print(f"{name:8s} " + " ".join(row))
xq, sx = M.quant_rows_fp8(x)
wq, sw = M.quant_rows_fp8(W13.view(E * 2 * F, D))
wq = wq.view(E, 2 * F, D)
ms = tm(lambda: ops.grouped_gemm_fp8(xq, sx, wq, sw.view(E, 2 * F), plan.offsets))
print(f"fp8 fwd W13 grouped GEMM: {2 * A * 2 * F * D / ms / 1e9:.0f} TF (e4m3, per-row scales applied in the epilogue)")
xb, sxb = M.quant_act_fp8_blk(x)
wqb, wtqb, swb, swtb = M.quant_weight_fp8_blk(W13)
ms = tm(lambda: ops.grouped_gemm_fp8_blk(xb, sxb, wqb, swb, plan.offsets))
print(f"fp8 fwd W13 grouped GEMM, 1x128 / 128x128 E8M0 block scales on the MFMA: {2 * A * 2 * F * D / ms / 1e9:.0f} TF")
dq, sdq = M.quant_act_fp8_blk(dy13)
ms = tm(lambda: ops.grouped_gemm_fp8_blk(dq, sdq, wtqb, swtb, plan.offsets))
print(f"fp8 dX W13 grouped GEMM (block scales, W^T bytes): {2 * A * 2 * F * D / ms / 1e9:.0f} TF")
ms = tm(lambda: M.quant_act_fp8_blk(x))
print(f"quant_act_fp8_blk [{A}x{D}]: {ms:.3f} ms = {A * D * 3.06 / ms / 1e6:.0f} GB/s")
M.bump_weight_epoch()
ms = tm(lambda: (M.bump_weight_epoch(), M.quant_weight_fp8_blk(W13)))
print(f"quant_weight_fp8_blk W13 [{E}x{2 * F}x{D}] (+ transposed bytes): {ms:.3f} ms = "
      f"{E * 2 * F * D * 4 / ms / 1e6:.0f} GB/s")
msq = tm(lambda: M.quant_rows_fp8(x))
print(f"quant_rows_fp8 [{A}x{D}]: {msq:.3f} ms = {A * D * 3 / msq / 1e6:.0f} GB/s")
a = torch.randn(A, D, device=dev, dtype=torch.bfloat16)
b = torch.randn(2 * F, D, device=dev, dtype=torch.bfloat16)
ms = tm(lambda: torch.mm(a, b.t()))
print(f"dense hipBLASLt [{A}x{D}]x[{D}x{2*F}]: {2 * A * 2 * F * D / ms / 1e9:.0f} TF")
# the 8-phase kernel on ONE expert = a dense GEMM: separates the core loop from grouping overheads
for S in (4096, 8192):
    off1 = torch.tensor([0, S], dtype=torch.int32, device=dev)
    xa = torch.rand(S, S, device=dev).sub_(0.5).bfloat16()
    wb = torch.rand(1, S, S, device=dev).sub_(0.5).bfloat16()
    fl = 2.0 * S ** 3
    r = []
    for mode, (a_, b_) in enumerate(((xa, wb), (xa, wb), (xa, xa))):
        ms = tm(lambda: ops.grouped_gemm8(a_, b_, off1, mode, None, False))
        r.append(f"mode{mode} {fl / ms / 1e9:6.0f}TF")
    ms = tm(lambda: torch.mm(xa, wb[0].t()))
    print(f"dense {S}^3 via gemm8 (E=1, uniform[-.5,.5)): " + " ".join(r) + f" | hipBLASLt NT {fl / ms / 1e9:6.0f}TF")

if os.environ.get("SPA_BENCH_ABLATE"):
    # where the 8-phase kernel's time goes: 1 no DMA, 2 no LDS fragment reads, 3 no vmcnt waits,
    # 4 = the non-interleaved DMA schedule
    S = 8192
    off1 = torch.tensor([0, S], dtype=torch.int32, device=dev)
    xa = torch.rand(S, S, device=dev).sub_(0.5).bfloat16()
    wb = torch.rand(1, S, S, device=dev).sub_(0.5).bfloat16()
    for abl in (0, 4, 1, 2, 3):
        os.environ["SPA_GG8_ABLATE"] = str(abl)
        r = []
        for mode in (0, 1, 2):
            ms = tm(lambda: ops.grouped_gemm8(xa, wb if mode < 2 else xa, off1, mode, None, False))
            r.append(f"mode{mode} {2.0 * S ** 3 / ms / 1e9:6.0f}TF")
        print(f"ablate {abl}: " + " ".join(r))
    os.environ["SPA_GG8_ABLATE"] = "0"
