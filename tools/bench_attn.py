"""Attention kernel micro-benchmark (LLaMA3-8B shape by default): TFLOP/s fwd / bwd.

--ab ENV=VAL[,ENV=VAL...]: also time both passes with those env settings in the same
process (the kernel choices are read per call), since MI355X devices differ by up to
~10 % and cross-box comparisons are noise. Each A/B runs in ABBA order (default, variant,
variant, default) and averages the two arms, because the clock drifts within a run."""
import argparse, math, time, sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from solvingpapers_amd.ops import _ext

ap = argparse.ArgumentParser()
ap.add_argument("--B", type=int, default=1); ap.add_argument("--T", type=int, default=8192)
ap.add_argument("--H", type=int, default=32); ap.add_argument("--Hkv", type=int, default=8)
ap.add_argument("--hd", type=int, default=128); ap.add_argument("--noncausal", action="store_true")
ap.add_argument("--hdv", type=int, default=0, help="v head dim (default = hd); 128 with --hd 192 = MLA")
ap.add_argument("--pad", type=int, default=0, help="also time the same problem zero-padded to this head dim")
ap.add_argument("--dropout", type=float, default=0.0)
ap.add_argument("--iters", type=int, default=10)
ap.add_argument("--packed", action="store_true", help="q/k/v as views of one fused qkv buffer (the model's layout)")
ap.add_argument("--ab", default="")
ap.add_argument("--interleave", action="store_true",
                help="also time each pass right after a LLaMA-8B w13-sized GEMM (the in-step order: "
                     "the GEMM's power draw sets the clock the attention kernel starts at)")
a = ap.parse_args()
ops = _ext.ops()
B, T, H, Hkv, hd = a.B, a.T, a.H, a.Hkv, a.hd
hdv = a.hdv or hd
causal = not a.noncausal
if a.packed:      # the model's layout: q / k / v are head slices of one fused [B, T, H + 2 Hkv, hd] buffer
    assert hdv == hd
    qkv = torch.randn(B, T, H + 2 * Hkv, hd, device="cuda", dtype=torch.bfloat16)
    q, k, v = qkv[:, :, :H], qkv[:, :, H:H + Hkv], qkv[:, :, H + Hkv:]
else:
    q = torch.randn(B, T, H, hd, device="cuda", dtype=torch.bfloat16)
    k = torch.randn(B, T, Hkv, hd, device="cuda", dtype=torch.bfloat16)
    v = torch.randn(B, T, Hkv, hdv, device="cuda", dtype=torch.bfloat16)
sc = 1 / math.sqrt(hd)
P, SEED = a.dropout, 1234
out, lse = ops.attn_fwd(q, k, v, sc, causal, P, SEED)
do = torch.randn_like(out)
dq, dk, dv = (torch.empty(t.shape, device="cuda", dtype=t.dtype) for t in (q, k, v))
def t(fn):
    # warm for >= 0.3 s first: the clock ramps over the first ~0.1 s of load, and a short warmup
    # made the first reading of a process ~15 % slow (0.62 vs 0.52 ms fwd at the LLaMA shape)
    w0 = time.perf_counter()
    while True:
        for _ in range(4): fn()
        torch.cuda.synchronize()
        if time.perf_counter() - w0 > 0.3: break
    s = time.perf_counter()
    for _ in range(a.iters): fn()
    torch.cuda.synchronize(); return (time.perf_counter() - s) / a.iters
cf = 0.5 if causal else 1.0
fl = 2 * B * H * T * T * (hd + hdv) * cf                 # useful fwd FLOPs (QK^T + PV)
flb = 2 * B * H * T * T * (3 * hd + 2 * hdv) * cf        # useful bwd FLOPs (S, dP, dV, dK, dQ)
tf = t(lambda: ops.attn_fwd(q, k, v, sc, causal, P, SEED))
tb = t(lambda: ops.attn_bwd(do, q, k, v, out, lse, dq, dk, dv, sc, causal, P, SEED))
print(f"attn B{B} T{T} H{H}/{Hkv} hd{hd}/{hdv} causal={causal} p={P}: fwd {tf*1e3:.3f} ms {fl/tf/1e12:.0f} TF | "
      f"bwd {tb*1e3:.3f} ms {flb/tb/1e12:.0f} TF", flush=True)
if a.interleave:
    xg = torch.randn(B * T, 4096, device="cuda", dtype=torch.bfloat16)
    wg = torch.randn(4096, 14336, device="cuda", dtype=torch.bfloat16)
    def ti(fn):
        """mean time of fn alone when each call follows a GEMM on the same stream (events bracket fn only)"""
        e0 = [torch.cuda.Event(enable_timing=True) for _ in range(a.iters)]
        e1 = [torch.cuda.Event(enable_timing=True) for _ in range(a.iters)]
        for _ in range(8): xg @ wg; fn()
        for i in range(a.iters):
            xg @ wg
            e0[i].record(); fn(); e1[i].record()
        torch.cuda.synchronize()
        return sum(x.elapsed_time(y) for x, y in zip(e0, e1)) / a.iters / 1e3
    tfi = ti(lambda: ops.attn_fwd(q, k, v, sc, causal, P, SEED))
    tbi = ti(lambda: ops.attn_bwd(do, q, k, v, out, lse, dq, dk, dv, sc, causal, P, SEED))
    print(f"   after a GEMM each: fwd {tfi*1e3:.3f} ms {fl/tfi/1e12:.0f} TF | bwd {tbi*1e3:.3f} ms {flb/tbi/1e12:.0f} TF",
          flush=True)
if a.pad:
    pad = lambda x: torch.nn.functional.pad(x, (0, a.pad - x.shape[-1]))
    qp, kp, vp = pad(q), pad(k), pad(v)
    op_, lp = ops.attn_fwd(qp, kp, vp, sc, causal)
    dop = torch.randn_like(op_)
    dqp, dkp, dvp = torch.empty_like(qp), torch.empty_like(kp), torch.empty_like(vp)
    tfp = t(lambda: ops.attn_fwd(qp, kp, vp, sc, causal))
    tbp = t(lambda: ops.attn_bwd(dop, qp, kp, vp, op_, lp, dqp, dkp, dvp, sc, causal))
    print(f"   same problem zero-padded to hd {a.pad}: fwd {tfp*1e3:.3f} ms ({fl/tfp/1e12:.0f} useful TF) | "
          f"bwd {tbp*1e3:.3f} ms ({flb/tbp/1e12:.0f} useful TF)", flush=True)
def _arm(key, val):
    """(fwd s, bwd s, out) with env key=val (val None: unset) for the duration of the call."""
    old = os.environ.get(key)
    if val is None:
        os.environ.pop(key, None)
    else:
        os.environ[key] = val
    try:
        tfx = t(lambda: ops.attn_fwd(q, k, v, sc, causal, P, SEED))
        tbx = t(lambda: ops.attn_bwd(do, q, k, v, out, lse, dq, dk, dv, sc, causal, P, SEED))
        ox, _ = ops.attn_fwd(q, k, v, sc, causal, P, SEED)
    finally:
        if old is None:
            os.environ.pop(key, None)
        else:
            os.environ[key] = old
    return tfx, tbx, ox


for setting in filter(None, a.ab.split(",")):
    key, val = setting.split("=")
    base = os.environ.get(key)
    # ABBA order (default, variant, variant, default): the chip's clock drifts over a run, so a
    # fixed variant-then-default order biases the comparison
    d1 = _arm(key, base)
    v1 = _arm(key, val)
    v2 = _arm(key, val)
    d2 = _arm(key, base)
    tf2, tb2 = (v1[0] + v2[0]) / 2, (v1[1] + v2[1]) / 2
    tf3, tb3 = (d1[0] + d2[0]) / 2, (d1[1] + d2[1]) / 2
    err = ((v1[2].float() - d1[2].float()).norm() / d1[2].float().norm()).item()
    print(f"   with {key}={val}: fwd {tf2*1e3:.3f} ms ({fl/tf2/1e12:.0f} TF, out rel diff {err:.1e}) vs default "
          f"{tf3*1e3:.3f} ms ({fl/tf3/1e12:.0f} TF) | bwd {tb2*1e3:.3f} ms ({flb/tb2/1e12:.0f} TF) vs "
          f"{tb3*1e3:.3f} ms", flush=True)

if os.environ.get("SPA_ATTN_STAMP"):
    st = ops.attn_bwd_stamps().double().cpu()
    # pipelined dK/dV kernel built with -DSPA_DKDV3_STAMP=1 (tools/build_variant.sh): per wave
    # staging, compute 1, compute 2, barrier wait, epilogue, intervals, whole wave (s_memtime)
    wave = torch.arange(st.shape[0]) % 8
    live = st[:, 5] > 0
    v5 = os.environ.get("SPA_ATTN_DKDV5", "0") != "0"
    names = ["DMA issue", "compute", "DMA wait", "barrier wait"] if v5 else ["staging", "compute 1", "compute 2", "barrier wait"]
    roles = (("A (S -> P, dV^T)", wave < 4), ("B (dP, dS, dK^T)", wave >= 4)) if v5 else \
        (("A (1 dV^T, 2 S->P)", wave < 4), ("B (1 dP+dS, 2 dK^T)", wave >= 4))
    for role, sel in roles:
        r = st[live & sel]
        per = r[:, :4].sum(0) / r[:, 5].sum()
        print(f"   dK/dV loop, role {role}: cycles per interval " + ", ".join(f"{n} {v:.0f}" for n, v in zip(names, per.tolist()))
              + f" | loop {per.sum().item():.0f} | epilogue per wave {r[:, 4].mean().item():.0f}"
              + f" | whole wave {r[:, 6].mean().item():.0f} over {r[:, 5].mean().item():.0f} intervals"
              + (f" ({r[:, 7].sum().item() / r[:, 5].sum().item() * 100:.0f} % pipelined)" if v5 else ""), flush=True)
