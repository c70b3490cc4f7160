"""Block-scaled fp8 grouped GEMMs: the 8-phase LDS-DMA kernel (gemm8_fp8.hip, 16x16x128 scaled
MFMA) vs the register-staged 32x32x64 kernel (moe_fp8.hip), same operands, interleaved rounds.
Forward, dX (on the transposed weight bytes) and dW (token-segment Wgrad) of both expert
projections, plus a dense 8192^3 product (E = 1). Prints one JSON line per shape.
    python tools/bench_fp8_g8.py [--experts 32] [--rows 32768] [--dim 7168] [--ffn 2048]"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from solvingpapers_amd.ops import _ext  # noqa: E402
from solvingpapers_amd.ops import moe as M  # noqa: E402


def tm(fn, iters):
    fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def ab(fns, iters, rounds):
    t = {k: [] for k in fns}
    for r in range(rounds):
        for k in (list(fns) if r % 2 == 0 else list(fns)[::-1]):
            t[k].append(tm(fns[k], iters))
    return {k: statistics.median(v) for k, v in t.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--experts", type=int, default=32)
    ap.add_argument("--rows", type=int, default=32768, help="routed rows (tokens x top-k)")
    ap.add_argument("--dim", type=int, default=7168)
    ap.add_argument("--ffn", type=int, default=2048)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--dense", type=int, default=8192)
    a = ap.parse_args()
    assert _ext.load(), "HIP extension missing"
    ops = _ext.ops()
    E, T, D, F = a.experts, a.rows, a.dim, a.ffn
    g = torch.Generator().manual_seed(0)
    cnt = torch.multinomial(torch.ones(E), T, replacement=True, generator=g).bincount(minlength=E)
    off = torch.cat([torch.zeros(1, dtype=torch.long), cnt.cumsum(0)]).int().cuda()
    poff = M.padded_offsets(off)
    ld = (T + E * 127 + 127) // 128 * 128
    for name, N, K in (("w13", 2 * F, D), ("w2", D, F)):
        x = torch.randn(T, K, device="cuda", dtype=torch.bfloat16)
        W = torch.randn(E, N, K, device="cuda", dtype=torch.bfloat16) * 0.02
        dy = torch.randn(T, N, device="cuda", dtype=torch.bfloat16)
        xq, sx = M.quant_act_fp8_blk(x)
        dq, sd = M.quant_act_fp8_blk(dy)
        wq, wtq, sw, swt = M.quant_weight_fp8_blk(W)
        aq, sa = M.quant_t_fp8_seg(dy, off, poff, ld)
        bq, sb = M.quant_t_fp8_seg(x, off, poff, ld)
        out = torch.empty(E, N, K, device="cuda", dtype=torch.bfloat16)
        fl = 2.0 * T * N * K
        res = {"shape": name, "experts": E, "rows": T, "N": N, "K": K}
        for mode, fns in (
            ("fwd", {"reg": lambda: ops.grouped_gemm_fp8_blk(xq, sx, wq, sw, off),
                     "g8": lambda: ops.gemm8_fp8_blk(xq, sx, wq, sw, off)}),
            ("dX", {"reg": lambda: ops.grouped_gemm_fp8_blk(dq, sd, wtq, swt, off),
                    "g8": lambda: ops.gemm8_fp8_blk(dq, sd, wtq, swt, off)}),
            ("dW", {"reg": lambda: ops.wgrad_fp8_blk(aq, sa, bq, sb, poff, out, False),
                    "g8": lambda: ops.wgrad8_fp8_blk(aq, sa, bq, sb, poff, out, False)}),
        ):
            med = ab(fns, a.iters, a.rounds)
            res[mode] = {k: round(fl / v / 1e9) for k, v in med.items()}
        bf = ab({"bf16": lambda: M.grouped_gemm(x, W, off, 0)}, a.iters, 2)["bf16"]
        res["fwd"]["bf16_g8"] = round(fl / bf / 1e9)
        print(json.dumps(res), flush=True)
        del x, W, dy, xq, dq, wq, wtq, aq, bq, out
    n = a.dense
    if n:
        x = torch.randn(n, n, device="cuda", dtype=torch.bfloat16)
        W = torch.randn(1, n, n, device="cuda", dtype=torch.bfloat16) * 0.02
        o1 = torch.tensor([0, n], dtype=torch.int32, device="cuda")
        xq, sx = M.quant_act_fp8_blk(x)
        wq, _, sw, _ = M.quant_weight_fp8_blk(W)
        med = ab({"reg": lambda: ops.grouped_gemm_fp8_blk(xq, sx, wq, sw, o1),
                  "g8": lambda: ops.gemm8_fp8_blk(xq, sx, wq, sw, o1)}, a.iters, a.rounds)
        print(json.dumps({"shape": f"dense {n}^3", **{k: round(2.0 * n ** 3 / v / 1e9) for k, v in med.items()}}),
              flush=True)


if __name__ == "__main__":
    main()
