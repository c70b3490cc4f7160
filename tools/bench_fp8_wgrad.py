"""Routed-expert weight gradient at DeepSeek-V3 widths: bf16 grouped dW (8-phase kernel, mode 2)
vs the fp8 path (two transposed 128-token-tile quantizations + block-scaled Wgrad GEMM), ABBA.
    python tools/bench_fp8_wgrad.py [--experts 32] [--rows 32768] [--dim 7168] [--ffn 2048]"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from solvingpapers_amd.ops import _ext  # noqa: E402
from solvingpapers_amd.ops import moe as M  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--experts", type=int, default=32)
    ap.add_argument("--rows", type=int, default=32768, help="routed rows (tokens x top-k)")
    ap.add_argument("--dim", type=int, default=7168)
    ap.add_argument("--ffn", type=int, default=2048)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=4)
    a = ap.parse_args()
    assert _ext.load(), "HIP extension missing"
    E, T, D, F = a.experts, a.rows, a.dim, a.ffn
    g = torch.Generator().manual_seed(0)
    cnt = torch.multinomial(torch.ones(E), T, replacement=True, generator=g).bincount(minlength=E)
    off = torch.cat([torch.zeros(1, dtype=torch.long), cnt.cumsum(0)]).int().cuda()
    res = {}
    for name, N, K in (("w13", 2 * F, D), ("w2", D, F)):
        dy = torch.randn(T, N, device="cuda", dtype=torch.bfloat16)
        x = torch.randn(T, K, device="cuda", dtype=torch.bfloat16)
        out = torch.empty(E, N, K, device="cuda", dtype=torch.float32)
        outb = torch.empty(E, N, K, device="cuda", dtype=torch.bfloat16)
        ld = (T + E * 127 + 127) // 128 * 128

        def bf16():
            M.grouped_gemm(dy, x, off, 2, out=outb)

        poff0 = M.padded_offsets(off)
        xq0 = M.quant_t_fp8_seg(x, off, poff0, ld)       # saved by the forward in the model

        def fp8():
            poff = M.padded_offsets(off)
            aq, sa, _, _ = M.quant_t_fp8_seg(dy, off, poff, ld, rows=True)   # + the dX row image
            M.wgrad_fp8_blk(aq, sa, xq0[0], xq0[1], poff, outb, False)

        def fp8_gemm():
            M.wgrad_fp8_blk(aq0, sa0, xq0[0], xq0[1], poff0, outb, False)
        aq0, sa0 = M.quant_t_fp8_seg(dy, off, poff0, ld)

        def tm(fn):
            fn()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            s.record()
            for _ in range(a.iters):
                fn()
            e.record()
            torch.cuda.synchronize()
            return s.elapsed_time(e) / a.iters

        t = {"bf16": [], "fp8": [], "gemm": []}
        fns = {"bf16": bf16, "fp8": fp8, "gemm": fp8_gemm}
        for r in range(a.rounds):
            for k in (("bf16", "fp8", "gemm") if r % 2 == 0 else ("gemm", "fp8", "bf16")):
                t[k].append(tm(fns[k]))
        fl = 2.0 * T * N * K
        med = {k: statistics.median(v) for k, v in t.items()}
        res[name] = {"N": N, "K": K, "bf16_ms": round(med["bf16"], 3), "fp8_ms": round(med["fp8"], 3),
                     "bf16_tflops": round(fl / med["bf16"] / 1e9, 1), "fp8_tflops_incl_quant": round(fl / med["fp8"] / 1e9, 1),
                     "fp8_gemm_only_tflops": round(fl / med["gemm"] / 1e9, 1),
                     "speedup": round(med["bf16"] / med["fp8"], 3)}
    print(json.dumps({"experts": E, "rows": T, **res}), flush=True)


if __name__ == "__main__":
    main()
