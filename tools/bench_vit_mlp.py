"""ViT-B/16 MLP block (T = 256 x 197 tokens, 768 -> 3072 -> 768, GELU) fwd + bwd: the fused
8-phase-kernel epilogues (ops/linear.py _MLPFn) against library GEMMs + separate activation /
bias passes, interleaved ABBA rounds in one process.
    python tools/bench_vit_mlp.py [--tokens 50432] [--iters 20] [--rounds 4]"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from solvingpapers_amd.ops import _ext  # noqa: E402
import importlib  # noqa: E402

L = importlib.import_module("solvingpapers_amd.ops.linear")   # (ops.linear is also a function)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=50432)
    ap.add_argument("--dim", type=int, default=768)
    ap.add_argument("--hidden", type=int, default=3072)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=4)
    a = ap.parse_args()
    assert _ext.load(), "HIP extension missing"
    T, D, F = a.tokens, a.dim, a.hidden
    dev = "cuda"
    x = (torch.randn(T, D, device=dev) * 0.5).bfloat16().requires_grad_()
    w1 = (torch.randn(F, D, device=dev) * D ** -0.5).bfloat16().requires_grad_()
    b1 = torch.zeros(F, device=dev, dtype=torch.bfloat16, requires_grad=True)
    w2 = (torch.randn(D, F, device=dev) * F ** -0.5).bfloat16().requires_grad_()
    b2 = torch.zeros(D, device=dev, dtype=torch.bfloat16, requires_grad=True)
    g = torch.randn(T, D, device=dev, dtype=torch.bfloat16)

    def run(fused, bwd=True):
        L.MLP_EPI = fused
        y = L.mlp(x, w1, b1, w2, b2, "gelu")
        if bwd:
            y.backward(g)
        return y

    def timed(fused, bwd):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        run(fused, bwd)
        torch.cuda.synchronize()
        s.record()
        for _ in range(a.iters):
            if bwd:
                run(fused, True)
            else:
                with torch.no_grad():
                    run(fused, False)
        e.record()
        torch.cuda.synchronize()
        return s.elapsed_time(e) / a.iters

    # numerics: fused vs unfused outputs / grads
    outs = {}
    for f in (True, False):
        for p in (x, w1, b1, w2, b2):
            p.grad = None
        y = run(f)
        outs[f] = [y.float()] + [p.grad.float() for p in (x, w1, b1, w2, b2)]
    diffs = [((u - v).norm() / v.norm()).item() for u, v in zip(outs[True], outs[False])]
    res = {k: [] for k in ("fused_fwd", "lib_fwd", "fused_fb", "lib_fb")}
    for r in range(a.rounds):
        order = [(True, "fused"), (False, "lib")] if r % 2 == 0 else [(False, "lib"), (True, "fused")]
        for f, name in order:
            res[name + "_fwd"].append(timed(f, False))
            res[name + "_fb"].append(timed(f, True))
    med = {k: round(statistics.median(v), 4) for k, v in res.items()}
    fl = 2 * T * D * F * 2
    print(json.dumps({"shape": [T, D, F], "ms": med, "fwd_tflops_fused": round(fl / med["fused_fwd"] / 1e9, 1),
                      "fwd_tflops_lib": round(fl / med["lib_fwd"] / 1e9, 1),
                      "fb_speedup": round(med["lib_fb"] / med["fused_fb"], 3),
                      "rel_diff_fused_vs_lib": [float(f"{d:.2e}") for d in diffs]}), flush=True)


if __name__ == "__main__":
    main()
