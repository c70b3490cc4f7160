#!/usr/bin/env python
"""Numerics of the headline's bf16 gradient accumulation (VERDICT r4 "next" item 5).

bench.py keeps the flat gradient buffer in bf16: every micro-batch's weight-gradient GEMM
reads the running sum, adds its fp32 accumulator and rounds once to bf16 (hipBLASLt beta=1 /
the wgrad8 kernels), so K micro-batches cost K roundings instead of the one the fp32 main-grad
path (--grad-fp32) pays when the optimizer reads it. Two measurements:

``--mode grad``  LLaMA3-8B widths (D4096, H32/8, FFN 14336, V 128256) at --layers L, T 8192,
    accum 4, the same weights and batches twice: flat gradient with bf16 accumulation vs fp32
    accumulation. Reports, per parameter and overall, ||g_bf16 - g_fp32|| / ||g_fp32||, next to
    the floor ||bf16(g_fp32) - g_fp32|| / ||g_fp32|| (the error a bf16 copy of the exact sum has
    anyway) -- their ratio says how many "roundings" the accumulation really costs -- the
    cosine of the two gradients and the fraction of elements whose sign (AdamW's first-step
    update direction) flips.

``--mode curve``  a ~110M-parameter LLaMA (D768, L12, H12/4, V 8192) on B8's learnable synthetic
    corpus (noisy affine token chain, bench/parity.py run_b8), accum 4 x (4 x 512) tokens, AdamW +
    warmup/cosine, --steps optimizer steps per arm: bf16 grads (seed s), fp32 grads (seed s), and
    bf16 grads with a different data/init seed (the run-to-run noise scale). Prints one JSON line
    per arm with the loss every 10 steps, then a summary line.

``--mode ring``  the DP reduction at N ranks: N ranks' bf16-accumulated flat
    gradients at LLaMA3-8B widths (same weights, different batches), reduced three ways against the
    exact fp64 average of what the ranks hold: RCCL's ring all-reduce in bf16 (reduce-scatter in ring
    chunk order: every hop reads the running bf16 partial, adds its own value in fp32 and rounds to
    bf16 -> N-1 roundings per element; ReduceOp.AVG's 1/N pre-scale is exact for N = 2^k; the
    all-gather only copies), the all-to-all reduce-scatter (every rank receives all N shards of its
    chunk and sums them in fp32 -> one rounding; parallel/data_parallel.py reduce="a2a"), and fp32
    buckets. Reports each error as a multiple of one bf16 rounding of the exact average.

The reference keeps fp32 gradients (deepseekv3/deepseekv3.ipynb:2411,2427-2447 under fp16
autocast; llama3/LLaMA-jax.ipynb:993-1001 trains in fp32).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from solvingpapers_amd.models import llama3  # noqa: E402
from solvingpapers_amd.train.optim import FlatAdamW  # noqa: E402
from solvingpapers_amd.utils.flat import FlatParams  # noqa: E402


def accumulated_grad(model, gdt, batches):
    """Flat gradient of sum_i loss_i / len(batches) with a ``gdt`` accumulation buffer."""
    flat = FlatParams(model, groups=model.param_groups(), grad_dtype=gdt, align=64)
    flat.zero_grad()
    n = len(batches)
    for x, y in batches:
        (model(x, y) / n).backward()
    torch.cuda.synchronize()
    return flat


def grad_error(layers=2, T=8192, accum=4, seed=1234):
    """Relative error of the bf16-accumulated flat gradient against the fp32 accumulation."""
    dev = torch.device("cuda")
    cfg = llama3.config("llama3_8b", n_layers=layers, max_seq_len=T)
    model = llama3.Llama3(cfg, device=dev, dtype=torch.bfloat16, seed=seed)
    g = torch.Generator(device=dev).manual_seed(seed + 1)
    batches = []
    for _ in range(accum):
        t = torch.randint(0, cfg.vocab_size, (1, T + 1), device=dev, generator=g)
        batches.append((t[:, :-1], t[:, 1:]))
    f32 = accumulated_grad(model, torch.float32, batches)
    g32 = f32.grad.clone()
    offs = [(n, f32.offsets[id(p)], p.numel()) for n, p in zip(f32.names, f32.params)]
    del f32
    b16 = accumulated_grad(model, torch.bfloat16, batches)
    g16 = b16.grad.float()
    del b16
    rows = []
    for name, o, n in offs:
        a, b = g32[o:o + n], g16[o:o + n]
        na = a.norm().item()
        err = (b - a).norm().item() / max(na, 1e-30)
        floor = (a.bfloat16().float() - a).norm().item() / max(na, 1e-30)
        rows.append({"param": name, "numel": n, "rel_err": err, "bf16_floor": floor,
                     "ratio": err / max(floor, 1e-30)})
    tot = (g16 - g32).norm().item() / g32.norm().item()
    floor = (g32.bfloat16().float() - g32).norm().item() / g32.norm().item()
    # AdamW's first step direction is sign-like (m / sqrt(v) = g / |g|): the fraction of
    # elements whose update sign flips is what the optimizer would see
    nz = g32 != 0
    flips = ((torch.sign(g16) != torch.sign(g32)) & nz).float().sum().item() / max(nz.sum().item(), 1)
    cos = torch.nn.functional.cosine_similarity(g16, g32, dim=0).item()
    return {"layers": layers, "T": T, "accum": accum, "rel_err": tot, "bf16_floor": floor,
            "ratio": tot / floor, "cosine": cos, "sign_flip_frac": flips,
            "worst": sorted(rows, key=lambda r: -r["ratio"])[:4]}


def ring_allreduce_bf16(xs, chunk_order=True):
    """Emulate RCCL's bf16 ring all-reduce (SUM) of the equal-shape bf16 tensors ``xs`` (one per
    rank): the buffer is cut into N chunks; chunk c's reduce-scatter starts at rank c+1 and walks the
    ring, each hop computing bf16(float(partial) + float(own)). Returns the bf16 result every rank
    holds after the all-gather."""
    N = len(xs)
    flat = [x.reshape(-1) for x in xs]
    n = flat[0].numel()
    out = torch.empty_like(flat[0])
    bounds = [n * c // N for c in range(N + 1)]
    for c in range(N):
        a, b = bounds[c], bounds[c + 1]
        order = [(c + 1 + i) % N for i in range(N)] if chunk_order else list(range(N))
        acc = flat[order[0]][a:b].clone()
        for r in order[1:]:
            acc = (acc.float() + flat[r][a:b].float()).to(torch.bfloat16)
        out[a:b] = acc
    return out.view_as(xs[0])


def a2a_reduce_bf16(xs):
    """The all-to-all reduce-scatter + all-gather (data_parallel reduce="a2a"): every shard summed in
    fp32 from the N received bf16 copies, rounded once."""
    acc = xs[0].float()
    for x in xs[1:]:
        acc += x.float()
    return acc.to(torch.bfloat16)


def ring_error(ranks=8, layers=2, T=8192, accum=4, seed=1234, chunk=1 << 26):
    """Relative errors of the N-rank DP average (ring bf16 / a2a bf16 / fp32 buckets) against the
    exact fp64 average of the ranks' bf16 gradients, and their ratio to one bf16 rounding."""
    dev = torch.device("cuda")
    cfg = llama3.config("llama3_8b", n_layers=layers, max_seq_len=T)
    model = llama3.Llama3(cfg, device=dev, dtype=torch.bfloat16, seed=seed)
    grads = []
    for r in range(ranks):
        g = torch.Generator(device=dev).manual_seed(seed + 101 * (r + 1))
        batches = []
        for _ in range(accum):
            t = torch.randint(0, cfg.vocab_size, (1, T + 1), device=dev, generator=g)
            batches.append((t[:, :-1], t[:, 1:]))
        f = accumulated_grad(model, torch.bfloat16, batches)
        grads.append(f.grad.clone())
        del f
    inv = 1.0 / ranks
    acc = {"ring": [0.0, 0.0], "a2a": [0.0, 0.0], "fp32": [0.0, 0.0], "floor": [0.0, 0.0]}
    n = grads[0].numel()
    nrm = 0.0
    for a in range(0, n, chunk):
        xs = [g[a:a + chunk] for g in grads]
        exact = torch.zeros(xs[0].shape, dtype=torch.float64, device=dev)
        for x in xs:
            exact += x.double()
        exact *= inv
        nrm += exact.square().sum().item()
        # ReduceOp.AVG pre-scales each input by 1/N (exact in bf16 for N = 2^k)
        pre = [(x.float() * inv).to(torch.bfloat16) for x in xs]
        outs = {"ring": ring_allreduce_bf16(pre), "a2a": a2a_reduce_bf16(pre),
                "fp32": sum(x.float() for x in xs) * inv, "floor": exact.to(torch.bfloat16)}
        for k, v in outs.items():
            acc[k][0] += (v.double() - exact).square().sum().item()
    nrm = math.sqrt(nrm)
    rel = {k: math.sqrt(v[0]) / nrm for k, v in acc.items()}
    fl = rel["floor"]
    return {"ranks": ranks, "layers": layers, "T": T, "accum": accum, "numel": n,
            "rel_err_ring_bf16": rel["ring"], "rel_err_a2a_bf16": rel["a2a"], "rel_err_fp32": rel["fp32"],
            "bf16_floor": fl, "ratio_ring": rel["ring"] / fl, "ratio_a2a": rel["a2a"] / fl,
            "ratio_fp32": rel["fp32"] / fl}


def corpus(V, n, dev, seed):
    """B8's learnable stream (bench/parity.py run_b8): 1024-token affine chains mod V with 10 %
    uniform noise tokens."""
    g = torch.Generator(device=dev).manual_seed(seed)
    noise = torch.rand(n, device=dev, generator=g) < 0.1
    draw = torch.randint(0, V, (n,), device=dev, generator=g)
    starts = torch.randint(0, V, (n // 1024, 1), device=dev, generator=g)
    c = ((torch.arange(1024, device=dev) * 48271 + starts) % V).reshape(-1)
    return torch.where(noise, draw, c)


def loss_curve(gdt, steps, seed, B=4, T=512, accum=4, lr=6e-4, every=10):
    dev = torch.device("cuda")
    cfg = llama3.config("llama3_8b", vocab_size=8192, dim=768, n_layers=12, n_heads=12, n_kv_heads=4,
                        ffn_hidden=2048, max_seq_len=T)
    model = llama3.Llama3(cfg, device=dev, dtype=torch.bfloat16, seed=seed)
    flat = FlatParams(model, groups=model.param_groups(), grad_dtype=gdt, align=64)
    opt = FlatAdamW(flat, lr=lr, betas=(0.9, 0.95), eps=1e-8, weight_decay=0.1, max_grad_norm=1.0)
    data = corpus(cfg.vocab_size, 1 << 22, dev, seed + 7)
    g = torch.Generator(device=dev).manual_seed(seed + 9)
    ar = torch.arange(T, device=dev)
    warm = max(steps // 20, 1)
    hist, t0 = [], time.time()
    for it in range(steps):
        lr_t = lr * (it + 1) / warm if it < warm else \
            0.1 * lr + 0.45 * lr * (1 + math.cos(math.pi * (it - warm) / max(steps - warm, 1)))
        opt.zero_grad()
        tot = torch.zeros((), device=dev)
        for _ in range(accum):
            i = torch.randint(0, data.numel() - T - 1, (B, 1), device=dev, generator=g) + ar
            loss = model(data[i], data[i + 1]) / accum
            loss.backward()
            tot += loss.detach()
        opt.step(lr=lr_t)
        if it % every == 0 or it == steps - 1:
            hist.append((it, round(tot.item(), 4)))
    return {"grad_dtype": str(gdt).replace("torch.", ""), "seed": seed, "steps": steps,
            "tokens_per_step": B * T * accum, "params": model.num_params(),
            "s": round(time.time() - t0, 1), "curve": hist}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", choices=["grad", "curve", "ring"], default="grad")
    ap.add_argument("--ranks", type=int, default=8)
    ap.add_argument("--layers", type=int, default=2)
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--seed", type=int, default=1)
    a = ap.parse_args()
    if a.mode == "ring":
        print(json.dumps(ring_error(ranks=a.ranks, layers=a.layers)), flush=True)
        return
    if a.mode == "grad":
        print(json.dumps(grad_error(layers=a.layers)), flush=True)
        return
    arms = [(torch.bfloat16, a.seed), (torch.float32, a.seed), (torch.bfloat16, a.seed + 100)]
    res = []
    for gdt, s in arms:
        r = loss_curve(gdt, a.steps, s)
        res.append(r)
        print(json.dumps(r), flush=True)
    tail = lambda r: sum(v for _, v in r["curve"][-5:]) / 5  # noqa: E731
    gap = [abs(x[1] - y[1]) for x, y in zip(res[0]["curve"], res[1]["curve"])]
    noise = [abs(x[1] - y[1]) for x, y in zip(res[0]["curve"], res[2]["curve"])]
    print(json.dumps({"summary": "loss-curve A/B", "final5_bf16": round(tail(res[0]), 4),
                      "final5_fp32": round(tail(res[1]), 4), "final5_bf16_seed2": round(tail(res[2]), 4),
                      "mean_abs_gap_bf16_vs_fp32": round(sum(gap) / len(gap), 4),
                      "mean_abs_gap_seed_noise": round(sum(noise) / len(noise), 4)}), flush=True)


if __name__ == "__main__":
    main()
