#!/usr/bin/env python
"""DeepSeek-V3-style (MLA + DeepSeekMoE) bf16 training tokens/s (BASELINE.json config #5,
SURVEY App. C): ``python bench/dsv3_train.py --steps K --warmup W [--layers L]``; under
torchrun with N>1 ranks the routed experts are expert-parallel over all N GPUs (EP=N,
all-to-all dispatch) and the dense parameters data-parallel (RCCL buckets)."""
from __future__ import annotations

import argparse
import os
import contextlib

import torch

from common import PEAK_BF16, report, sdist, timed
from solvingpapers_amd.models import deepseekv3 as ds
from solvingpapers_amd.parallel.data_parallel import DataParallel
from solvingpapers_amd.train.optim import FlatAdamW
from solvingpapers_amd.utils.flat import FlatParams


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--preset", default="dsv3_style")
    ap.add_argument("--layers", type=int, default=None)
    ap.add_argument("--seq", type=int, default=4096)
    ap.add_argument("--mb", type=int, default=2)
    ap.add_argument("--experts", type=int, default=None, help="routed experts (whole job; EP splits them)")
    ap.add_argument("--dense-layers", type=int, default=None)
    ap.add_argument("--accum", type=int, default=1, help="micro-batches accumulated per optimizer step")
    ap.add_argument("--fp8", action="store_true",
                    help="DeepSeek-V3 fp8 recipe: routed experts + dense projections in block-scaled e4m3")
    ap.add_argument("--fp8-experts-only", action="store_true", help="with --fp8: dense projections stay bf16")
    # DeepSeek-V3's own recipe (sec. 3.3.2) keeps the AdamW moments in bf16 next to fp32 master
    # weights; at 8K tokens per step the optimizer over 7.3B parameters is ~24 % of the
    # dsv3_style step with fp32 moments, so bf16 is the default here
    ap.add_argument("--bf16-moments", dest="bf16_moments", action="store_true", default=True,
                    help="AdamW moments in bf16 (DeepSeek-V3 sec. 3.3.2; fp32 master weights kept; default)")
    ap.add_argument("--fp32-moments", dest="bf16_moments", action="store_false", help="AdamW moments in fp32")
    ap.add_argument("--no-opt-overlap", action="store_true", help="run AdamW on the main stream")
    ap.add_argument("--no-pair", dest="pair", action="store_false",
                    help="with --accum even: run the micro-batches one by one instead of in layer-interleaved "
                         "pairs (DeepSeekV3.forward_pair: each EP all-to-all overlaps the other micro-batch)")
    ap.add_argument("--ep-capacity", type=float, default=None,
                    help="DSV3Config.ep_capacity (> 0: host-sync-free padded EP dispatch)")
    ap.add_argument("--gemm-table", default="auto",
                    help="TunableOp GEMM table to look up (default tuning/tunableop_<preset>.csv where one exists "
                         "and the bench runs at T 4096); 'none' disables")
    a = ap.parse_args()
    info = sdist.init_distributed()
    world, dev = info.world_size, info.device
    tuned = False
    if a.gemm_table != "none" and dev.type == "cuda":   # after init: every rank loads it on its own GPU
        from solvingpapers_amd.utils.tuning import ROOT, load_gemm_tuning
        path = a.gemm_table
        if path == "auto":
            path = os.path.join(ROOT, "tuning", f"tunableop_{a.preset}.csv")
            # depth and expert count leave every dense GEMM shape as it is; the sequence length does not
            path = path if a.seq == 4096 and os.path.exists(path) else None
        if path:
            tuned = load_gemm_tuning(path)
            assert tuned, path
    kw = {"block_size": a.seq}
    if a.layers:
        kw["n_layers"] = a.layers
    if a.experts:
        kw["n_experts"] = a.experts
    if a.dense_layers is not None:
        kw["n_dense_layers"] = a.dense_layers
    if a.fp8:
        kw["moe_fp8"] = True
        kw["fp8_linears"] = not a.fp8_experts_only
    c = ds.config(a.preset, **kw)
    # SPA_FORCE_COLLECTIVES=1 under a 1-rank torch.distributed.run: the EP exchanges, DP buckets and
    # routing-bias all-reduce go through RCCL at world size 1 (multi-GPU pre-flight on one GPU)
    multi = world > 1 or (sdist.force_collectives() and torch.distributed.is_initialized())
    if a.ep_capacity is not None:
        kw["ep_capacity"] = a.ep_capacity
        c = ds.config(a.preset, **kw)
    ep = torch.distributed.group.WORLD if multi else None
    m = ds.DeepSeekV3(c, device=dev, dtype=torch.bfloat16, seed=1, ep_group=ep)
    pair = a.pair and a.accum % 2 == 0
    flat = FlatParams(m, groups=m.param_groups(), grad_dtype=torch.bfloat16, align=64 * world)
    dp = DataParallel(m, flat) if multi else None
    opt = FlatAdamW(flat, lr=3e-4, betas=(0.9, 0.95), weight_decay=0.1, max_grad_norm=1.0, ep_group=ep,
                    moment_dtype=torch.bfloat16 if a.bf16_moments else torch.float32)
    overlap = not a.no_opt_overlap and torch.cuda.is_available()
    if overlap:   # AdamW per bucket on a side stream, each layer's forward waits for its bucket
        m.param_wait_cb = flat.group_waiter(m.param_groups())
    for l in m.moe_layers():
        l.balance_group = None
    gen = torch.Generator(device=dev).manual_seed(7 + info.rank)
    B, T = a.mb, a.seq
    last = [None]

    def step():
        opt.zero_grad()
        n = 2 if pair else 1
        for i in range(0, a.accum, n):
            t = [torch.randint(0, c.vocab_size, (B, T + 1), device=dev, generator=gen) for _ in range(n)]
            inner = dp is not None and i + n < a.accum
            with dp.no_sync() if inner else contextlib.nullcontext():
                if pair:
                    loss = m.forward_pair(t[0][:, :-1], t[0][:, 1:], t[1][:, :-1], t[1][:, 1:]) / a.accum
                else:
                    loss = m(t[0][:, :-1], t[0][:, 1:]) / a.accum
                loss.backward()
        if dp is not None:
            dp.finish_grad_sync()
        opt.step(overlap=overlap)
        last[0] = loss * a.accum / (2 if pair else 1)

    el = timed(step, a.steps, a.warmup)
    tok_s = world * B * T * a.accum * a.steps / el
    tf = tok_s * m.flops_per_token(T) / world / 1e12
    report("training tokens/sec, DeepSeek-V3-style MLA+MoE " + ("fp8 (e4m3 block-scaled GEMMs)" if a.fp8 else "bf16"),
           tok_s, "tokens/s", a.steps, a.warmup, el,
           {"model": a.preset + (f"-L{a.layers}" if a.layers else "") + (f"-E{a.experts}" if a.experts else "")
            + ("-fp8" if a.fp8 else ""), "global_batch": world * B * a.accum, "seq_len": T, "grad_accum": a.accum, "microbatch_pairs": pair, "adam_moments": "bf16" if a.bf16_moments else "fp32",
            "parallelism": f"ep{world}-dp{world}" + ("-forced-collectives" if world == 1 else "") if multi else "1gpu",
            "ep_capacity": c.ep_capacity,
            "params": m.num_params(),
            "active_params": m.num_params(active=True)},
           tflops_per_gpu=round(tf, 1), mfu_vs_2_5PF=round(tf * 1e12 / PEAK_BF16, 4), loss=round(float(last[0].detach()), 4),
           gemm_table=tuned)
    sdist.cleanup()


if __name__ == "__main__":
    main()
