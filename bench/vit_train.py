#!/usr/bin/env python
"""ViT-B/16 bf16 training images/s, data parallel over RCCL (BASELINE.json config #3,
SURVEY App. C: 224^2, patch 16, D768, L12, H12, MLP 3072). Per-layer gradient buckets
all-reduced during backward; fused AdamW over the flat buffers.
``[torchrun --nproc-per-node N ...] python bench/vit_train.py --steps K --warmup W``"""
from __future__ import annotations

import argparse
import os

import torch

from common import PEAK_BF16, report, sdist, timed
from solvingpapers_amd.models import vit
from solvingpapers_amd.ops import cross_entropy
from solvingpapers_amd.parallel.data_parallel import DataParallel
from solvingpapers_amd.train.optim import FlatAdamW
from solvingpapers_amd.utils.flat import FlatParams


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--mb", type=int, default=256, help="images per GPU per step")
    ap.add_argument("--gemm-table", default="auto",
                    help="TunableOp GEMM table to look up (default tuning/tunableop_vit_b16.csv, tuned at these "
                         "shapes: +2.0 %% B N N B, profiles/r5_vit_gemm_table_abba.txt); 'none' disables")
    ap.add_argument("--graph", action="store_true",
                    help="capture the whole training step (fwd + bwd + AdamW) in one HIP graph and replay it "
                         "(measured 1.3 %% slower than eager at batch 256: the step is not launch bound, "
                         "profiles/r5_vit_gemm_table_abba.txt)")
    a = ap.parse_args()
    info = sdist.init_distributed()
    tuned = False
    if a.gemm_table != "none" and info.device.type == "cuda":   # after init: every rank loads it on its own GPU
        from solvingpapers_amd.utils.tuning import ROOT, load_gemm_tuning
        path = os.path.join(ROOT, "tuning", "tunableop_vit_b16.csv") if a.gemm_table == "auto" else a.gemm_table
        tuned = load_gemm_tuning(path)
        assert tuned or a.gemm_table == "auto", path
    world, dev = info.world_size, info.device
    c = vit.config("vit_b16")
    m = vit.ViT(c, device=dev, dtype=torch.bfloat16)
    flat = FlatParams(m, groups=m.param_groups(), grad_dtype=torch.bfloat16, align=64 * world)
    dp = DataParallel(m, flat) if world > 1 else None
    if dp is not None:
        dp.broadcast_params()
    graph = a.graph and world == 1 and dev.type == "cuda"
    opt = FlatAdamW(flat, lr=1e-3, betas=(0.9, 0.999), weight_decay=0.05, max_grad_norm=1.0, graph_safe=graph)
    g = torch.Generator(device=dev).manual_seed(3 + info.rank)
    x = torch.randn(a.mb, 3, 224, 224, device=dev, dtype=torch.bfloat16, generator=g)
    y = torch.randint(0, 1000, (a.mb,), device=dev, generator=g)
    last = [None]

    def step():
        opt.zero_grad()
        loss = cross_entropy(m(x), y)
        loss.backward()
        if dp is not None:
            dp.finish_grad_sync()
        opt.step()
        last[0] = loss

    if graph:
        from solvingpapers_amd.utils.graphs import StepGraph
        step = StepGraph(step, warmup=2).replay
    el = timed(step, a.steps, a.warmup)
    ips = world * a.mb * a.steps / el
    n = sum(p.numel() for p in m.parameters())
    tokens = c.num_patches + 1
    flops_img = 6 * n * tokens + 12 * c.transformer_blocks * c.embedding_dim * tokens * tokens
    tf = ips * flops_img / world / 1e12
    report("training images/sec, ViT-B/16 bf16", ips, "images/s", a.steps, a.warmup, el,
           {"model": "vit_b16", "global_batch": world * a.mb, "seq_len": tokens, "parallelism": f"dp{world}",
            "params": n}, tflops_per_gpu=round(tf, 1), mfu_vs_2_5PF=round(tf * 1e12 / PEAK_BF16, 4),
           loss=round(float(last[0].detach()), 4), gemm_table=tuned, hip_graph=graph)
    sdist.cleanup()


if __name__ == "__main__":
    main()
