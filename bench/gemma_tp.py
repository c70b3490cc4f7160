#!/usr/bin/env python
"""Gemma-7B-shape (MQA, 1 KV head) bf16 training tokens/s with tensor parallelism over all
ranks (BASELINE.json config #4: TP=8 on one node). Sequence parallel by default: each layer
boundary is a reduce-scatter of the row-parallel output followed by an all-gather of the residual
shard (norms and the MQA K/V projection on the gathered sequence), vocab-parallel embedding + CE;
two chunks -- the micro-batches of an even --accum (Gemma.forward_pair), else the batch or
sequence halves -- overlap each other's boundaries (models/gemma.py _forward_sp_pair).
``[torchrun --nproc-per-node N ...] python bench/gemma_tp.py --steps K --warmup W [--layers L] [--accum 2]``"""
from __future__ import annotations

import argparse
import os

import torch
import torch.distributed as dist

from common import PEAK_BF16, report, sdist, timed
from solvingpapers_amd.models import gemma
from solvingpapers_amd.train.optim import FlatAdamW
from solvingpapers_amd.utils.flat import FlatParams


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--seq", type=int, default=8192)
    ap.add_argument("--batch", type=int, default=1,
                    help="sequences per step (even under SP: the chunk pair splits the batch, not each sequence)")
    ap.add_argument("--accum", type=int, default=1,
                    help="micro-batches of --batch sequences per step; even: run in overlapped pairs (Gemma.forward_pair)")
    ap.add_argument("--layers", type=int, default=None)
    ap.add_argument("--no-sp", dest="sp", action="store_false",
                    help="plain Megatron TP (default: sequence parallelism inside the TP group)")
    ap.add_argument("--no-pipeline", dest="pipeline", action="store_false",
                    help="no overlapped pairs (default under SP: two chunks -- the micro-batches of an even "
                         "--accum, else batch / sequence halves -- whose layer-boundary reduce-scatter -> "
                         "all-gather runs under the other chunk's compute)")
    ap.add_argument("--no-opt-overlap", action="store_true", help="run AdamW on the compute stream")
    ap.add_argument("--gemm-table", default="auto",
                    help="TunableOp GEMM table to look up (default tuning/tunableop_gemma7b.csv, tuned at the TP=1 "
                         "T=8192 shapes: +0.6 %% ABBA, profiles/r4_gemma_gemm_table_abba.txt); 'none' disables")
    a = ap.parse_args()
    info = sdist.init_distributed()
    tuned = False
    if a.gemm_table != "none":   # after init: the device is set, so every rank loads it on its own GPU
        from solvingpapers_amd.utils.tuning import ROOT, load_gemm_tuning
        path = os.path.join(ROOT, "tuning", "tunableop_gemma7b.csv") if a.gemm_table == "auto" else a.gemm_table
        tuned = load_gemm_tuning(path)
        assert tuned or a.gemm_table == "auto" or not torch.cuda.is_available(), a.gemm_table
    world, dev = info.world_size, info.device
    kw = {"max_seq_len": a.seq}
    if a.layers:
        kw["n_layers"] = a.layers
    c = gemma.config("gemma_7b_mqa", **kw)
    tp = dist.group.WORLD if world > 1 else None
    m = gemma.Gemma(c, device=dev, dtype=torch.bfloat16, tp_group=tp, seed=1, sequence_parallel=a.sp,
                    tp_pipeline=a.pipeline)
    flat = FlatParams(m, groups=m.param_groups(), grad_dtype=torch.bfloat16)
    # global grad norm: TP-sharded squares summed over the group, replicated params counted once
    opt = FlatAdamW(flat, lr=3e-4, betas=(0.9, 0.95), weight_decay=0.1, max_grad_norm=1.0, tp_group=tp)
    # AdamW (HBM-bound) on a side stream, each layer's forward waiting only for its own bucket: the
    # update overlaps the next step's compute-bound forward (as bench.py)
    overlap = dev.type == "cuda" and not a.no_opt_overlap
    if overlap:
        m.param_wait_cb = flat.group_waiter(m.param_groups())
    g = torch.Generator(device=dev).manual_seed(11)                 # same tokens on every TP rank
    last = [None]

    def step():
        opt.zero_grad()
        pair = a.accum % 2 == 0 and m.tp_pipeline
        for i in range(a.accum // 2 if pair else a.accum):
            t = torch.randint(0, c.vocab_size, (a.batch, a.seq + 1), device=dev, generator=g)
            if pair:
                u = torch.randint(0, c.vocab_size, (a.batch, a.seq + 1), device=dev, generator=g)
                loss = m.forward_pair(t[:, :-1], t[:, 1:], u[:, :-1], u[:, 1:])
            else:
                loss = m(t[:, :-1], t[:, 1:])
            loss.backward()
        m.sync_sequence_parallel_grads()
        opt.step(overlap=overlap)
        last[0] = loss / 2 if pair else loss

    el = timed(step, a.steps, a.warmup)
    tok_s = a.accum * a.batch * a.seq * a.steps / el                 # accum x batch sequences per step for the TP group
    tf = tok_s * m.flops_per_token(a.seq) / world / 1e12
    report("training tokens/sec, Gemma-7B-shape MQA bf16 (TP)", tok_s, "tokens/s", a.steps, a.warmup, el,
           {"model": "gemma_7b_mqa" + (f"-L{a.layers}" if a.layers else ""), "global_batch": a.accum * a.batch, "seq_len": a.seq,
            "parallelism": f"tp{world}" + ("-sp" if m.sp else "") + ("-pair" if m.sp and m.tp_pipeline else "")}, tflops_per_gpu=round(tf, 1), mfu_vs_2_5PF=round(tf * 1e12 / PEAK_BF16, 4), gemm_table=tuned,
           loss=round(float(last[0].detach()), 4))
    sdist.cleanup()


if __name__ == "__main__":
    main()
