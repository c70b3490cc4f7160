#!/usr/bin/env python
"""Headline benchmark: LLaMA3-8B-shape bf16 training tokens/s on 1..8 MI355X.

Contract (driver): ``python bench.py --gpus N --steps K --warmup W``; for N>1 it
runs one rank per GPU (RCCL over xGMI). Launched under ``torch.distributed.run`` it
uses that process group; launched directly with ``--gpus N > 1`` (no WORLD_SIZE in
the env) it starts ``torch.distributed.run --nproc-per-node N`` itself as a CHILD
process before anything touches the GPU, and exits with the child's exit code
(non-zero if any rank failed). ``n_gpus`` in the JSON is the live process group's
world size, next to the backend and the visible device count.
W untimed warmup steps, then EXACTLY K timed steps bracketed by barrier +
torch.cuda.synchronize() on both sides; the max elapsed over ranks is used and
rank 0 prints one JSON line. ``value`` = whole-job tokens/s (all GPUs).

A step is a full training step: forward, fused CE loss, backward (per-layer
RCCL gradient buckets overlapped with backward when N>1), grad-norm clip,
fused AdamW over the flat fp32 master/moment buffers. Synthetic token ids,
random-init weights of the LLaMA3-8B architecture (D4096 L32 H32 KV8 FFN14336
V128256), seq 8192, micro-batch 1 per GPU, 4 micro-batches accumulated per
optimizer step (weak scaling: global batch = 4N sequences = 32K tokens per GPU
per step). Every micro-batch runs its full forward + backward inside the timed
region; only the inner micro-batches skip the gradient all-reduce (no_sync) and
the last one launches it, so the per-step optimizer / grad-norm / all-reduce
cost (~40 ms on 1 GPU, more at N=8) is paid once per 32K tokens as in a real
LLaMA-scale run (global batches of millions of tokens). The accumulation sweep (round 1,
1 MI355X, profiles/r1_bench_accum_sweep.jsonl): accum 1: 18.6K tok/s, 2: 19.4K, 4: 20.35K,
8: 20.6K. The current figure is the driver's own run of this file (BENCH_rNN.json; history in
BASELINE.md).
"""
from __future__ import annotations

import argparse
import contextlib
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

BASELINE_TOKS = None  # BASELINE.json "published": {} -> no reference number for this config
PEAK_BF16 = 2.5e15


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def self_launch(n: int, argv) -> int:
    """Start ``torch.distributed.run`` with n ranks of this script as a child process (no
    exec: nothing here has touched the GPU, and the parent only waits) and return its exit
    code. Rendezvous on 127.0.0.1 (the container hostname may not resolve)."""
    env = dict(os.environ)
    # RCCL moves buffers between the ranks' GPUs through HIP IPC; on these hosts the driver only
    # supports dmabuf IPC (HSA_ENABLE_IPC_MODE_LEGACY=0), which the harness already exports. Only
    # default it when the caller's environment says nothing, never override a set value.
    if "HSA_ENABLE_IPC_MODE_LEGACY" not in env:
        env["HSA_ENABLE_IPC_MODE_LEGACY"] = "0"
    env["SPA_BENCH_SELF"] = "1"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__), *argv]
    print(f"bench.py: launching {n} ranks: {' '.join(cmd)}", file=sys.stderr, flush=True)
    return subprocess.call(cmd, env=env, cwd=ROOT)


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--model", default="llama3_8b")
    ap.add_argument("--seq", type=int, default=8192)
    ap.add_argument("--mb", type=int, default=1, help="micro-batch per GPU")
    ap.add_argument("--accum", type=int, default=4, help="micro-batches accumulated per optimizer step")
    ap.add_argument("--zero1", action="store_true")
    ap.add_argument("--layers", type=int, default=None, help="override layer count (NOT for headline runs)")
    ap.add_argument("--no-opt-overlap", action="store_true", help="run AdamW on the main stream")
    ap.add_argument("--grad-fp32", action="store_true", default=os.environ.get("SPA_GRAD_FP32") == "1",
                    help="fp32 main gradients (accumulated and all-reduced in fp32) instead of bf16 "
                         "(env SPA_GRAD_FP32=1)")
    ap.add_argument("--gemm-table", default=None, help="TunableOp GEMM table (default tuning/tunableop_llama8b.csv; "
                    "SPA_GEMM_TUNING=0 disables)")
    a = ap.parse_args(argv)
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return self_launch(a.gpus, argv)
    return run(a)


def run(a):
    import torch
    import torch.distributed as tdist

    from solvingpapers_amd.models import llama3
    from solvingpapers_amd.parallel import dist as sdist
    from solvingpapers_amd.parallel.data_parallel import DataParallel
    from solvingpapers_amd.train.optim import FlatAdamW
    from solvingpapers_amd.utils.flat import FlatParams
    from solvingpapers_amd.utils.prof import annotate
    from solvingpapers_amd.utils.tuning import load_gemm_tuning

    info = sdist.init_distributed()
    world = tdist.get_world_size() if tdist.is_initialized() else 1   # the LIVE group
    if world != a.gpus and info.is_main:
        print(f"warning: --gpus {a.gpus} but the process group has {world} ranks; reporting {world}",
              file=sys.stderr)
    dev = info.device
    cuda = dev.type == "cuda"

    def sync():
        if cuda:
            torch.cuda.synchronize()
    torch.backends.cuda.matmul.allow_tf32 = False
    tuned = load_gemm_tuning(a.gemm_table) if cuda else False

    kw = {} if a.layers is None else {"n_layers": a.layers}
    cfg = llama3.config(a.model, max_seq_len=a.seq, **kw)
    dtype = torch.bfloat16 if cuda else torch.float32
    model = llama3.Llama3(cfg, device=dev, dtype=dtype, seed=1234)
    gdt = torch.float32 if a.grad_fp32 else dtype
    flat = FlatParams(model, groups=model.param_groups(), grad_dtype=gdt, align=64 * world)
    # SPA_FORCE_COLLECTIVES=1 under a 1-rank torch.distributed.run drives the DP buckets / ZeRO-1
    # through RCCL at world size 1 (the multi-GPU pre-flight, profiles/r6_rccl_preflight.txt)
    multi = world > 1 or (sdist.force_collectives() and tdist.is_initialized())
    dp = DataParallel(model, flat, zero1=a.zero1) if multi else None
    if dp is not None:
        dp.broadcast_params(0)
    shard = (dp.shard_ranges(), None) if (dp is not None and a.zero1) else None
    opt = FlatAdamW(flat, lr=3e-4, betas=(0.9, 0.95), eps=1e-8, weight_decay=0.1, max_grad_norm=1.0, shard=shard)
    overlap = cuda and not a.no_opt_overlap and not a.zero1
    if overlap:
        model.param_wait_cb = flat.group_waiter(model.param_groups())

    gen = torch.Generator(device=dev).manual_seed(1000 + info.rank)
    V, T, B = cfg.vocab_size, a.seq, a.mb

    def batch():
        t = torch.randint(0, V, (B, T + 1), device=dev, generator=gen)
        return t[:, :-1], t[:, 1:]

    last_loss = [None]

    def step():
        opt.zero_grad()
        for i in range(a.accum):
            x, y = batch()
            sync = (i == a.accum - 1)
            with (dp.no_sync() if (dp is not None and not sync) else contextlib.nullcontext()):
                with annotate("forward"):
                    loss = model(x, y) / a.accum
                with annotate("backward"):
                    loss.backward()
        if dp is not None:
            with annotate("grad_sync"):
                dp.finish_grad_sync()
        with annotate("optimizer"):
            opt.step(overlap=overlap)
        if dp is not None:
            dp.gather_params()
        last_loss[0] = loss

    for _ in range(a.warmup):
        step()
    sdist.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    sync()
    sdist.barrier()
    t1 = time.perf_counter()
    elapsed = sdist.all_reduce_max(t1 - t0)
    loss_v = float(last_loss[0].item()) * a.accum

    tokens = world * B * T * a.accum * a.steps
    tok_s = tokens / elapsed
    flops_tok = model.flops_per_token(T)
    tflops_gpu = tok_s * flops_tok / world / 1e12
    if info.is_main:
        out = {
            "metric": "training tokens/sec, LLaMA3-8B-shape bf16",
            "value": round(tok_s, 2),
            "unit": "tokens/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(elapsed / a.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": (tok_s / BASELINE_TOKS) if BASELINE_TOKS else None,
            "dtype": "bf16" if cuda else "fp32",
            "data": "synthetic (random token ids, random-init weights)",
            "config": {
                "model": a.model if a.layers is None else f"{a.model}-L{a.layers}",
                "global_batch": world * B * a.accum,
                "seq_len": T,
                "parallelism": f"dp{world}" + ("-zero1" if a.zero1 else "") + ("-forced-collectives" if multi and world == 1 else ""),
                "micro_batch": B,
                "grad_accum": a.accum,
                "params": model.num_params(),
            },
            "tflops_per_gpu": round(tflops_gpu, 1),
            "mfu_vs_2.5PF": round(tflops_gpu * 1e12 / PEAK_BF16, 4),
            "gemm_table": tuned,
            "loss": round(loss_v, 4),
            "mem_gb": round(torch.cuda.max_memory_allocated() / 1e9, 1) if cuda else None,
            # device-wide use at the end (torch's pool + RCCL / hipBLASLt / runtime buffers)
            "dev_mem_used_gb": round((lambda f, t: (t - f) / 1e9)(*torch.cuda.mem_get_info()), 1) if cuda else None,
            "dp_reduce": dp.reduce if dp is not None else None,
            "world_size": world,
            "backend": tdist.get_backend() if tdist.is_initialized() else "none",
            "device_count": torch.cuda.device_count() if cuda else 0,
            "grad_dtype": str(gdt).replace("torch.", ""),
            "streamk_data_parallel": os.environ.get("TENSILE_STREAMK_DATA_PARALLEL"),
            # the communication / runtime knobs of this run (RCCL, HIP IPC, hipBLASLt, torch c10d)
            "env": {k: v for k, v in sorted(os.environ.items())
                    if k.startswith(("NCCL_", "RCCL_", "TORCH_NCCL_", "TENSILE_", "HSA_ENABLE_IPC", "GPU_MAX_HW_QUEUES",
                                     "PYTORCH_TUNABLEOP", "SPA_"))},
            "launcher": "bench.py self-launch" if os.environ.get("SPA_BENCH_SELF") else
                        ("torch.distributed.run" if "TORCHELASTIC_RUN_ID" in os.environ else "direct"),
        }
        print(json.dumps(out), flush=True)
    sdist.cleanup()
    return 0


if __name__ == "__main__":
    sys.exit(main())
