#!/usr/bin/env python
"""Same-config parity runs on MI355X (BASELINE.md "Same-config parity runs"): the
reference's own model configs (SURVEY App. B presets) timed and trained here, next to
the numbers the reference published on Tesla T4s.

  B1  LLaMA-tiny training tok/s    (llama3_ref: 2L d256 4h/2kv T128 B16, SGD 3e-4)  ref 29.0K tok/s (1xT4 fp32)
  B5  GPT-tiny training tok/s      (gpt_ref: 8L d256 1 head T256 B128, AdamW)        ref 16.2K tok/s (1xT4 fp32)
  B9  DeepSeek-V3-tiny tok/s       (dsv3_ref: 6L d512 T256 B16, AdamW, dropout .1)   ref 5.3K tok/s (2xT4 fp16)
  B13 Gemma-tiny tok/s             (gemma_ref: 12L d768, 2 q-heads x 768 over 1 K/V head, T128 B64,
                                    AdamW 2.5e-4, dropout .1; the reference recorded no throughput)
  B14 ViT-MNIST test accuracy, B15 AE MSE, B16 VAE loss, B17 KD student accuracy: trained
      with the reference epochs on synthetic MNIST-like digits (no dataset access) —
      quality parity unpinned, reported for completeness with wall-clock.

Throughput runs use synthetic token ids; ``--graph`` captures the whole training step
(forward + backward + optimizer) in one HIP graph (these tiny configs are launch-bound).
Prints one JSON line per run. ``python bench/parity.py [--which B1,B5,B9,B14,...]``
"""
from __future__ import annotations

import argparse
import json
import time

import torch

from common import sdist

REF = {"B1": 29.0e3, "B5": 16.2e3, "B9": 5.3e3, "B13": None, "B14": 97.25, "B15": 0.012954, "B16": 13881.32, "B17": 97.50}


def _lm_throughput(tag, model, flat, opt, V, B, T, steps, warmup, dtype_name, graph):
    from solvingpapers_amd.utils.graphs import StepGraph
    dev = flat.device
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randint(0, V, (B, T), device=dev, generator=g)
    y = torch.randint(0, V, (B, T), device=dev, generator=g)
    out = {}

    def step():
        opt.zero_grad()
        loss = model(x, y)
        loss.backward()
        opt.step()
        out["loss"] = loss

    run = StepGraph(step, warmup=2).replay if graph else step  # opt built graph_safe below
    for _ in range(warmup):
        x.random_(0, V, generator=g)
        run()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        run()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    tok_s = B * T * steps / el
    print(json.dumps({"run": tag, "metric": "training tokens/sec", "value": round(tok_s, 1), "unit": "tokens/s",
                      "reference": REF[tag], "vs_reference": round(tok_s / REF[tag], 2) if REF[tag] else None,
                      "dtype": dtype_name,
                      "ms_per_step": round(el / steps * 1e3, 3), "hip_graph": graph,
                      "loss": round(float(out["loss"].detach()), 4), "n_gpus": 1}), flush=True)


def run_b1(a, dev, dt, name):
    from solvingpapers_amd.models import llama3
    from solvingpapers_amd.train.optim import FlatSGD
    from solvingpapers_amd.utils.flat import FlatParams
    c = llama3.config("llama3_ref")
    m = llama3.Llama3(c, device=dev, dtype=dt, seed=0)
    flat = FlatParams(m, groups=m.param_groups())
    opt = FlatSGD(flat, lr=3e-4, graph_safe=a.graph)
    _lm_throughput("B1", m, flat, opt, c.vocab_size, 16, 128, a.steps, a.warmup, name, a.graph)


def run_b5(a, dev, dt, name):
    from solvingpapers_amd.models import gpt
    from solvingpapers_amd.train.optim import FlatAdamW
    from solvingpapers_amd.utils.flat import FlatParams
    c = gpt.config("gpt_ref")
    m = gpt.GPT(c, device=dev, dtype=dt, seed=0)
    flat = FlatParams(m, groups=m.param_groups() if hasattr(m, "param_groups") else None)
    opt = FlatAdamW(flat, lr=3e-4, weight_decay=0.01, graph_safe=a.graph)
    _lm_throughput("B5", m, flat, opt, c.vocab_size, c.batch_size, c.block_size, a.steps, a.warmup, name, a.graph)


def run_b9(a, dev, dt, name):
    from solvingpapers_amd.models import deepseekv3 as ds
    from solvingpapers_amd.train.optim import FlatAdamW
    from solvingpapers_amd.utils.flat import FlatParams
    c = ds.config("dsv3_ref")
    m = ds.DeepSeekV3(c, device=dev, dtype=dt, seed=0)
    flat = FlatParams(m, groups=m.param_groups())
    opt = FlatAdamW(flat, lr=6e-4, betas=(0.9, 0.95), eps=1e-8, weight_decay=0.1, max_grad_norm=1.0,
                    graph_safe=a.graph)
    _lm_throughput("B9", m, flat, opt, c.vocab_size, 16, 256, a.steps, a.warmup, name, a.graph)


def run_b13(a, dev, dt, name):
    from solvingpapers_amd.models import gemma
    from solvingpapers_amd.train.optim import FlatAdamW
    from solvingpapers_amd.utils.flat import FlatParams
    c = gemma.config("gemma_ref")
    m = gemma.GemmaRef(c).to(device=dev, dtype=dt)
    flat = FlatParams(m)
    opt = FlatAdamW(flat, lr=2.5e-4, weight_decay=0.01, graph_safe=a.graph)
    _lm_throughput("B13", m, flat, opt, c.vocab_size, c.batch_size, c.block_size, a.steps, a.warmup, name, a.graph)


def run_quality(tag, dev):
    t0 = time.perf_counter()
    if tag == "B14":
        from solvingpapers_amd.models import vit
        _, accs = vit.train(vit.config("vit_mnist_ref"), device=dev, log=lambda *_: None)
        val, unit = accs[-1], "test accuracy %"
    elif tag in ("B15", "B16"):
        from solvingpapers_amd.models import autoencoder
        _, hist = autoencoder.train(autoencoder.AEConfig(kind="ae" if tag == "B15" else "vae",
                                                         epochs=5 if tag == "B15" else 10, device=dev),
                                    log=lambda *_: None)
        val, unit = hist[-1], "MSE" if tag == "B15" else "BCE+KL per 128-image batch"
    else:
        from solvingpapers_amd.models import kd
        _, _, hist = kd.train(kd.KDConfig(device=dev), log=lambda *_: None)
        val, unit = hist[-1][1], "student test accuracy %"
    print(json.dumps({"run": tag, "metric": unit, "value": round(float(val), 6), "reference": REF[tag],
                      "data": "synthetic MNIST-like digits (parity unpinned: reference used MNIST)",
                      "wall_s": round(time.perf_counter() - t0, 2)}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--which", default="B1,B5,B9,B14,B15,B16,B17")
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--graph", action="store_true")
    a = ap.parse_args()
    info = sdist.init_distributed()
    dt = {"bf16": torch.bfloat16, "fp32": torch.float32}[a.dtype]
    for tag in a.which.split(","):
        if tag == "B1":
            run_b1(a, info.device, dt, a.dtype)
        elif tag == "B5":
            run_b5(a, info.device, dt, a.dtype)
        elif tag == "B9":
            run_b9(a, info.device, dt, a.dtype)
        elif tag == "B13":
            run_b13(a, info.device, dt, a.dtype)
        else:
            run_quality(tag, str(info.device))


if __name__ == "__main__":
    main()
