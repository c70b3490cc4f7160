"""How much TP / EP communication do the two-chunk pipelines hide? (1-GPU proxy)

The TP=8 Gemma-7B-shape and EP=8 DeepSeek-V3-width configs need 8 GPUs; a 1-GPU box can
still run ONE rank's share of the work (TP=8 local shards: 2 query heads, 1/8 of the GeGLU
hidden and vocabulary; EP=8: 32 of 256 routed experts receiving N*k rows) with every
collective replaced by parallel/comm.ProxyGroup: the data stays put and a streaming kernel
with ``--nwg`` workgroups occupies a comm stream for the time the collective would take on
xGMI at the modelled bandwidth (``--ar-gbps`` RCCL all-reduce bus bandwidth,
``--a2a-gbps`` all-to-all bytes leaving a rank per second -- inputs, not measurements).

Arms (fwd + bwd, same process, interleaved rounds):
  compute   collectives skipped                                  (proxy mode "off")
  blocking  collectives modelled, the caller waits at each one   (no overlap; = compute + comm)
  pipelined collectives modelled, two-chunk two-stream pipeline  (models/gemma.py, models/deepseekv3.py)
  pipe_comp the pipelined form with collectives skipped          (chunking's own compute cost)

hidden = 1 - (pipelined - pipe_comp) / (blocking - compute): the fraction of the collective
time that no longer adds to the layer time. One JSON line per config.

  python tools/overlap_proxy.py [--which tp,ep] [--layers 2] [--seq 8192]
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from solvingpapers_amd.ops import _ext  # noqa: E402
from solvingpapers_amd.parallel.comm import ProxyGroup  # noqa: E402
from solvingpapers_amd.utils.flat import FlatParams  # noqa: E402


def _time(fn, iters):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def _arms(make_step, groups, iters, rounds):
    """make_step(pipelined) -> step fn. groups: the ProxyGroups whose mode is switched."""
    steps = {"compute": (make_step(False), "off"), "blocking": (make_step(False), "blocking"),
             "pipelined": (make_step(True), "overlap"), "pipe_comp": (make_step(True), "off")}
    res = {k: [] for k in steps}
    comm_ms = {}
    for r in range(rounds):
        for k, (fn, mode) in steps.items():
            for g in groups:
                g.mode = mode
            fn()                                         # warm (allocator, proxy calibration)
            for g in groups:
                g.reset_stats()
            res[k].append(_time(fn, iters))
            comm_ms[k] = sum(g.modelled_s for g in groups) * 1e3 / iters
    med = {k: statistics.median(v) for k, v in res.items()}
    exposed = med["pipelined"] - med["pipe_comp"]
    total = med["blocking"] - med["compute"]
    return med, comm_ms, exposed, total


def tp_gemma(a):
    from solvingpapers_amd.models import gemma
    dev = torch.device("cuda")
    c = gemma.config("gemma_7b_mqa", n_layers=a.layers, max_seq_len=a.seq)
    g1 = ProxyGroup(8, dev, a.ar_gbps, a.a2a_gbps, a.nwg)
    g2 = ProxyGroup(8, dev, a.ar_gbps, a.a2a_gbps, a.nwg)
    models = {}
    for pipe in (False, True):
        m = gemma.Gemma(c, device=dev, dtype=torch.bfloat16, tp_group=g1, tp_group2=g2 if pipe else None, seed=1)
        FlatParams(m, groups=m.param_groups(), grad_dtype=torch.bfloat16)
        models[pipe] = m
    ids = torch.randint(0, c.vocab_size, (1, a.seq + 1), device=dev)

    def make(pipe):
        m = models[pipe]

        def step():
            from solvingpapers_amd.utils.grad import next_generation
            next_generation()
            m(ids[:, :-1], ids[:, 1:]).backward()
        return step

    med, comm_ms, exposed, total = _arms(make, (g1, g2), a.iters, a.rounds)
    return {"config": "gemma_7b_mqa TP=8 local shard (2 q-heads x 256, GeGLU 3072, V/8)", "layers": a.layers,
            "seq": a.seq, "ms": {k: round(v, 3) for k, v in med.items()},
            "modelled_comm_ms": round(comm_ms["blocking"], 3), "comm_added_blocking_ms": round(total, 3),
            "comm_exposed_pipelined_ms": round(exposed, 3),
            "hidden": round(1 - exposed / total, 3) if total > 0 else None}


def ep_moe(a):
    from solvingpapers_amd.models import deepseekv3 as ds
    dev = torch.device("cuda")
    c = ds.config("dsv3_v3", moe_fp8=a.fp8)
    g1 = ProxyGroup(8, dev, a.ar_gbps, a.a2a_gbps, a.nwg)
    g2 = ProxyGroup(8, dev, a.ar_gbps, a.a2a_gbps, a.nwg)
    mods = {}
    for pipe in (False, True):
        m = ds.MoE(c, ep_group=g1, ep_group2=g2 if pipe else None, device=dev, dtype=torch.bfloat16)
        m.reset_parameters(0.02, torch.Generator(device=dev).manual_seed(3))
        FlatParams(m, grad_dtype=torch.bfloat16)
        mods[pipe] = m.train()
    x = (torch.randn(1, a.tokens, c.dim, device=dev) * 0.5).bfloat16().requires_grad_()
    gy = torch.randn_like(x)

    def make(pipe):
        m = mods[pipe]

        def step():
            from solvingpapers_amd.utils.grad import next_generation
            next_generation()
            x.grad = None
            m(x).backward(gy)
        return step

    med, comm_ms, exposed, total = _arms(make, (g1, g2), a.iters, a.rounds)
    return {"config": f"dsv3_v3 MoE layer EP=8 local shard (32 of 256 experts, top-8, D 7168, F 2048, 1 shared)"
                      f"{' fp8' if a.fp8 else ''}", "tokens": a.tokens,
            "ms": {k: round(v, 3) for k, v in med.items()}, "modelled_comm_ms": round(comm_ms["blocking"], 3),
            "comm_added_blocking_ms": round(total, 3), "comm_exposed_pipelined_ms": round(exposed, 3),
            "hidden": round(1 - exposed / total, 3) if total > 0 else None}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--which", default="tp,ep")
    ap.add_argument("--layers", type=int, default=2)
    ap.add_argument("--seq", type=int, default=8192)
    ap.add_argument("--tokens", type=int, default=4096)
    ap.add_argument("--fp8", action="store_true")
    ap.add_argument("--ar-gbps", type=float, default=300.0)
    ap.add_argument("--a2a-gbps", type=float, default=300.0)
    ap.add_argument("--nwg", type=int, default=16)
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    assert _ext.load(), "HIP extension missing"
    base = {"ar_busbw_gbps": a.ar_gbps, "a2a_gbps": a.a2a_gbps, "proxy_nwg": a.nwg}
    for w in a.which.split(","):
        out = tp_gemma(a) if w == "tp" else ep_moe(a)
        print(json.dumps({**out, **base}), flush=True)


if __name__ == "__main__":
    main()
