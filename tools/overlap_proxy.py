"""How much TP / EP communication do the two-chunk pipelines hide? (1-GPU proxy)

The TP=8 Gemma-7B-shape and EP=8 DeepSeek-V3-width configs need 8 GPUs; a 1-GPU box can
still run ONE rank's share of the work (TP=8 local shards: 2 query heads, 1/8 of the GeGLU
hidden and vocabulary; EP=8: 32 of 256 routed experts receiving N*k rows) with every
collective replaced by parallel/comm.ProxyGroup: the data stays put and a streaming kernel
with ``--nwg`` workgroups occupies a comm stream for the time the collective would take on
xGMI at the modelled bandwidth (``--ar-gbps`` RCCL all-reduce bus bandwidth,
``--a2a-gbps`` all-to-all bytes leaving a rank per second -- inputs, not measurements).

Arms (fwd + bwd, same process, interleaved rounds):
  compute       plain layer, collectives skipped                      (proxy mode "off")
  blocking      plain layer, collectives modelled, each one waited    (= compute + comm)
  <form>:overlap  a two-chunk form, collectives modelled and overlapped (models/gemma.py,
                models/deepseekv3.py: TP interleave / two_stream; EP interleaved2/4 / two_stream)
  <form>:off    the same form with collectives skipped                (chunking's own cost)

hidden = 1 - (overlap - off) / (blocking - compute): the fraction of the collective time that
no longer adds to the layer time. One JSON line per config.

  python tools/overlap_proxy.py [--which tp,ep] [--layers 2] [--seq 8192]
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

# a real TP / EP run (world > 1 over RCCL) selects hipBLASLt's data-parallel stream-K grid in
# parallel/dist.py init_distributed (a persistent whole-chip grid stalls next to a collective);
# the one-process proxy must run the same GEMM configuration. Set before hipBLASLt loads.
if os.environ.get("SPA_STREAMK_DP", "1") != "0":
    os.environ.setdefault("TENSILE_STREAMK_DATA_PARALLEL", "1")

import torch  # noqa: E402

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


ARMS = None   # --arms: run only these (profiling one arm under rocprofv3)


def tp_gemma(a):
    """Plain layer (compute / blocking arms) and both two-chunk schedules of models/gemma.py:
    "interleave" (one stream, staged) and "two_stream" (half B on a second compute stream)."""
    from solvingpapers_amd.models import gemma
    dev = torch.device("cuda")
    c = gemma.config("gemma_7b_mqa", n_layers=a.layers, max_seq_len=a.seq)
    g1 = ProxyGroup(8, dev, a.ar_gbps, a.a2a_gbps, a.nwg)
    g2 = ProxyGroup(8, dev, a.ar_gbps, a.a2a_gbps, a.nwg)
    models = {}
    for name, kw in (("plain", {}), ("interleave", dict(tp_group2=g2, tp_schedule="interleave")),
                     ("two_stream", dict(tp_group2=g2, tp_schedule="two_stream"))):
        if a.variants and name != "plain" and name not in a.variants.split(","):
            continue
        m = gemma.Gemma(c, device=dev, dtype=torch.bfloat16, tp_group=g1, seed=1, **kw)
        FlatParams(m, groups=m.param_groups(), grad_dtype=torch.bfloat16)
        models[name] = m
    ids = torch.randint(0, c.vocab_size, (a.batch, a.seq + 1), device=dev)

    def step_of(m):
        def step():
            from solvingpapers_amd.utils.grad import next_generation
            next_generation()
            m(ids[:, :-1], ids[:, 1:]).backward()
        return step

    arms = {"compute": (step_of(models["plain"]), "off"), "blocking": (step_of(models["plain"]), "blocking")}
    for name in models:
        if name != "plain":
            arms[name + ":overlap"] = (step_of(models[name]), "overlap")
            arms[name + ":off"] = (step_of(models[name]), "off")
    if ARMS:
        arms = {k: v for k, v in arms.items() if k in ARMS}
    res = {k: [] for k in arms}
    comm = 0.0
    for r in range(a.rounds):
        for k, (fn, mode) in arms.items():
            for g in (g1, g2):
                g.mode = mode
            fn()
            for g in (g1, g2):
                g.reset_stats()
            res[k].append(_time(fn, a.iters))
            if k == "blocking":
                comm = (g1.modelled_s + g2.modelled_s) * 1e3 / a.iters
    med = {k: round(statistics.median(v), 3) for k, v in res.items()}
    out = {"config": "gemma_7b_mqa TP=8 local shard (2 q-heads x 256, GeGLU 3072, V/8)", "layers": a.layers,
           "batch": a.batch, "seq": a.seq, "split": "batch" if a.batch % 2 == 0 else "sequence",
           "ms": med, "modelled_comm_ms": round(comm, 3)}
    if not ARMS:
        total = med["blocking"] - med["compute"]
        out["comm_added_blocking_ms"] = round(total, 3)
        for name in models:
            if name == "plain":
                continue
            exposed = med[name + ":overlap"] - med[name + ":off"]
            out[f"hidden_{name}"] = round(1 - exposed / total, 3) if total > 0 else None
            out[f"vs_blocking_{name}"] = round(med["blocking"] / med[name + ":overlap"], 3)
    return out


def ep_moe(a):
    """Variants: plain (one exchange per layer), one-stream interleaved chunks (2 and 4), and two
    chunks on two streams / communicators; each timed with collectives modelled and skipped."""
    from solvingpapers_amd.models import deepseekv3 as ds
    dev = torch.device("cuda")
    c = ds.config("dsv3_v3", moe_fp8=a.fp8)
    g1 = ProxyGroup(8, dev, a.ar_gbps, a.a2a_gbps, a.nwg)
    g2 = ProxyGroup(8, dev, a.ar_gbps, a.a2a_gbps, a.nwg)
    variants = {"plain": dict(ep_chunks=1), "interleaved2": dict(ep_chunks=2), "interleaved4": dict(ep_chunks=4),
                "two_stream": dict(ep_group2=g2, ep_schedule="two_stream")}
    if a.variants:
        variants = {k: v for k, v in variants.items() if k in a.variants.split(",") or k == "plain"}
    mods = {}
    for name, kw in variants.items():
        m = ds.MoE(c, ep_group=g1, device=dev, dtype=torch.bfloat16, **kw)
        m.reset_parameters(0.02, torch.Generator(device=dev).manual_seed(3))
        FlatParams(m, grad_dtype=torch.bfloat16)
        mods[name] = m.train()
    x = (torch.randn(1, a.tokens, c.dim, device=dev) * 0.5).bfloat16().requires_grad_()
    gy = torch.randn_like(x)

    def step_of(m):
        def step():
            from solvingpapers_amd.utils.grad import next_generation
            next_generation()
            x.grad = None
            m(x).backward(gy)
        return step

    arms = {}
    for name, m in mods.items():
        arms[name + ":off"] = (step_of(m), "off")
        arms[name + ":overlap" if name != "plain" else "plain:blocking"] = (step_of(m), "overlap" if name != "plain" else "blocking")
    if ARMS:
        arms = {k: v for k, v in arms.items() if k in ARMS}
    res = {k: [] for k in arms}
    comm = 0.0
    for r in range(a.rounds):
        for k, (fn, mode) in arms.items():
            for g in (g1, g2):
                g.mode = mode
            fn()
            for g in (g1, g2):
                g.reset_stats()
            res[k].append(_time(fn, a.iters))
            if k == "plain:blocking":
                comm = (g1.modelled_s + g2.modelled_s) * 1e3 / a.iters
    med = {k: round(statistics.median(v), 3) for k, v in res.items()}
    out = {"config": f"dsv3_v3 MoE layer EP=8 local shard (32 of 256 experts, top-8, D 7168, F 2048, 1 shared)"
                     f"{' fp8' if a.fp8 else ''}", "tokens": a.tokens, "ms": med, "modelled_comm_ms": round(comm, 3)}
    if not ARMS:
        total = med["plain:blocking"] - med["plain:off"]
        out["comm_added_blocking_ms"] = round(total, 3)
        for name in variants:
            if name == "plain":
                continue
            exposed = med[name + ":overlap"] - med[name + ":off"]
            out[f"hidden_{name}"] = round(1 - exposed / total, 3) if total > 0 else None
            out[f"vs_blocking_{name}"] = round(med["plain:blocking"] / med[name + ":overlap"], 3)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--which", default="tp,ep")
    ap.add_argument("--layers", type=int, default=2)
    ap.add_argument("--seq", type=int, default=8192)
    ap.add_argument("--batch", type=int, default=1, help="TP: sequences per step (even: the pipeline splits by batch)")
    ap.add_argument("--tokens", type=int, default=4096)
    ap.add_argument("--fp8", action="store_true")
    ap.add_argument("--ar-gbps", type=float, default=300.0)
    ap.add_argument("--a2a-gbps", type=float, default=300.0)
    ap.add_argument("--nwg", type=int, default=16)
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--arms", default="", help="comma list of arm names (default all), e.g. interleave:overlap")
    ap.add_argument("--variants", default="", help="EP: subset of interleaved2,interleaved4,two_stream; "
                                                   "TP: subset of interleave,two_stream")
    a = ap.parse_args()
    global ARMS
    ARMS = [x for x in a.arms.split(",") if x] or None
    assert _ext.load(), "HIP extension missing"
    base = {"ar_busbw_gbps": a.ar_gbps, "a2a_gbps": a.a2a_gbps, "proxy_nwg": a.nwg,
            "streamk_data_parallel": os.environ.get("TENSILE_STREAMK_DATA_PARALLEL") == "1"}
    for w in a.which.split(","):
        out = tp_gemma(a) if w == "tp" else ep_moe(a)
        print(json.dumps({**out, **base}), flush=True)


if __name__ == "__main__":
    main()
