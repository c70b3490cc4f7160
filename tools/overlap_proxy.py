"""How much TP / EP communication do the two-chunk pipelines hide? (1-GPU proxy)

The TP=8 Gemma-7B-shape and EP=8 DeepSeek-V3-width configs need 8 GPUs; a 1-GPU box can
still run ONE rank's share of the work (TP=8 local shards: 2 query heads, 1/8 of the GeGLU
hidden and vocabulary; EP=8: 32 of 256 routed experts receiving N*k rows) with every
collective replaced by parallel/comm.ProxyGroup: the data stays put and a streaming kernel
with ``--nwg`` workgroups occupies a comm stream for the time the collective would take on
xGMI at the modelled bandwidth (``--ar-gbps`` RCCL all-reduce bus bandwidth,
``--a2a-gbps`` all-to-all bytes leaving a rank per second -- inputs, not measurements).

Arms (fwd + bwd, same process, interleaved rounds):
  compute / off   plain layers, collectives skipped                     (proxy mode "off")
  blocking        plain layers, collectives modelled, each one waited   (= compute + comm)
  <form>:overlap  an overlapping form, collectives modelled and overlapped (TP: Gemma's
                  sequence-parallel chunk pair; EP: DeepSeekV3.forward_pair, two micro-batches)
  <form>:off      the same form with collectives skipped                (the form's own cost)

hidden = 1 - (overlap - off) / (blocking - compute): the fraction of the collective time that
no longer adds to the layer time; pair_vs_blocking: overlapped time over blocking time, the
headline figure. One JSON line per config.

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
    """TP=8 Gemma-7B shapes, sequence parallel (the TP default): one rank's share of ``--layers``
    layers, fwd + bwd of ``--batch`` sequences of ``--seq`` tokens. Arms:
      compute / blocking   the plain SP forward, collectives skipped / modelled and waited at once
      pair:off / pair:overlap   Gemma._forward_sp_pair (two chunks: batch halves when --batch is
                           even, else sequence halves; each chunk's layer-boundary reduce-scatter
                           -> all-gather runs under the other chunk's compute)
    --micro: a step is two gradient-accumulation micro-batches of --batch sequences; compute /
    blocking run them one after the other, the pair arms as Gemma.forward_pair (no chunk split)."""
    from solvingpapers_amd.models import gemma
    dev = torch.device("cuda")
    c = gemma.config("gemma_7b_mqa", n_layers=a.layers, max_seq_len=a.seq)
    g1 = ProxyGroup(8, dev, a.ar_gbps, a.a2a_gbps, a.nwg, synth_gather=True)
    m = gemma.Gemma(c, device=dev, dtype=torch.bfloat16, tp_group=g1, seed=1).train()
    FlatParams(m, groups=m.param_groups(), grad_dtype=torch.bfloat16)
    ids = torch.randint(0, c.vocab_size, (a.batch, a.seq + 1), device=dev)
    ids2 = torch.randint(0, c.vocab_size, (a.batch, a.seq + 1), device=dev)
    split = "micro" if a.micro else m._pair_split(ids[:, :-1])
    assert split is not None, "the pair needs T divisible by 2 x TP (or an even batch)"

    def step_of(pair):
        def step():
            from solvingpapers_amd.utils.grad import next_generation
            next_generation()
            m.tp_pipeline = pair
            if not a.micro:
                m(ids[:, :-1], ids[:, 1:]).backward()
            elif pair:
                m.forward_pair(ids[:, :-1], ids[:, 1:], ids2[:, :-1], ids2[:, 1:]).backward()
            else:   # gradient accumulation, one micro-batch after the other
                m(ids[:, :-1], ids[:, 1:]).backward()
                m(ids2[:, :-1], ids2[:, 1:]).backward()
            m.sync_sequence_parallel_grads()
        return step

    arms = {"compute": (step_of(False), "off"), "blocking": (step_of(False), "blocking"),
            "pair:off": (step_of(True), "off"), "pair:overlap": (step_of(True), "overlap")}
    if ARMS:
        arms = {k: v for k, v in arms.items() if k in ARMS}
    res = {k: [] for k in arms}
    comm = 0.0
    for r in range(a.rounds):
        for k, (fn, mode) in arms.items():
            g1.mode = mode
            fn()
            g1.reset_stats()
            res[k].append(_time(fn, a.iters))
            if k == "blocking":
                comm = g1.modelled_s * 1e3 / a.iters
    med = {k: round(statistics.median(v), 3) for k, v in res.items()}
    out = {"config": "gemma_7b_mqa TP=8 SP local shard (2 q-heads x 256, GeGLU 3072, V/8)", "layers": a.layers,
           "batch": a.batch, "seq": a.seq, "split": split, "micro_batches": 2 if a.micro else 1, "ms": med, "modelled_comm_ms": round(comm, 3)}
    if not ARMS:
        total = med["blocking"] - med["compute"]
        out["comm_added_blocking_ms"] = round(total, 3)
        out["pair_compute_cost_ms"] = round(med["pair:off"] - med["compute"], 3)
        out["hidden_pair"] = round(1 - (med["pair:overlap"] - med["pair:off"]) / total, 3) if total > 0 else None
        out["pair_vs_blocking"] = round(med["pair:overlap"] / med["blocking"], 3)
    return out


def ep_moe(a):
    """EP=8 DeepSeek-V3 widths, one rank's share: ``--layers`` decoder layers (MLA attention +
    MoE with 32 of 256 routed experts, top-8, 1 shared; --fp8: e4m3 dispatch payload and expert
    GEMMs), two micro-batches of ``--tokens`` tokens per step, fwd + bwd. Arms:
      off / blocking   the micro-batches one after the other (forward()), collectives skipped /
                       modelled and waited at once
      pair:off / pair:overlap   DeepSeekV3.forward_pair (layer-interleaved micro-batches)
    --capacity CF adds the accum-1 comparison (micro-batches one after the other, collectives
    modelled and overlapped as far as each path allows):
      one:overlap     exact split sizes: one host sync per MoE layer (the pipeline drains there)
      cap:overlap / cap:off   the host-sync-free padded dispatch at capacity factor CF (P*C rows on
                      the wire instead of N*k; one overflow-flag read per forward)"""
    from solvingpapers_amd.models import deepseekv3 as ds
    dev = torch.device("cuda")
    c = ds.config("dsv3_v3", moe_fp8=a.fp8, n_layers=a.layers, n_dense_layers=0, mtp_heads=0,
                  vocab_size=a.vocab, block_size=a.tokens)
    g1 = ProxyGroup(8, dev, a.ar_gbps, a.a2a_gbps, a.nwg)
    if a.balanced:
        # a trained, aux-free-balanced router stand-in: token t -> experts (t k + j) mod E (every
        # expert and every peer gets exactly its share), weights softmax over the chosen logits
        def balanced_route(logits, k, bias=None, bias_in_weights=True):
            N, E = logits.shape
            idx = ((torch.arange(N, device=logits.device)[:, None] * k + torch.arange(k, device=logits.device))
                   % E).to(torch.int32)
            return idx, torch.softmax(logits.gather(1, idx.long()).float(), -1)
        ds.route = balanced_route
    m = ds.DeepSeekV3(c, device=dev, dtype=torch.bfloat16, seed=3, ep_group=g1).train()
    FlatParams(m, groups=m.param_groups(), grad_dtype=torch.bfloat16)
    ids = torch.randint(0, c.vocab_size, (2, 1, a.tokens + 1), device=dev)
    x0, y0, x1, y1 = ids[0, :, :-1], ids[0, :, 1:], ids[1, :, :-1], ids[1, :, 1:]

    def step_of(pair, cap=0.0):
        def step():
            from solvingpapers_amd.utils.grad import next_generation
            next_generation()
            m.c.ep_capacity = cap
            for l in m.moe_layers():
                l.c.ep_capacity = cap
            if pair:
                m.forward_pair(x0, y0, x1, y1).backward()
            else:
                m(x0, y0).backward()
                m(x1, y1).backward()
        return step

    arms = {"off": (step_of(False), "off"), "blocking": (step_of(False), "blocking"),
            "pair:off": (step_of(True), "off"), "pair:overlap": (step_of(True), "overlap")}
    if a.capacity > 0:
        arms.update({"one:overlap": (step_of(False), "overlap"), "cap:off": (step_of(False, a.capacity), "off"),
                     "cap:overlap": (step_of(False, a.capacity), "overlap")})
    if ARMS:
        arms = {k: v for k, v in arms.items() if k in ARMS}
    res = {k: [] for k in arms}
    comm = 0.0
    for r in range(a.rounds):
        for k, (fn, mode) in arms.items():
            g1.mode = mode
            fn()
            g1.reset_stats()
            res[k].append(_time(fn, a.iters))
            if k == "blocking":
                comm = g1.modelled_s * 1e3 / a.iters
    med = {k: round(statistics.median(v), 3) for k, v in res.items()}
    out = {"config": f"dsv3_v3 widths EP=8 local shard, {a.layers} MLA+MoE layers (32 of 256 experts, top-8, D 7168, "
                     f"F 2048, 1 shared){' fp8' if a.fp8 else ''}, 2 micro-batches x {a.tokens} tokens, vocab {a.vocab}",
           "ms": med, "modelled_comm_ms": round(comm, 3), "routing": "balanced" if a.balanced else "model"}
    if not ARMS:
        total = med["blocking"] - med["off"]
        out["comm_added_blocking_ms"] = round(total, 3)
        out["pair_compute_cost_ms"] = round(med["pair:off"] - med["off"], 3)
        out["hidden_pair"] = round(1 - (med["pair:overlap"] - med["pair:off"]) / total, 3) if total > 0 else None
        out["pair_vs_blocking"] = round(med["pair:overlap"] / med["blocking"], 3)
        if a.capacity > 0:
            from solvingpapers_amd.parallel.expert_parallel import capacity_scale
            out["capacity_factor"] = a.capacity
            out["capacity_scale_after"] = capacity_scale()     # > 1: some forward overflowed and re-ran
            out["cap_vs_one"] = round(med["cap:overlap"] / med["one:overlap"], 3)
            out["cap_compute_cost_ms"] = round(med["cap:off"] - med["off"], 3)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--which", default="tp,ep")
    ap.add_argument("--layers", type=int, default=2)
    ap.add_argument("--seq", type=int, default=8192)
    ap.add_argument("--batch", type=int, default=1, help="TP: sequences per step (even: the pipeline splits by batch)")
    ap.add_argument("--micro", action="store_true", help="TP: two accumulation micro-batches per step")
    ap.add_argument("--tokens", type=int, default=4096)
    ap.add_argument("--vocab", type=int, default=1024,
                    help="EP: vocabulary of the tied head (1024 isolates the MoE layers; dsv3_v3 has 129280, whose "
                         "head is the compute a real step runs under the last combine / first combine-grad)")
    ap.add_argument("--fp8", action="store_true", default=True, help="EP: fp8 experts + dispatch (config #5)")
    ap.add_argument("--bf16", dest="fp8", action="store_false")
    ap.add_argument("--ar-gbps", type=float, default=300.0)
    ap.add_argument("--a2a-gbps", type=float, default=300.0)
    ap.add_argument("--nwg", type=int, default=16)
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--arms", default="", help="comma list of arm names (default all), e.g. pair:overlap")
    ap.add_argument("--balanced", action="store_true", help="EP: round-robin routing (every peer exactly its "
                    "share) instead of the random-init router, whose loads are skewed")
    ap.add_argument("--capacity", type=float, default=0.0, help="EP: also time the host-sync-free dispatch at this "
                    "capacity factor against the exact-split path, micro-batches one by one (accum-1 form)")
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
