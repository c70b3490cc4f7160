"""What does a collective running beside the backward cost the backward's GEMMs?

bench.py at N > 1 all-reduces per-layer gradient buckets on RCCL's stream while the last
micro-batch's backward is still running (parallel/data_parallel.py). RCCL's ring kernels hold one
workgroup per channel on a CU for the whole collective, and hipBLASLt's stream-K GEMMs launch a
grid sized to the whole chip, so a co-running collective can delay GEMM workgroups instead of
using idle bandwidth. A 1-GPU box has no second GPU to all-reduce with; this script stands in a
limited-grid streaming kernel (``spa::stream_copy_wg``: ``nwg`` workgroups copying memory, the
footprint of an RCCL ring kernel with ``nwg`` channels) on a side stream and measures:

  * fwd+bwd alone, the proxy alone,
  * both together (proxy launched when the backward starts, sized to last about as long as the
    backward alone),

and prints whether overlapping beats running the two back to back. One JSON line per arm.

  python tools/overlap_interference.py --layers 4 --nwg 16,32,64
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from solvingpapers_amd.models import llama3  # noqa: E402
from solvingpapers_amd.ops import _ext  # noqa: E402
from solvingpapers_amd.utils.tuning import load_gemm_tuning  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", type=int, default=4)
    ap.add_argument("--seq", type=int, default=8192)
    ap.add_argument("--nwg", default="16,32,64")
    ap.add_argument("--mb", type=int, default=256, help="proxy buffer MB")
    ap.add_argument("--iters", type=int, default=3)
    a = ap.parse_args()
    assert _ext.load(), "HIP extension missing"
    ops = _ext.ops()
    load_gemm_tuning(None)
    dev = torch.device("cuda:0")
    cfg = llama3.config("llama3_8b", max_seq_len=a.seq, n_layers=a.layers)
    model = llama3.Llama3(cfg, device=dev, dtype=torch.bfloat16, seed=1)
    x = torch.randint(0, cfg.vocab_size, (1, a.seq), device=dev)
    y = torch.randint(0, cfg.vocab_size, (1, a.seq), device=dev)
    src = torch.empty(a.mb << 20, dtype=torch.uint8, device=dev)
    dst = torch.empty_like(src)
    side = torch.cuda.Stream()
    ev = lambda: torch.cuda.Event(enable_timing=True)  # noqa: E731

    def fwd_bwd(proxy=None):
        """proxy = (nwg, reps): launched on the side stream once the forward is done."""
        for p in model.parameters():
            p.grad = None
        e0, e1, e2, p0, p1 = ev(), ev(), ev(), ev(), ev()
        e0.record()
        loss = model(x, y)
        e1.record()
        if proxy is not None:
            side.wait_event(e1)
            with torch.cuda.stream(side):
                p0.record(side)
                ops.stream_copy_wg(src, dst, proxy[0], proxy[1])
                p1.record(side)
        loss.backward()
        e2.record()
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        bwd = e1.elapsed_time(e2)
        return bwd, (p0.elapsed_time(p1) if proxy is not None else None)

    def proxy_alone(nwg, reps):
        p0, p1 = ev(), ev()
        p0.record()
        ops.stream_copy_wg(src, dst, nwg, reps)
        p1.record()
        torch.cuda.synchronize()
        return p0.elapsed_time(p1)

    for _ in range(2):
        fwd_bwd()
    bwd0 = min(fwd_bwd()[0] for _ in range(a.iters))
    print(json.dumps({"arm": "bwd_alone", "layers": a.layers, "bwd_ms": round(bwd0, 3)}), flush=True)
    for nwg in [int(v) for v in a.nwg.split(",")]:
        proxy_alone(nwg, 1)
        one = proxy_alone(nwg, 1)
        reps = max(1, int(round(bwd0 / one)))
        alone = proxy_alone(nwg, reps)
        gbs = 2 * src.numel() * reps / alone / 1e6
        res = [fwd_bwd((nwg, reps)) for _ in range(a.iters)]
        bwd = min(r[0] for r in res)
        px = min(r[1] for r in res)
        together = max(bwd, px)
        print(json.dumps({"arm": "overlap", "nwg": nwg, "reps": reps, "proxy_alone_ms": round(alone, 3),
                          "proxy_GBps": round(gbs, 1), "bwd_with_proxy_ms": round(bwd, 3),
                          "proxy_with_bwd_ms": round(px, 3), "serial_ms": round(bwd0 + alone, 3),
                          "overlapped_ms": round(together, 3),
                          "bwd_slowdown": round(bwd / bwd0, 3),
                          "overlap_pays": together < bwd0 + alone}), flush=True)


if __name__ == "__main__":
    main()
