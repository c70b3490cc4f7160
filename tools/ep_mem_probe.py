"""Where the forced-collective EP path's extra memory goes (profiles/r6_rccl_preflight.txt: dsv3_v3 fp8 at
one EP=8 rank's share peaked 240.8 GB through a 1-rank RCCL group vs 146.7 GB without one). Runs one
micro-batch forward + backward of a reduced dsv3_v3 (2 layers, 1 MoE) per mode and prints the live /
peak allocations after each phase. Launch with torch.distributed.run --nproc-per-node 1 and
SPA_FORCE_COLLECTIVES=1 for the EP arm (the script runs both arms when the group exists).

Round 6 finding (profiles/r6_ep_memory.txt): the EP arm's live memory grew by ~3.3 GB (fp8) / 3.8 GB (bf16)
per extra micro-batch because the RCCL Work objects of the dispatch / combine exchanges stayed referenced
from their hand-off boxes after wait(), and a Work keeps its input and output buffers alive; the boxes now
drop them once waited (comm._A2AFinish / _A2AStart, expert_parallel._Fp8Dispatch*). --check prints the
per-micro-batch growth as one JSON line (tests/test_preflight_gpu.py)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.distributed as dist

from solvingpapers_amd.models import deepseekv3 as ds
from solvingpapers_amd.parallel import dist as sdist


def gb(x):
    return round(x / 1e9, 2)


def arm(name, group, fp8, T=4096, history=True):
    torch.cuda.empty_cache()
    torch.cuda.reset_peak_memory_stats()
    c = ds.config("dsv3_v3", n_layers=2, n_dense_layers=1, n_experts=32, block_size=T, moe_fp8=fp8, fp8_linears=fp8)
    m = ds.DeepSeekV3(c, device="cuda", dtype=torch.bfloat16, seed=1, ep_group=group)
    base = torch.cuda.memory_allocated()
    ids = torch.randint(0, c.vocab_size, (1, T + 1), device="cuda")
    loss = m(ids[:, :-1], ids[:, 1:])
    torch.cuda.synchronize()
    fwd_live, fwd_peak = torch.cuda.memory_allocated() - base, torch.cuda.max_memory_allocated() - base
    loss.backward()
    torch.cuda.synchronize()
    bwd_peak = torch.cuda.max_memory_allocated() - base
    after = torch.cuda.memory_allocated() - base
    grads = sum(p.grad.numel() * p.grad.element_size() for p in m.parameters() if p.grad is not None)
    del loss
    lives = []
    if name != "local" and history:
        torch.cuda.memory._record_memory_history(max_entries=200000)
    for _ in range(3):                          # more micro-batches: does the residue grow?
        l2 = m(ids[:, :-1], ids[:, 1:])
        l2.backward()
        del l2
        torch.cuda.synchronize()
        lives.append(gb(torch.cuda.memory_allocated() - base))
    import gc
    gc.collect()
    torch.cuda.synchronize()
    after_gc = gb(torch.cuda.memory_allocated() - base)
    print({"arm": name, "live_after_each_extra_microbatch_gb": lives, "live_after_gc_collect_gb": after_gc}, flush=True)
    from solvingpapers_amd.parallel import comm
    boxes = [o for o in gc.get_objects() if isinstance(o, comm._Box)]
    print({"arm": name, "live_boxes": len(boxes),
           "referrer_types": sorted({type(r).__name__ for b in boxes[:8] for r in gc.get_referrers(b)})}, flush=True)
    if name != "local" and history:
        snap = torch.cuda.memory._snapshot()
        torch.cuda.memory._record_memory_history(enabled=None)
        from collections import Counter
        sites = Counter()
        for seg in snap["segments"]:
            for blk in seg["blocks"]:
                if blk["state"] != "active_allocated" or blk["size"] < (64 << 20):
                    continue
                fr = [f for f in blk.get("frames", []) if "solvingpapers_amd" in f.get("filename", "") or "tools/" in f.get("filename", "")]
                key = " <- ".join(f"{f['filename'].split('solvingpapers_amd/')[-1]}:{f['line']}:{f['name']}" for f in fr[:4])
                sites[(key, blk["size"] >> 20)] += 1
        for (k, mb), n in sites.most_common(25):
            print(f"LIVE {n} x {mb} MiB  {k}", flush=True)
    loss = None
    res = {"arm": name, "fp8": fp8, "growth_gb": round(lives[-1] - lives[0], 3), "live_boxes": len(boxes)}
    print({"arm": name, "fp8": fp8, "params_gb": gb(base), "saved_after_fwd_gb": gb(fwd_live),
           "fwd_peak_gb": gb(fwd_peak), "bwd_peak_gb": gb(bwd_peak), "live_after_bwd_gb": gb(after),
           "grads_gb": gb(grads)}, flush=True)
    del m, loss
    import gc
    gc.collect()
    return res


def main():
    import argparse
    import json
    ap = argparse.ArgumentParser()
    ap.add_argument("--seq", type=int, default=4096)
    ap.add_argument("--check", action="store_true", help="EP arm only, no allocation history; print one JSON line")
    a = ap.parse_args()
    sdist.init_distributed()
    grp = dist.group.WORLD if dist.is_initialized() else None
    if a.check:
        out = [arm("ep-forced" if grp is not None else "local", grp, fp8, a.seq, history=False) for fp8 in (True, False)]
        print(json.dumps({"arms": out}), flush=True)
    else:
        for fp8 in (True, False):
            arm("local", None, fp8, a.seq)
            if grp is not None:
                arm("ep-forced", grp, fp8, a.seq)
    sdist.cleanup()


if __name__ == "__main__":
    main()
