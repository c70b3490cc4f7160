"""Child process of tests/test_rccl_gpu.py: every collective path of the framework through a
REAL RCCL process group of size 1 on cuda:0 (SPA_FORCE_COLLECTIVES=1 makes the world-1 paths take
the exchange code instead of short-circuiting; see parallel/dist.py force_collectives).

Checked here, each against the same computation without a process group:
  * init_process_group("nccl", device_id=cuda:0), barrier(device_ids=...), all_reduce_max;
  * DataParallel per-layer buckets with ReduceOp.AVG on a bf16 gradient buffer, launched from the
    backward's ready markers, with no_sync accumulation over two micro-batches;
  * ZeRO-1: reduce_scatter_tensor + sharded AdamW + all_gather_into_tensor;
  * both DP reductions: "ring" (the two above) and "a2a" (all_to_all_single of the bucket, the
    fp32 shard sum kernel on a side stream, in-place all_gather_into_tensor);
  * comm.all_to_all_single with explicit splits issued from the launch stream (after=event);
  * the EP dispatch: count all-to-all, pinned D2H of the split sizes, row exchange, device regroup,
    combine exchange -- bf16 and fp8 (e4m3 + E8M0) payloads, forward and backward;
  * the async routing-bias all-reduce of aux-free balancing (MoE._update_bias / finish_pending).
Prints RCCL_WORLD1_OK on success; any failed check raises (non-zero exit)."""
import contextlib
import os
import sys

import torch


def rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / b.norm().clamp_min(1e-12)).item()


def step(tag, msg=""):
    print(f"[rccl-world1] {tag} ok {msg}", flush=True)


# SPA_TEST_DEVICE=cpu: the same paths over a gloo group on the CPU (tests/test_parallel_cpu.py)
CPU = os.environ.get("SPA_TEST_DEVICE") == "cpu"
DEV = "cpu" if CPU else "cuda:0"
DT = torch.float32 if CPU else torch.bfloat16


def sync():
    if not CPU:
        torch.cuda.synchronize()


def llama():
    from solvingpapers_amd.models import llama3
    c = llama3.config("llama3_tiny", max_seq_len=256)
    return llama3.Llama3(c, device=DEV, dtype=DT, seed=3)


def dp_run(use_dp, zero1, ids, reduce=None):
    import torch.distributed as dist
    from solvingpapers_amd.parallel.data_parallel import DataParallel
    from solvingpapers_amd.train.optim import FlatAdamW
    from solvingpapers_amd.utils.flat import FlatParams
    m = llama()
    flat = FlatParams(m, groups=m.param_groups(), grad_dtype=DT, align=64)
    dp = DataParallel(m, flat, zero1=zero1, reduce=reduce) if use_dp else None
    if dp is not None:
        assert dp.active and dp.backend == dist.get_backend() == ("gloo" if CPU else "nccl")
    shard = (dp.shard_ranges(), None) if zero1 else None
    opt = FlatAdamW(flat, lr=1e-3, weight_decay=0.1, max_grad_norm=1.0, shard=shard)
    opt.zero_grad()
    for i in range(2):
        ctx = dp.no_sync() if (dp is not None and i == 0) else contextlib.nullcontext()
        with ctx:
            (m(ids[i:i + 1, :-1], ids[i:i + 1, 1:]) / 2).backward()
    if dp is not None:
        assert len(dp._launched) > 0, "no bucket launched from the backward's ready markers"
        dp.finish_grad_sync()
    g = flat.grad.float().clone()
    opt.step()
    if dp is not None:
        dp.gather_params()
    sync()
    return g, flat.param.float().clone()


def moe_run(group, fp8, aux_free=False):
    from solvingpapers_amd.models import deepseekv3 as ds
    c = ds.config("dsv3_tiny", dim=256, n_experts=8, top_k=2, n_shared=1, expert_hidden=256, aux_free=aux_free,
                  moe_fp8=fp8, balance_stat="counts")
    m = ds.MoE(c, ep_group=group, device=DEV, dtype=DT)
    m.reset_parameters(0.05, torch.Generator(device=DEV).manual_seed(3))
    g = torch.Generator().manual_seed(7)
    x = torch.randn(2, 64, 256, generator=g).to(DEV, DT).requires_grad_(True)
    gy = torch.randn(2, 64, 256, generator=g).to(DEV)
    y = m(x)
    (y.float() * gy).sum().backward()
    pend = len(m._pending_bias)
    m.finish_pending()
    sync()
    return y.detach().float(), x.grad.float(), m.w13.grad.float(), m.w2.grad.float(), m.routing_bias.clone(), pend


def main():
    assert os.environ.get("SPA_FORCE_COLLECTIVES") == "1" and os.environ.get("WORLD_SIZE") == "1"
    import torch.distributed as dist
    from solvingpapers_amd.ops import _ext
    from solvingpapers_amd.parallel import comm
    from solvingpapers_amd.parallel import dist as sdist
    from solvingpapers_amd.parallel import expert_parallel as ep
    assert CPU or _ext.load(), "HIP extension must load on the GPU box"
    fp8s = (False,) if CPU else (False, True)
    # reference computations first, with no process group
    ids = torch.randint(0, 1024, (2, 257), generator=torch.Generator().manual_seed(7)).to(DEV)
    ref_g, ref_p = dp_run(False, False, ids)
    ref_moe = {fp8: moe_run(None, fp8) for fp8 in fp8s}
    ref_bias = moe_run(None, False, aux_free=True)

    info = sdist.init_distributed()
    want = "gloo" if CPU else "nccl"
    assert dist.is_initialized() and dist.get_backend() == want, dist.get_backend()
    assert info.backend == want and info.device == torch.device(DEV) and sdist.is_dist()
    step("init", f"backend={dist.get_backend()} world={dist.get_world_size()}")
    sdist.barrier()
    assert sdist.all_reduce_max(3.5) == 3.5
    if not CPU:   # gloo has no AVG
        t = torch.full((1000,), 2.0, device=DEV, dtype=torch.bfloat16)
        dist.all_reduce(t, op=dist.ReduceOp.AVG)
        assert torch.all(t == 2.0)
    step("barrier/all_reduce_max/AVG")

    # an AVG over one rank is the identity: equal up to the run-to-run atomics of a few kernels
    # reduce="ring": RCCL all-reduce / reduce-scatter (AVG); "a2a": all-to-all + device fp32 shard
    # sum (spa::shard_sum_ on a side stream) + in-place all-gather -- the bf16 default
    for red in ("ring", "a2a"):
        g, p = dp_run(True, False, ids, red)
        assert rel(g, ref_g) < 1e-3, ("DP bucket grads", red, rel(g, ref_g))
        assert (p - ref_p).abs().max().item() < 1e-2, ("DP params", red, (p - ref_p).abs().max().item())
        step("dp buckets + no_sync", f"reduce={red} grad numel={g.numel()} rel={rel(g, ref_g):.2e}")
        g, p = dp_run(True, True, ids, red)
        assert (p - ref_p).abs().max().item() < 1e-2, ("ZeRO-1 params", red, (p - ref_p).abs().max().item())
        step("zero1 reduce-scatter + all_gather", f"reduce={red}")

    # all_to_all_single with explicit splits from the launch stream
    src = torch.randn(300, 64, device=DEV)
    ev = None
    if not CPU:
        ev = torch.cuda.Event()
        ev.record()
    out = comm.alloc_for_launch((300, 64), src)
    w = comm.all_to_all_single(out, src, [300], [300], dist.group.WORLD, async_op=True, after=ev)
    w.wait()
    sync()
    assert torch.equal(out, src)
    step("all_to_all_single after=event")

    # EP dispatch / combine through RCCL (bf16 and fp8 payloads)
    seen = []
    orig = ep.EPPrep.splits

    def splits(self, P, El):
        seen.append(self.host is not None and (CPU or self.host.is_pinned()))
        return orig(self, P, El)
    ep.EPPrep.splits = splits
    for fp8 in fp8s:
        got = moe_run(dist.group.WORLD, fp8)
        want = ref_moe[fp8]
        for name, a, b in zip(("y", "dx", "dw13", "dw2"), got[:4], want[:4]):
            r = rel(a, b)
            assert r < (6e-2 if fp8 else 1e-2), (fp8, name, r)   # fp8 dispatch re-tiles dW's quantization
        step("ep dispatch", f"fp8={fp8}")
    ep.EPPrep.splits = orig
    assert seen and all(seen), seen
    step("ep pinned D2H split sizes", f"{len(seen)} layers")

    got = moe_run(dist.group.WORLD, False, aux_free=True)
    assert got[5] == 1, ("routing-bias all-reduce was not issued async", got[5])
    assert ref_bias[5] == 0
    assert torch.equal(got[4], ref_bias[4]) and got[4].abs().max() > 0
    step("async routing-bias all-reduce")
    sdist.cleanup()
    print("RCCL_WORLD1_OK", flush=True)


if __name__ == "__main__":
    main()
    sys.exit(0)
