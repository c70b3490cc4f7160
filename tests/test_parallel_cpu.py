"""Distributed correctness without a cluster: gloo, world size 2 on CPU.

* DP: per-layer bucketed all-reduce during backward == single-process grads on the
  concatenated batch; ZeRO-1 (reduce-scatter + sharded AdamW + all-gather) == plain DP.
* TP: Gemma (MQA, vocab-parallel embedding/CE, column/row-parallel projections)
  sharded over 2 ranks == the unsharded model (loss and every gradient).
* EP: expert-parallel MoE (all-to-all dispatch/combine) == local MoE.
"""
import contextlib
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _init(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(0)


def _llama(seed=0):
    from solvingpapers_amd.models import llama3
    c = llama3.config("llama3_ref", vocab_size=64, dim=64, n_heads=4, n_kv_heads=2, ffn_hidden=128, init="std")
    return llama3.Llama3(c, seed=seed)


def _dp_worker(rank, world, port, q, zero1, accum=1, reduce=None):
    _init(rank, world, port)
    from solvingpapers_amd.parallel.data_parallel import DataParallel
    from solvingpapers_amd.train.optim import FlatAdamW
    from solvingpapers_amd.utils.flat import FlatParams
    m = _llama()
    flat = FlatParams(m, groups=m.param_groups(), align=64)
    dp = DataParallel(m, flat, zero1=zero1, reduce=reduce)
    shard = (dp.shard_ranges(), None) if zero1 else None
    opt = FlatAdamW(flat, lr=1e-2, weight_decay=0.1, max_grad_norm=1.0, shard=shard)
    g = torch.Generator().manual_seed(1)
    ids = torch.randint(0, 64, (4, 17), generator=g)
    per = 4 // world
    mine = ids[rank * per:(rank + 1) * per]
    for _ in range(2):
        opt.zero_grad()
        if accum == 1:
            m(mine[:, :-1], mine[:, 1:]).backward()
        else:  # one sample per micro-batch; communication only on the last one
            for i in range(accum):
                ctx = dp.no_sync() if i < accum - 1 else contextlib.nullcontext()
                with ctx:
                    (m(mine[i:i + 1, :-1], mine[i:i + 1, 1:]) / accum).backward()
        dp.finish_grad_sync()
        if zero1:
            grads = None
        else:
            grads = flat.grad.clone()
        opt.step()
        dp.gather_params()
    q.put((rank, None if grads is None else grads.numpy(), flat.param.clone().numpy()))
    dist.destroy_process_group()


def _run(fn, world, *args):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=fn, args=(r, world, port, q) + args) for r in range(world)]
    for p in ps:
        p.start()
    out = [q.get(timeout=300) for _ in ps]
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    return sorted(out, key=lambda x: x[0])


def _single_reference(steps=2):
    from solvingpapers_amd.train.optim import FlatAdamW
    from solvingpapers_amd.utils.flat import FlatParams
    m = _llama()
    flat = FlatParams(m, groups=m.param_groups(), align=64)
    opt = FlatAdamW(flat, lr=1e-2, weight_decay=0.1, max_grad_norm=1.0)
    g = torch.Generator().manual_seed(1)
    ids = torch.randint(0, 64, (4, 17), generator=g)
    grads = None
    for _ in range(steps):
        opt.zero_grad()
        # mean over the 2 halves == mean over ranks of per-rank means
        loss = 0.5 * (m(ids[:2, :-1], ids[:2, 1:]) + m(ids[2:, :-1], ids[2:, 1:]))
        loss.backward()
        grads = flat.grad.clone()
        opt.step()
    return grads, flat.param.clone()


def test_dp_grads_and_params_match_single_process():
    ref_g, ref_p = _single_reference()
    out = _run(_dp_worker, 2, False)
    for rank, g, p in out:
        g, p = torch.from_numpy(g), torch.from_numpy(p)
        assert torch.allclose(g, ref_g, atol=1e-5, rtol=1e-4), (rank, (g - ref_g).abs().max())
        assert torch.allclose(p, ref_p, atol=1e-5), (rank, (p - ref_p).abs().max())


@pytest.mark.parametrize("zero1", [False, True])
def test_dp_grad_accumulation_no_sync_matches_single_process(zero1):
    """bench.py --accum: inner micro-batches skip the bucket all-reduce (no_sync), the last
    one launches it; the result equals the un-accumulated single-process step."""
    ref_g, ref_p = _single_reference()
    out = _run(_dp_worker, 2, zero1, 2)
    for rank, g, p in out:
        if g is not None:
            g = torch.from_numpy(g)
            assert torch.allclose(g, ref_g, atol=1e-5, rtol=1e-4), (rank, (g - ref_g).abs().max())
        p = torch.from_numpy(p)
        assert torch.allclose(p, ref_p, atol=1e-5), (rank, (p - ref_p).abs().max())


@pytest.mark.parametrize("world,zero1,accum", [(2, False, 1), (2, True, 2), (4, False, 1), (4, True, 1)])
def test_dp_a2a_reduce_matches_single_process(world, zero1, accum):
    """reduce="a2a" (the bf16 default: one all-to-all of the bucket, an fp32 sum of the N received
    shard copies, then the all-gather; ZeRO-1 stops after the sum) equals the single-process step
    at world 2 and 4, with and without ZeRO-1 / accumulation."""
    ref_g, ref_p = _single_reference()
    out = _run(_dp_worker, world, zero1, accum, "a2a")
    for rank, g, p in out:
        if g is not None:
            g = torch.from_numpy(g)
            assert torch.allclose(g, ref_g, atol=1e-5, rtol=1e-4), (rank, (g - ref_g).abs().max())
        p = torch.from_numpy(p)
        assert torch.allclose(p, ref_p, atol=1e-5), (rank, (p - ref_p).abs().max())


def test_zero1_matches_dp():
    _, ref_p = _single_reference()
    out = _run(_dp_worker, 2, True)
    for rank, _, p in out:
        p = torch.from_numpy(p)
        assert torch.allclose(p, ref_p, atol=1e-5), (rank, (p - ref_p).abs().max())


def _tp_worker(rank, world, port, q, mode="plain", nb=2):
    _init(rank, world, port)
    from solvingpapers_amd.models import gemma
    from solvingpapers_amd.parallel.tensor_parallel import shard_gemma_from_full
    from solvingpapers_amd.utils.flat import FlatParams
    c = gemma.config("gemma_tiny", vocab_size=64, dim=64, n_heads=4, head_dim=16, ffn_hidden=128)
    full = gemma.Gemma(c, seed=5)
    grp = dist.new_group([0, 1])
    local = gemma.Gemma(c, tp_group=grp, seed=5, sequence_parallel=mode != "plain",
                        tp_pipeline=mode in ("pair", "micro"))
    assert local.sp == (mode != "plain")
    shard_gemma_from_full(full, local, rank, world)
    flat = FlatParams(local)
    ids = torch.randint(0, 64, (2, 13), generator=torch.Generator().manual_seed(2))[:nb]
    if mode == "pair":
        assert local._pair_split(ids[:, :-1]) == ("batch" if nb == 2 else "sequence")
    if mode == "micro":
        loss = local.forward_pair(ids[:1, :-1], ids[:1, 1:], ids[1:, :-1], ids[1:, 1:])
    else:
        loss = local(ids[:, :-1], ids[:, 1:])
    loss.backward()
    local.sync_sequence_parallel_grads()
    grads = {n: p.main_grad.clone().numpy() for n, p in local.named_parameters()}
    from solvingpapers_amd.train.optim import FlatAdamW
    gn = FlatAdamW(flat, max_grad_norm=1.0, tp_group=grp).grad_norm().item()
    q.put((rank, loss.item(), (grads, gn)))
    dist.destroy_process_group()


@pytest.mark.parametrize("mode,nb", [("plain", 2), ("sp", 2), ("pair", 2), ("pair", 1), ("micro", 2)])
def test_tensor_parallel_gemma_matches_unsharded(mode, nb):
    """TP=2 == the unsharded model: plain Megatron TP ("plain"); sequence parallelism ("sp":
    reduce-scatter / all-gather over T, norms and the MQA K/V projection on sequence shards,
    their grads summed over TP); and the overlapped chunk pair under SP ("pair", Gemma.
    _forward_sp_pair): batch halves (nb 2) or sequence halves with half B attending to half
    A's K/V (nb 1); and Gemma.forward_pair over two micro-batches ("micro": == the sum of the
    two micro-batch losses)."""
    from solvingpapers_amd.models import gemma
    from solvingpapers_amd.utils.flat import FlatParams
    c = gemma.config("gemma_tiny", vocab_size=64, dim=64, n_heads=4, head_dim=16, ffn_hidden=128)
    full = gemma.Gemma(c, seed=5)
    FlatParams(full)
    ids = torch.randint(0, 64, (2, 13), generator=torch.Generator().manual_seed(2))[:nb]
    if mode == "micro":
        loss = full(ids[:1, :-1], ids[:1, 1:]) + full(ids[1:, :-1], ids[1:, 1:])
    else:
        loss = full(ids[:, :-1], ids[:, 1:])
    loss.backward()
    fg = {n: p.main_grad for n, p in full.named_parameters()}
    out = _run(_tp_worker, 2, mode, nb)
    world = 2
    full_norm = torch.sqrt(sum((g.float() ** 2).sum() for g in fg.values())).item()
    for rank, l, (grads, gn) in out:
        assert abs(l - loss.item()) < 1e-5
        assert abs(gn - full_norm) < 1e-4 * full_norm, (gn, full_norm)   # TP-aware global grad norm
        for n, g in grads.items():
            g = torch.from_numpy(g)
            f = fg[n]
            if n == "embed":
                vl = f.shape[0] // world
                f = f[rank * vl:(rank + 1) * vl]
            elif n.endswith(".wq"):
                h = f.shape[0] // world
                f = f[rank * h:(rank + 1) * h]
            elif n.endswith(".wo") or n.endswith(".w2"):
                h = f.shape[1] // world
                f = f[:, rank * h:(rank + 1) * h]
            elif n.endswith(".w13"):
                F2 = f.shape[0] // 2
                fl = F2 // world
                f = torch.cat([f[rank * fl:(rank + 1) * fl], f[F2 + rank * fl:F2 + (rank + 1) * fl]])
            assert torch.allclose(g, f, atol=1e-5, rtol=1e-4), (n, (g - f).abs().max())


def _moe_cfg():
    from solvingpapers_amd.models import deepseekv3 as ds
    return ds.config("dsv3_tiny", dim=32, n_experts=4, top_k=2, n_shared=1, expert_hidden=24, aux_free=False)


def _moe_inputs():
    g = torch.Generator().manual_seed(7)
    x = torch.randn(2, 2, 6, 32, generator=g)          # [rank, B, T, D]
    gy = torch.randn(2, 2, 6, 32, generator=g)
    return x, gy


def _ep_worker(rank, world, port, q, mode="plain"):
    _init(rank, world, port)
    from dataclasses import replace
    from solvingpapers_amd.models import deepseekv3 as ds
    from solvingpapers_amd.parallel import expert_parallel as ep
    from solvingpapers_amd.parallel.expert_parallel import shard_experts
    c = _moe_cfg()
    if mode == "capacity":
        # host-sync-free padded dispatch; capacity 4 = the exact bound here (never overflows), and
        # the split-size host read must never happen
        c = replace(c, ep_capacity=4.0)

        def no_host_sync(*a, **k):
            raise AssertionError("capacity mode read the split sizes on the host")
        ep.EPPrep.splits = no_host_sync
    torch.manual_seed(0)
    full = ds.MoE(c)
    full.reset_parameters(0.1, torch.Generator().manual_seed(3))
    grp = dist.new_group([0, 1])
    m = ds.MoE(c, ep_group=grp)
    # the EP constructor's own init: rank r holds shard_experts(unsharded init, r, P), i.e.
    # distinct experts on every rank (not E/P experts drawn again from the shared sequence)
    m.reset_parameters(0.1, torch.Generator().manual_seed(3))
    assert torch.equal(m.w13, shard_experts(full.w13, rank, world))
    assert torch.equal(m.w2, shard_experts(full.w2, rank, world))
    assert torch.equal(m.gate, full.gate) and torch.equal(m.shared.w13, full.shared.w13)
    x, gy = _moe_inputs()
    xr = x[rank].clone().requires_grad_(True)
    y = m(xr)
    (y * gy[rank]).sum().backward()
    if mode == "capacity":
        assert not ep.capacity_overflowed()
    q.put((rank, y.detach().numpy(), xr.grad.numpy(), m.w13.grad.numpy(), m.w2.grad.numpy(), m.gate.grad.numpy()))
    dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["plain", "capacity"])
def test_expert_parallel_moe_matches_local(mode):
    """EP=2 (all-to-all dispatch/combine, 2 experts per rank) == one process holding all
    4 experts: outputs, input grads, and each rank's expert grads (which collect the
    contributions of BOTH ranks' tokens), through the staged layer (one exchange each way)."""
    from solvingpapers_amd.models import deepseekv3 as ds
    c = _moe_cfg()
    torch.manual_seed(0)
    full = ds.MoE(c)
    full.reset_parameters(0.1, torch.Generator().manual_seed(3))
    x, gy = _moe_inputs()
    xs = x.clone().requires_grad_(True)
    ys = [full(xs[r]) for r in range(2)]
    sum((y * gy[r]).sum() for r, y in enumerate(ys)).backward()
    out = _run(_ep_worker, 2, mode)
    for rank, y, gx, g13, g2, gg in out:
        assert torch.allclose(torch.from_numpy(y), ys[rank].detach(), atol=1e-5)
        assert torch.allclose(torch.from_numpy(gx), xs.grad[rank], atol=1e-5)
        assert torch.allclose(torch.from_numpy(g13), full.w13.grad[rank * 2:(rank + 1) * 2], atol=1e-5)
        assert torch.allclose(torch.from_numpy(g2), full.w2.grad[rank * 2:(rank + 1) * 2], atol=1e-5)
        # gate grads are rank-local (DP all-reduces them later)


class _NanOnRank(torch.nn.Module):
    """Wraps a model; rank ``bad_rank`` returns a NaN loss at training step ``bad_step``."""

    def __init__(self, inner, bad_rank, bad_step):
        super().__init__()
        self.inner, self.bad_rank, self.bad_step, self.calls = inner, bad_rank, bad_step, 0

    def param_groups(self):
        return self.inner.param_groups()

    def forward(self, x, y):
        loss = self.inner(x, y)
        if self.training:
            if dist.get_rank() == self.bad_rank and self.calls == self.bad_step:
                loss = loss * float("nan")
            self.calls += 1
        return loss


def _nan_worker(rank, world, port, q, zero1):
    _init(rank, world, port)
    from solvingpapers_amd.train.trainer import TrainConfig, Trainer
    m = _NanOnRank(_llama(seed=rank), bad_rank=1, bad_step=1)   # different seeds: broadcast must fix
    g = torch.Generator().manual_seed(1)
    ids = torch.randint(0, 64, (8, 17), generator=g)

    def batch(i):
        j = (2 * i + rank) % 4
        return ids[2 * j:2 * j + 2, :-1], ids[2 * j:2 * j + 2, 1:]
    tr = Trainer(m, TrainConfig(steps=4, lr=1e-2, zero1=zero1, max_bad_steps=3), batch)
    snap = {}
    orig = tr.train_step

    def spy(s):
        out = orig(s)
        snap[s] = tr.flat.param.clone()
        return out
    tr.train_step = spy
    tr.fit()
    oks = [h["ok"] for h in tr.history if "loss" in h]
    q.put((rank, oks, {k: v.numpy() for k, v in snap.items()}))
    dist.destroy_process_group()


@pytest.mark.parametrize("zero1", [False, True])
def test_nan_on_one_rank_skips_update_on_every_rank(zero1):
    """a NaN on ONE rank must make EVERY rank skip the same step (no
    mismatched collectives, no divergence). The skip is decided on the globally reduced grad
    norm inside the fused optimizer kernel; ranks also start identical (broadcast before the
    optimizer copies its fp32 master)."""
    out = _run(_nan_worker, 2, zero1)
    (_, ok0, s0), (_, ok1, s1) = out
    assert ok0 == ok1 == [True, False, True, True]
    for s in range(4):
        assert (s0[s] == s1[s]).all(), s                  # replicas never diverge
    assert (s0[1] == s0[0]).all()                          # step 1 applied no update
    assert not (s0[2] == s0[1]).all()                      # later steps do


def _ep_fp8_inputs():
    g = torch.Generator().manual_seed(11)
    E, D, F, N, k = 4, 128, 128, 24, 2
    x = torch.randn(2, N, D, generator=g)
    idx = torch.stack([torch.randperm(E, generator=g)[:k] for _ in range(2 * N)]).view(2, N, k).int()
    w = torch.rand(2, N, k, generator=g)
    W13 = torch.randn(E, 2 * F, D, generator=g) * 0.05
    W2 = torch.randn(E, D, F, generator=g) * 0.05
    gy = torch.randn(2, N, D, generator=g)
    return x, idx, w, W13, W2, gy


def _ep_fp8_worker(rank, world, port, q, capacity=0.0):
    _init(rank, world, port)
    from solvingpapers_amd.parallel.expert_parallel import ep_moe_ffn, shard_experts
    x, idx, w, W13, W2, gy = _ep_fp8_inputs()
    grp = dist.new_group([0, 1])
    w13 = shard_experts(W13, rank, world).clone().requires_grad_(True)
    w2 = shard_experts(W2, rank, world).clone().requires_grad_(True)
    xr = x[rank].clone().requires_grad_(True)
    from solvingpapers_amd.parallel import comm
    seen = []
    real = comm.all_to_all_single

    def spy(out, inp, out_splits, in_splits, group, async_op=False, after=None):
        seen.append((str(inp.dtype), inp.shape[1] * inp.element_size()))
        return real(out, inp, out_splits, in_splits, group, async_op=async_op, after=after)
    comm.all_to_all_single = spy
    boxes, init = [], comm._Box.__init__

    def track(self):
        init(self)
        boxes.append(self)
    comm._Box.__init__ = track
    y, _ = ep_moe_ffn(xr, idx[rank], w[rank], w13, w2, 4, grp, fp8=True, capacity=capacity)
    (y * gy[rank]).sum().backward()
    comm.all_to_all_single = real
    comm._Box.__init__ = init
    # every exchange's Work (which holds its input and output buffers) and pending buffer is
    # released once waited: on RCCL a retained Work kept ~3 GB per MoE layer and micro-batch alive
    assert len(boxes) >= 2
    for b in boxes:
        assert b.work is None and b.bwork is None and b.dx is None and b.gkeep is None and b.recv is None
    if capacity:
        from solvingpapers_amd.parallel.expert_parallel import capacity_overflowed
        assert not capacity_overflowed()
    q.put((rank, y.detach().numpy(), xr.grad.numpy(), w13.grad.numpy(), w2.grad.numpy(), seen))
    dist.destroy_process_group()


@pytest.mark.parametrize("capacity", [0.0, 4.0])
def test_expert_parallel_fp8_dispatch_matches_local_fp8(capacity):
    """fp8 dispatch (e4m3 rows + E8M0 1x128 scales over the all-to-all, fused with the
    block-scaled W13 GEMM) == the single-process block-scaled fp8 MoE: outputs and input grads
    to fp32 rounding; expert grads to the fp8 rounding of the dW operands (the EP path forms dW13
    from the dequantized received rows, as DeepSeek-V3 does, and both paths quantize the dW
    operands in 128-token tiles that group the two ranks' tokens differently)."""
    from solvingpapers_amd.ops.moe import moe_ffn
    x, idx, w, W13, W2, gy = _ep_fp8_inputs()
    W13r, W2r = W13.clone().requires_grad_(True), W2.clone().requires_grad_(True)
    xs = x.clone().requires_grad_(True)
    ys = [moe_ffn(xs[r], idx[r], w[r], W13r, W2r, fp8=True)[0] for r in range(2)]
    sum((y * gy[r]).sum() for r, y in enumerate(ys)).backward()
    for rank, y, gx, g13, g2, seen in _run(_ep_fp8_worker, 2, capacity):
        # the default EP path's dispatch payload: e4m3 rows + E8M0 scales, 144 B per 128-wide row
        # (128 + 1 scale byte, padded to 16) -- 0.56x a bf16 row; combine and the backward's dX in
        # the activation dtype
        assert seen[0] == ("torch.uint8", 128 + 16), seen
        assert all(dt != "torch.uint8" for dt, _ in seen[1:]), seen
        assert torch.allclose(torch.from_numpy(y), ys[rank].detach(), atol=1e-4)
        assert torch.allclose(torch.from_numpy(gx), xs.grad[rank], atol=1e-4)
        ref13 = W13r.grad[rank * 2:(rank + 1) * 2]
        assert ((torch.from_numpy(g13) - ref13).norm() / ref13.norm()) < 5e-2
        ref2 = W2r.grad[rank * 2:(rank + 1) * 2]           # fp8 dW: 128-token quantization blocks
        assert ((torch.from_numpy(g2) - ref2).norm() / ref2.norm()) < 5e-2   # group tokens differently


def _gemma_tp_cfg():
    from solvingpapers_amd.models import gemma
    return gemma.config("gemma_tiny", vocab_size=64, dim=64, n_heads=4, head_dim=16, ffn_hidden=128)


def _trainer_batches():
    ids = torch.randint(0, 64, (2, 13), generator=torch.Generator().manual_seed(3))
    return lambda i: (ids[:, :-1], ids[:, 1:])


def _trainer_tp_worker(rank, world, port, q):
    _init(rank, world, port)
    from solvingpapers_amd.models import gemma
    from solvingpapers_amd.parallel.groups import build_groups
    from solvingpapers_amd.train.trainer import TrainConfig, Trainer
    groups = build_groups(tp=2)
    local = gemma.Gemma(_gemma_tp_cfg(), tp_group=groups.tp_group, seed=5)
    tr = Trainer(local, TrainConfig(steps=3, lr=1e-2, clip=1.0, resume="never"), _trainer_batches(), groups=groups)
    assert tr.dp is None and tr.dp_size == 1
    tr.fit()
    q.put((rank, {n: p.detach().clone().numpy() for n, p in local.named_parameters()}))
    dist.destroy_process_group()


def test_trainer_tensor_parallel_keeps_shards_and_matches_unsharded():
    """Trainer(groups=tp=world) must not wrap a DataParallel over the world (it would
    broadcast rank 0's shards and average different shards' gradients). After 3 AdamW steps with
    TP-aware clipping each rank's shards equal the slices of the unsharded run."""
    from solvingpapers_amd.models import gemma
    from solvingpapers_amd.train.trainer import TrainConfig, Trainer
    full = gemma.Gemma(_gemma_tp_cfg(), seed=5)
    Trainer(full, TrainConfig(steps=3, lr=1e-2, clip=1.0, resume="never"), _trainer_batches()).fit()
    fp = {n: p.detach() for n, p in full.named_parameters()}
    out = _run(_trainer_tp_worker, 2)
    world = 2
    assert not torch.equal(torch.from_numpy(out[0][1]["layers.0.wq"]), torch.from_numpy(out[1][1]["layers.0.wq"]))
    for rank, params in out:
        for n, g in params.items():
            g = torch.from_numpy(g)
            f = fp[n]
            if n == "embed":
                vl = f.shape[0] // world
                f = f[rank * vl:(rank + 1) * vl]
            elif n.endswith(".wq"):
                h = f.shape[0] // world
                f = f[rank * h:(rank + 1) * h]
            elif n.endswith(".wo") or n.endswith(".w2"):
                h = f.shape[1] // world
                f = f[:, rank * h:(rank + 1) * h]
            elif n.endswith(".w13"):
                F2 = f.shape[0] // 2
                fl = F2 // world
                f = torch.cat([f[rank * fl:(rank + 1) * fl], f[F2 + rank * fl:F2 + (rank + 1) * fl]])
            assert torch.allclose(g, f, atol=1e-4, rtol=1e-3), (rank, n, (g - f).abs().max())


def _pair_worker(rank, world, port, q, aux_free):
    _init(rank, world, port)
    from solvingpapers_amd.models import deepseekv3 as ds
    c = ds.config("dsv3_tiny", vocab_size=64, dim=32, n_heads=2, kv_lora_rank=16, qk_nope_dim=8, qk_rope_dim=8,
                  v_head_dim=16, n_experts=4, top_k=2, expert_hidden=24, dense_hidden=48, n_layers=3,
                  n_dense_layers=1, mtp_heads=1, aux_free=aux_free)
    grp = dist.new_group([0, 1]) if world > 1 else None
    g = torch.Generator().manual_seed(5)
    ids = torch.randint(0, 64, (2, world, 2, 13), generator=g)       # [micro-batch, rank, B, T+1]
    res = {}
    for mode in ("two_calls", "pair"):
        m = ds.DeepSeekV3(c, seed=3, ep_group=grp)
        x0, y0 = ids[0, rank, :, :-1], ids[0, rank, :, 1:]
        x1, y1 = ids[1, rank, :, :-1], ids[1, rank, :, 1:]
        if mode == "pair":
            loss = m.forward_pair(x0, y0, x1, y1)
        else:
            loss = m(x0, y0) + m(x1, y1)
        loss.backward()
        m.finish_pending_updates()
        res[mode] = (float(loss), {n: p.grad.clone() for n, p in m.named_parameters() if p.grad is not None},
                     [l.routing_bias.clone() for l in m.moe_layers()])
    (l2, g2, b2), (lp, gp, bp) = res["two_calls"], res["pair"]
    ok = abs(l2 - lp) < 1e-5 and set(g2) == set(gp) and all(torch.allclose(g2[k], gp[k], atol=1e-5) for k in g2)
    # each MoE layer moves its routing bias right after micro-batch 0's routing, so micro-batch 1
    # routes with it in both modes (the reference's update-after-every-forward order)
    ok = ok and all(torch.equal(a, b) for a, b in zip(b2, bp))
    if aux_free:
        ok = ok and all(b.abs().max() > 0 for b in bp)
    q.put((rank, ok, l2, lp))
    if world > 1:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,aux_free", [(1, False), (2, False), (2, True)])
def test_dsv3_forward_pair_matches_two_forwards(world, aux_free):
    """DeepSeekV3.forward_pair (two micro-batches, layer-interleaved so each all-to-all overlaps
    the other micro-batch's compute) == two forward() calls: loss, every gradient and the routing
    biases (updated from the load counts) -- on one rank and on EP=2 (gloo), dense + MoE + MTP
    layers."""
    for rank, ok, l2, lp in _run(_pair_worker, world, aux_free):
        assert ok, (rank, l2, lp)


def _gemma_dp_pair_worker(rank, world, port, q, forced_pair):
    _init(rank, world, port)
    from solvingpapers_amd.models import gemma
    from solvingpapers_amd.train.trainer import TrainConfig, Trainer
    m = gemma.Gemma(_gemma_tp_cfg(), seed=5)
    assert not m.pair_overlaps()
    calls = []
    if forced_pair:   # the Trainer pairs only on an overlap: force it; TP 1 takes the fallback pair
        m.pair_overlaps = lambda: True
        real_fp = m.forward_pair
        m.forward_pair = lambda *a: calls.append(1) or real_fp(*a)
    ids = torch.randint(0, 64, (4, world, 2, 13), generator=torch.Generator().manual_seed(7))
    tr = Trainer(m, TrainConfig(steps=2, grad_accum=2, lr=1e-2, clip=1.0, resume="never"),
                 lambda i: (ids[i, rank, :, :-1], ids[i, rank, :, 1:]))
    assert tr.dp is not None
    tr.fit()
    assert len(calls) == (2 if forced_pair else 0)
    q.put((rank, tr.flat.param.clone().numpy()))
    dist.destroy_process_group()


def test_gemma_dp_paired_fallback_matches_one_by_one():
    """Gemma.forward_pair at TP 1 runs the two micro-batches one after the other
    under ONE backward; its layer markers must fire the DP bucket only after BOTH micro-batches'
    backward passed them (_PairReady), or the async all-reduce races micro-batch 0's commits.
    DP = 2 (gloo), grad_accum 2: paired fallback == unpaired loop, identical on both ranks."""
    ref = _run(_gemma_dp_pair_worker, 2, False)
    out = _run(_gemma_dp_pair_worker, 2, True)
    p0 = torch.from_numpy(ref[0][1])
    for (_, a), (_, b) in zip(ref, out):
        a, b = torch.from_numpy(a), torch.from_numpy(b)
        assert torch.allclose(a, p0, atol=1e-6)
        assert torch.allclose(b, p0, atol=1e-5), (b - p0).abs().max()


def test_forced_collectives_world1_gloo():
    """SPA_FORCE_COLLECTIVES=1 at world size 1 (the path tests/test_rccl_gpu.py drives through RCCL
    on the GPU box): DP buckets, ZeRO-1, the launch all-to-all, the EP exchange and the async
    routing-bias all-reduce run through a real size-1 gloo group and match the group-less run."""
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(here)
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(_port()), SPA_FORCE_COLLECTIVES="1", SPA_TEST_DEVICE="cpu",
               SPA_DIST_BACKEND="gloo", PYTHONPATH=root + os.pathsep + os.environ.get("PYTHONPATH", ""))
    r = subprocess.run([sys.executable, "-u", os.path.join(here, "rccl_world1_child.py")], env=env, cwd=root,
                       timeout=300, capture_output=True, text=True)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    assert "RCCL_WORLD1_OK" in r.stdout


def _cap_overflow_worker(rank, world, port, q, fp8):
    """DeepSeekV3 EP=2 with a capacity far below the routed load: every forward overflows first,
    is re-run with each layer's rows set from the load it saw, and must then equal the exact-split
    model."""
    _init(rank, world, port)
    from dataclasses import replace
    from solvingpapers_amd.models import deepseekv3 as ds
    from solvingpapers_amd.parallel import expert_parallel as ep
    c = ds.config("dsv3_tiny", dim=128, n_experts=4, top_k=2, expert_hidden=128, n_layers=2, n_dense_layers=0,
                  dropout=0.0, attn_dropout=0.0, moe_fp8=fp8)
    grp = dist.new_group([0, 1])
    g = torch.Generator().manual_seed(5)
    ids = torch.randint(0, c.vocab_size, (2, 2, 33), generator=g)[rank]
    res = {}
    for cap in (0.0, 0.1):
        m = ds.DeepSeekV3(replace(c, ep_capacity=cap), seed=3, ep_group=grp)
        m.train()
        calls = []
        real = m._forward
        m._forward = lambda *a, _r=real, **k: (calls.append(1), _r(*a, **k))[1]
        loss = m(ids[:, :-1], ids[:, 1:])
        loss.backward()
        m.finish_pending_updates()
        res[cap] = (loss.item(), {n: p.grad.clone() for n, p in m.named_parameters() if p.grad is not None},
                    [l.routing_bias.clone() for l in m.moe_layers()], len(calls))
    (l0, g0, b0, n0), (l1, g1, b1, n1) = res[0.0], res[0.1]
    # the tiny capacity overflowed once; the layers' capacity states then track the loads, so the
    # re-run fits
    assert n0 == 1 and n1 == 2, (n0, n1)
    assert abs(l0 - l1) < 1e-5, (l0, l1)
    assert g0.keys() == g1.keys()
    for n in g0:
        assert torch.allclose(g0[n], g1[n], atol=1e-5, rtol=1e-4), (n, (g0[n] - g1[n]).abs().max())
    for a, b in zip(b0, b1):                            # the bias moved once, not once per attempt
        assert torch.equal(a, b)
    q.put((rank, n1))
    dist.destroy_process_group()


@pytest.mark.parametrize("fp8", [False, True])
def test_ep_capacity_overflow_reruns_exactly(fp8):
    out = _run(_cap_overflow_worker, 2, fp8)
    assert len(out) == 2 and out[0][1] == out[1][1]     # both ranks agreed on every re-run


def _cap_decode_worker(rank, world, port, q, mode):
    """Capacity-mode EP (ep_capacity > 0) at EP=2 on the inference paths: step() with a cache takes
    the exact dispatch, the "bound" dispatch (graph decode) uses never-overflowing fixed blocks, and
    neither leaves overflow flags behind; forward() falls back to the exact dispatch after
    _CAP_ATTEMPTS overflowing attempts instead of raising."""
    _init(rank, world, port)
    from dataclasses import replace
    from solvingpapers_amd.models import deepseekv3 as ds
    from solvingpapers_amd.parallel import expert_parallel as ep
    c = ds.config("dsv3_tiny", dim=128, n_experts=4, top_k=2, expert_hidden=128, n_layers=2, n_dense_layers=0,
                  dropout=0.0, attn_dropout=0.0, mtp_heads=0)
    grp = dist.new_group([0, 1])
    g = torch.Generator().manual_seed(7)
    ids = torch.randint(0, c.vocab_size, (2, 2, 17), generator=g)[rank]
    ref = ds.DeepSeekV3(replace(c, ep_capacity=0.0), seed=3, ep_group=grp).eval()
    cap = ds.DeepSeekV3(replace(c, ep_capacity=0.1), seed=3, ep_group=grp).eval()
    with torch.no_grad():
        if mode == "step":
            outs = []
            for m in (ref, cap):
                cache = m.new_cache(2, 32)
                a = m.step(ids[:, :12], cache, 0)
                b = m.step(ids[:, 12:13], cache, 12)
                outs.append((a, b))
            assert not ep._CAP["pending"], "step() left capacity flags behind"
            for x, y in zip(*outs):
                assert torch.allclose(x, y, atol=1e-5, rtol=1e-4), (x - y).abs().max()
        elif mode == "bound":
            n0, _ = ref.hidden(ids)
            with cap.ep_dispatch("bound"):
                n1, _ = cap.hidden(ids)
            assert not ep._CAP["pending"], "bound dispatch set overflow flags"
            assert torch.allclose(n0, n1, atol=1e-5, rtol=1e-4), (n0 - n1).abs().max()
        else:                                   # "fallback": one capacity attempt, then exact
            cap.train()
            ref.train()
            cap._CAP_ATTEMPTS = 1
            calls = []
            real = cap._forward
            cap._forward = lambda *a, _r=real, **k: (calls.append(1), _r(*a, **k))[1]
            l1 = cap(ids[:, :-1], ids[:, 1:]).item()
            l0 = ref(ids[:, :-1], ids[:, 1:]).item()
            assert len(calls) == 2 and abs(l0 - l1) < 1e-5, (calls, l0, l1)
            assert all(m.dispatch_mode is None for m in cap.moe_layers())
    q.put((rank, mode))
    dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["step", "bound", "fallback"])
def test_ep_capacity_inference_paths_and_fallback(mode):
    out = _run(_cap_decode_worker, 2, mode)
    assert len(out) == 2
