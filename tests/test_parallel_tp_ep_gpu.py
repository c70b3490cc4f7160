"""Tensor- and expert-parallel rehearsal on the GPU box (VERDICT r1 'what's weak' #6).

The 1-GPU box cannot host two RCCL ranks (RCCL wants a device per rank), so two ranks share
cuda:0 over gloo (SPA_DIST_BACKEND=gloo; gloo moves CUDA tensors through host copies). What
runs on the device: the HIP kernels under the TP region ops (column/row-parallel projections,
vocab-parallel embedding + cross-entropy, sequence-parallel reduce-scatter / all-gather) and
under the EP dispatch (routing, permute, the ep_regroup kernel, bf16 and fp8 grouped GEMMs,
combine), each checked against ONE process running the unsharded model on the same card.
"""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _init(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), SPA_DIST_BACKEND="gloo")
    from solvingpapers_amd.parallel import dist as sdist
    info = sdist.init_distributed()
    assert info.backend == "gloo" and info.device == torch.device("cuda", 0)
    return sdist


def _spawn(fn, world, *args):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=fn, args=(r, world, port, q) + args) for r in range(world)]
    for p in ps:
        p.start()
    out = [q.get(timeout=110) for _ in ps]
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    return sorted(out, key=lambda r: r[0])


def _rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / b.norm().clamp_min(1e-12)).item()


# --------------------------------------------------------------------------- TP (Gemma)
def _gemma_cfg():
    from solvingpapers_amd.models import gemma
    return gemma.config("gemma_tiny", vocab_size=256, dim=256, n_heads=4, head_dim=64, ffn_hidden=512,
                        max_seq_len=128)


def _gemma_ids():
    return torch.randint(0, 256, (2, 66), generator=torch.Generator().manual_seed(2))


def _tp_worker(rank, world, port, q, mode, nb):
    sdist = _init(rank, world, port)
    import torch.distributed as dist
    from solvingpapers_amd.models import gemma
    from solvingpapers_amd.parallel.tensor_parallel import shard_gemma_from_full
    from solvingpapers_amd.utils.flat import FlatParams
    c = _gemma_cfg()
    full = gemma.Gemma(c, device="cuda:0", dtype=torch.bfloat16, seed=5)
    grp = dist.new_group([0, 1])
    local = gemma.Gemma(c, tp_group=grp, seed=5, sequence_parallel=mode != "plain",
                        tp_pipeline=mode in ("pair", "micro"), device="cuda:0", dtype=torch.bfloat16)
    shard_gemma_from_full(full, local, rank, world)
    FlatParams(local, grad_dtype=torch.float32)
    ids = _gemma_ids().cuda()[:nb]
    if mode == "pair":      # the overlapped chunk pair inside one forward
        assert local._pair_split(ids[:, :-2]) == ("batch" if nb == 2 else "sequence")
    if mode == "micro":     # two accumulation micro-batches as the pair (Gemma.forward_pair)
        loss = local.forward_pair(ids[:1, :-2], ids[:1, 1:-1], ids[1:, :-2], ids[1:, 1:-1])
    else:
        loss = local(ids[:, :-2], ids[:, 1:-1])
    loss.backward()
    local.sync_sequence_parallel_grads()
    torch.cuda.synchronize()
    grads = {n: p.main_grad.float().cpu().numpy() for n, p in local.named_parameters()}
    q.put((rank, float(loss), grads))
    sdist.cleanup()


@pytest.mark.parametrize("mode,nb", [("plain", 2), ("sp", 2), ("pair", 2), ("pair", 1), ("micro", 2)])
def test_gemma_tp2_on_one_gpu_matches_unsharded(mode, nb):
    from solvingpapers_amd.models import gemma
    from solvingpapers_amd.ops import _ext
    from solvingpapers_amd.utils.flat import FlatParams
    assert _ext.load(), "HIP extension must load on the GPU box"
    c = _gemma_cfg()
    full = gemma.Gemma(c, device="cuda:0", dtype=torch.bfloat16, seed=5)
    FlatParams(full, grad_dtype=torch.float32)
    ids = _gemma_ids().cuda()[:nb]
    if mode == "micro":
        loss = full(ids[:1, :-2], ids[:1, 1:-1]) + full(ids[1:, :-2], ids[1:, 1:-1])
    else:
        loss = full(ids[:, :-2], ids[:, 1:-1])
    loss.backward()
    fg = {n: p.main_grad.float().cpu() for n, p in full.named_parameters()}
    ref_loss = float(loss.detach())
    del full
    torch.cuda.synchronize()
    world = 2
    for rank, l, grads in _spawn(_tp_worker, world, mode, nb):
        assert abs(l - ref_loss) < 2e-2 * abs(ref_loss), (rank, l, ref_loss)
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
            assert _rel(g, f) < 3e-2, (rank, n, _rel(g, f))


# --------------------------------------------------------------------------- EP (DeepSeek MoE)
def _moe_cfg(fp8):
    from solvingpapers_amd.models import deepseekv3 as ds
    return ds.config("dsv3_tiny", dim=256, n_experts=8, top_k=2, n_shared=1, expert_hidden=256, aux_free=False,
                     moe_fp8=fp8)


def _moe_inputs():
    g = torch.Generator().manual_seed(7)
    x = torch.randn(2, 2, 64, 256, generator=g)          # [rank, B, T, D]
    gy = torch.randn(2, 2, 64, 256, generator=g)
    return x, gy


def _ep_worker(rank, world, port, q, fp8):
    sdist = _init(rank, world, port)
    import torch.distributed as dist
    from solvingpapers_amd.models import deepseekv3 as ds
    c = _moe_cfg(fp8)
    grp = dist.new_group([0, 1])
    m = ds.MoE(c, ep_group=grp, device="cuda:0", dtype=torch.bfloat16)
    m.reset_parameters(0.05, torch.Generator(device="cuda:0").manual_seed(3))
    x, gy = _moe_inputs()
    xr = x[rank].to("cuda:0", torch.bfloat16).requires_grad_(True)
    y = m(xr)
    (y.float() * gy[rank].cuda()).sum().backward()
    torch.cuda.synchronize()
    q.put((rank, y.detach().float().cpu().numpy(), xr.grad.float().cpu().numpy(), m.w13.grad.float().cpu().numpy(),
           m.w2.grad.float().cpu().numpy()))
    sdist.cleanup()


@pytest.mark.parametrize("fp8", [False, True])
def test_dsv3_moe_ep2_on_one_gpu_matches_local(fp8):
    """EP=2 (gloo all-to-all of CUDA rows, device regroup kernel, grouped GEMMs) == one process
    holding all 8 experts: outputs, input grads and each rank's expert grads."""
    from solvingpapers_amd.models import deepseekv3 as ds
    c = _moe_cfg(fp8)
    full = ds.MoE(c, device="cuda:0", dtype=torch.bfloat16)
    full.reset_parameters(0.05, torch.Generator(device="cuda:0").manual_seed(3))
    x, gy = _moe_inputs()
    xs = x.to("cuda:0", torch.bfloat16).requires_grad_(True)
    ys = [full(xs[r]) for r in range(2)]
    sum((y.float() * gy[r].cuda()).sum() for r, y in enumerate(ys)).backward()
    ref = [y.float().cpu() for y in ys]
    gx = xs.grad.float().cpu()
    g13, g2 = full.w13.grad.float().cpu(), full.w2.grad.float().cpu()
    del full
    torch.cuda.synchronize()
    tol = 6e-2 if fp8 else 2e-2
    El = c.n_experts // 2
    for rank, y, dx, w13g, w2g in _spawn(_ep_worker, 2, fp8):
        assert _rel(torch.from_numpy(y), ref[rank]) < tol, rank
        assert _rel(torch.from_numpy(dx), gx[rank]) < tol, rank
        assert _rel(torch.from_numpy(w13g), g13[rank * El:(rank + 1) * El]) < tol, rank
        assert _rel(torch.from_numpy(w2g), g2[rank * El:(rank + 1) * El]) < tol, rank


def test_ep_regroup_kernel_matches_index_path():
    """csrc/kernels/ep.hip: both directions against the vectorised index construction, with
    empty (src, expert) segments and bf16 / fp8-sized rows."""
    from solvingpapers_amd.parallel.expert_parallel import _em_dest, regroup_rows
    g = torch.Generator().manual_seed(0)
    for P, El, D, dt in ((2, 4, 256, torch.bfloat16), (8, 32, 7168, torch.bfloat16), (4, 3, 48, torch.uint8)):
        rc = torch.randint(0, 9, (P, El), generator=g)
        rc[0, 1] = 0
        rc[P - 1, El - 1] = 0
        R = int(rc.sum())
        x = (torch.randn(R, D, generator=g) * 50).to(dt) if dt != torch.uint8 else \
            torch.randint(0, 255, (R, D), generator=g, dtype=torch.uint8)
        dest = _em_dest(rc)
        want = torch.empty_like(x)
        want[dest] = x
        got = regroup_rows(x.cuda(), rc.cuda(), True).cpu()
        assert torch.equal(got, want), (P, El)
        back = regroup_rows(got.cuda(), rc.cuda(), False).cpu()
        assert torch.equal(back, x), (P, El)
