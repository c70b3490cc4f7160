"""Context parallelism (parallel/context_parallel.py): sequence-sharded attention over 2 gloo
ranks (all-to-all sequence <-> head exchange) == single-process attention on the full sequence,
forward and every input gradient; GQA (kv heads split) and MQA (kv replicated)."""
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


def _inputs(Hkv):
    g = torch.Generator().manual_seed(0)
    B, T, H, hd = 2, 12, 4, 8
    q = torch.randn(B, T, H, hd, generator=g)
    k = torch.randn(B, T, Hkv, hd, generator=g)
    v = torch.randn(B, T, Hkv, hd, generator=g)
    do = torch.randn(B, T, H, hd, generator=g)
    return q, k, v, do


def _worker(rank, world, port, Hkv, causal, q_out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from solvingpapers_amd.parallel.context_parallel import context_parallel_attention
    q, k, v, do = _inputs(Hkv)
    Tl = q.shape[1] // world
    sl = slice(rank * Tl, (rank + 1) * Tl)
    ql, kl, vl = (t[:, sl].clone().requires_grad_() for t in (q, k, v))
    o = context_parallel_attention(ql, kl, vl, causal=causal)
    o.backward(do[:, sl])
    # numpy, not torch tensors: a torch tensor on an mp queue is a shared-memory handle whose
    # backing file can vanish when this worker exits before the parent reads it
    q_out.put((rank, o.detach().numpy(), ql.grad.numpy(), kl.grad.numpy(), vl.grad.numpy()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("Hkv,causal", [(2, True), (1, True), (4, False)])
def test_context_parallel_attention_matches_full(Hkv, causal):
    from solvingpapers_amd.ops import flash_attention
    world = 2
    ctx = mp.get_context("spawn")
    q_out = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, Hkv, causal, q_out)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q_out.get(timeout=120) for _ in range(world)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    q, k, v, do = _inputs(Hkv)
    q, k, v = (t.clone().requires_grad_() for t in (q, k, v))
    o = flash_attention(q, k, v, causal=causal)
    o.backward(do)
    cat = lambda i: torch.cat([torch.from_numpy(r[i]) for r in res], dim=1)  # noqa: E731
    for i, want in ((1, o.detach()), (2, q.grad), (3, k.grad), (4, v.grad)):
        assert torch.allclose(cat(i), want, atol=1e-5, rtol=1e-4), i


def _llama_worker(rank, world, port, q_out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from solvingpapers_amd.models import llama3
    c = llama3.config("llama3_ref", vocab_size=64, dim=64, n_heads=4, n_kv_heads=2, ffn_hidden=128, init="std")
    m = llama3.Llama3(c, seed=0).set_context_parallel(dist.group.WORLD)
    ids = torch.randint(0, 64, (2, 17), generator=torch.Generator().manual_seed(1))
    Tl = 16 // world
    sl = slice(rank * Tl, (rank + 1) * Tl)
    loss = m(ids[:, :-1][:, sl], ids[:, 1:][:, sl])
    loss.backward()
    grads = {}
    for n, p in m.named_parameters():
        g = p.grad.clone()
        dist.all_reduce(g)
        grads[n] = (g / world).numpy()
    lt = loss.detach().clone()
    dist.all_reduce(lt)
    q_out.put((rank, float(lt) / world, grads))
    dist.barrier()
    dist.destroy_process_group()


def test_llama_context_parallel_matches_single_process():
    from solvingpapers_amd.models import llama3
    world = 2
    ctx = mp.get_context("spawn")
    q_out = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_llama_worker, args=(r, world, port, q_out)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q_out.get(timeout=180) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    c = llama3.config("llama3_ref", vocab_size=64, dim=64, n_heads=4, n_kv_heads=2, ffn_hidden=128, init="std")
    m = llama3.Llama3(c, seed=0)
    ids = torch.randint(0, 64, (2, 17), generator=torch.Generator().manual_seed(1))
    loss = m(ids[:, :-1], ids[:, 1:])
    loss.backward()
    _, l_cp, grads = res[0]
    assert abs(l_cp - loss.item()) < 1e-5
    for n, p in m.named_parameters():
        assert torch.allclose(torch.from_numpy(grads[n]), p.grad, atol=1e-5, rtol=1e-4), n
