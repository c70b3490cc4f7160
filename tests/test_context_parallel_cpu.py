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
    q_out.put((rank, o.detach(), ql.grad, kl.grad, vl.grad))
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
    cat = lambda i: torch.cat([r[i] for r in res], dim=1)  # noqa: E731
    for i, want in ((1, o.detach()), (2, q.grad), (3, k.grad), (4, v.grad)):
        assert torch.allclose(cat(i), want, atol=1e-5, rtol=1e-4), i
