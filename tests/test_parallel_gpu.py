"""Multi-rank DP on the GPU box (SURVEY §4.2 T5 rehearsal on one card).

The driver's 1-GPU box cannot host two RCCL ranks (RCCL needs a device per rank), so two
ranks share cuda:0 over gloo (SPA_DIST_BACKEND=gloo; gloo all-reduces CUDA tensors through
host copies). What this covers on the device: the HIP kernels under the per-layer
gradient-ready hooks, async bucket all-reduce launched mid-backward, no_sync accumulation,
and the flat AdamW step — against one process running the same two micro-batches.
"""
import contextlib
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


def _model(seq=256):
    from solvingpapers_amd.models import llama3
    c = llama3.config("llama3_tiny", max_seq_len=seq)
    return llama3.Llama3(c, device="cuda:0", dtype=torch.bfloat16, seed=3)


def _ids(seq=256):
    g = torch.Generator().manual_seed(7)
    return torch.randint(0, 1024, (4, seq + 1), generator=g)


def _setup(m):
    from solvingpapers_amd.train.optim import FlatAdamW
    from solvingpapers_amd.utils.flat import FlatParams
    flat = FlatParams(m, groups=m.param_groups(), grad_dtype=torch.float32, align=64)
    opt = FlatAdamW(flat, lr=1e-3, weight_decay=0.1, max_grad_norm=1.0)
    return flat, opt


def _worker(rank, world, port, q, accum, seq):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), SPA_DIST_BACKEND="gloo")
    from solvingpapers_amd.parallel import dist as sdist
    from solvingpapers_amd.parallel.data_parallel import DataParallel
    info = sdist.init_distributed()
    assert info.backend == "gloo" and info.device == torch.device("cuda", 0)
    m = _model(seq)
    flat, opt = _setup(m)
    dp = DataParallel(m, flat)
    ids = _ids(seq).cuda()[rank * 2:(rank + 1) * 2]
    opt.zero_grad()
    for i in range(accum):
        x = ids[i * 2 // accum:(i + 1) * 2 // accum]
        with (dp.no_sync() if i < accum - 1 else contextlib.nullcontext()):
            (m(x[:, :-1], x[:, 1:]) / accum).backward()
    dp.finish_grad_sync()
    g = flat.grad.float().cpu().clone()
    opt.step()
    torch.cuda.synchronize()
    q.put((rank, g.numpy(), flat.param.float().cpu().numpy()))
    sdist.cleanup()


# seq 1024, accum 1: 2048 tokens per rank's micro-batch, so the feed-forward takes swiglu_mlp's
# transposed-operand weight gradients (ops/linear.py, T >= 2048) under the DP bucket hooks
@pytest.mark.parametrize("accum,seq", [(1, 256), (2, 256), (1, 1024)])
def test_dp2_gloo_on_one_gpu_matches_single_process(accum, seq):
    from solvingpapers_amd.ops import _ext
    assert _ext.load(), "HIP extension must load on the GPU box"
    m = _model(seq)
    flat, opt = _setup(m)
    ids = _ids(seq).cuda()
    opt.zero_grad()
    loss = 0.5 * (m(ids[:2, :-1], ids[:2, 1:]) + m(ids[2:, :-1], ids[2:, 1:]))
    loss.backward()
    ref_g = flat.grad.float().cpu().clone()
    opt.step()
    ref_p = flat.param.float().cpu().clone()
    del m, flat, opt
    torch.cuda.synchronize()

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q, accum, seq)) for r in range(2)]
    for p in ps:
        p.start()
    out = [q.get(timeout=100) for _ in ps]
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, g, p in out:
        g, p = torch.from_numpy(g), torch.from_numpy(p)
        rel = ((g - ref_g).norm() / ref_g.norm()).item()
        assert rel < 2e-2, (rank, rel)
        # bf16 params after one AdamW step (lr 1e-3): equal up to the bf16 rounding of the update
        assert (p - ref_p).abs().max().item() < 2e-2, rank
