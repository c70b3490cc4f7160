"""Process-group bootstrap: one process per GPU, torch.distributed over RCCL.

On ROCm the ``"nccl"`` backend IS RCCL (xGMI point-to-point links between the
8 MI355X of a node). CPU tests use ``"gloo"`` with the same code paths.
Launch: ``python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ...``.
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass
from typing import Optional

import torch
import torch.distributed as dist


@dataclass
class DistInfo:
    rank: int = 0
    world_size: int = 1
    local_rank: int = 0
    backend: str = "none"
    device: torch.device = torch.device("cpu")

    @property
    def is_main(self):
        return self.rank == 0


_INFO = DistInfo()


def force_collectives() -> bool:
    """``SPA_FORCE_COLLECTIVES=1`` (tests): create the process group and run every collective path
    (DP buckets, ZeRO-1, EP exchanges, the routing-bias all-reduce) even at world size 1, so one GPU
    drives them through RCCL before a multi-GPU run does (tests/test_rccl_gpu.py)."""
    return os.environ.get("SPA_FORCE_COLLECTIVES", "0") == "1"


def init_distributed(backend: Optional[str] = None, timeout_s: int = 1800) -> DistInfo:
    """Initialise from torchrun env vars (RANK/WORLD_SIZE/LOCAL_RANK/MASTER_*). With more than
    one RCCL rank it also selects hipBLASLt's data-parallel stream-K grid (SPA_STREAMK_DP=0
    keeps the default persistent grid), see below."""
    global _INFO
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    cuda = torch.cuda.is_available()
    if backend is None:
        # SPA_DIST_BACKEND=gloo: rehearse the multi-rank paths on a box with fewer GPUs than ranks
        backend = os.environ.get("SPA_DIST_BACKEND") or ("nccl" if cuda else "gloo")
    if world > 1 and backend == "nccl" and os.environ.get("SPA_STREAMK_DP", "1") != "0":
        # Gradient buckets all-reduce on RCCL's stream while the backward runs. hipBLASLt's
        # stream-K GEMMs size a persistent grid to the whole chip, so a co-running RCCL kernel
        # stalls their workgroups: a 1-GPU stand-in (tools/overlap_interference.py) slowed the
        # LLaMA-8B-shape backward 1.39x; with Tensile's data-parallel stream-K grid 1.18x, and
        # backward+collective overlapped 65.5 -> 57.1 ms (profiles/r2_overlap_streamk_env.jsonl)
        # for +0.9 % GEMM time standalone. Set before the first GEMM loads hipBLASLt.
        os.environ.setdefault("TENSILE_STREAMK_DATA_PARALLEL", "1")
    if cuda:
        ndev = torch.cuda.device_count()
        dev_idx = local if (backend == "nccl" or local < ndev) else local % ndev
        torch.cuda.set_device(dev_idx)
        device = torch.device("cuda", dev_idx)
    else:
        device = torch.device("cpu")
    if (world > 1 or force_collectives()) and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
        kw = dict(backend=backend, rank=rank, world_size=world, timeout=datetime.timedelta(seconds=timeout_s))
        if backend == "nccl" and cuda:
            kw["device_id"] = device
        restart = os.environ.get("TORCHELASTIC_RESTART_COUNT")
        if restart is not None and int(restart) > 0:
            # after an elastic restart the workers share the agent's store with the dead round:
            # namespace this round's keys, or a new rank can read a dead peer's address
            # (gloo: 'connectFullMesh ... Connection refused') and the restart fails
            store, _, _ = next(dist.rendezvous("env://", rank, world, timeout=kw["timeout"]))
            kw["store"] = dist.PrefixStore(f"spa_restart{restart}", store)
        dist.init_process_group(**kw)
    _INFO = DistInfo(rank, world, local, backend if dist.is_initialized() else "none", device)
    return _INFO


def info() -> DistInfo:
    return _INFO


def is_dist() -> bool:
    return dist.is_available() and dist.is_initialized() and (dist.get_world_size() > 1 or force_collectives())


def barrier(group=None):
    if is_dist():
        if _INFO.backend == "nccl":
            dist.barrier(group=group, device_ids=[torch.cuda.current_device()])
        else:
            dist.barrier(group=group)


def all_reduce_max(x: float) -> float:
    if not is_dist():
        return x
    t = torch.tensor([x], dtype=torch.float64, device=_INFO.device if _INFO.backend == "nccl" else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def all_reduce_mean(t: torch.Tensor, group=None) -> torch.Tensor:
    if not is_dist():
        return t
    t = t.clone()
    dist.all_reduce(t, group=group)
    return t / dist.get_world_size(group)


def cleanup():
    if dist.is_available() and dist.is_initialized():
        dist.destroy_process_group()
