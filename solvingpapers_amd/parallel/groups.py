"""Process-group layout for combined data / tensor / expert parallelism on one node.

The reference's only multi-GPU path is single-process ``nn.DataParallel`` over 2 GPUs
(deepseekv3/deepseekv3.ipynb:1709-1711, 2345-2346). Here every rank is one GPU and the
world is factored as

    world = tp x data,          data = ep x expert_dp

* ``tp``  (tensor parallel): contiguous blocks of ``tp`` ranks -- on an 8-GPU node those
  are the GPUs whose activations all-reduce 4x per layer, so keep them adjacent;
* ``dp``  (data parallel for DENSE parameters): the ranks with the same TP coordinate --
  every EP rank is also a DP rank (it feeds its own tokens);
* ``ep``  (expert parallel): ``ep`` consecutive data ranks split the routed experts and
  exchange tokens with two all-to-alls per MoE layer (xGMI is a full point-to-point mesh,
  so an all-to-all drives all 7 links at once);
* ``expert_dp``: ranks holding the SAME experts (same EP coordinate in different EP
  groups); expert gradients are summed only over this group.

Every rank must call ``build_groups`` with the same arguments (``dist.new_group`` is
collective over the world); each group handle is None when its size is 1.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional

import torch.distributed as dist


@dataclass
class ProcessGroups:
    world: int
    rank: int
    tp: int
    ep: int
    dp: int                     # dense data-parallel degree = world // tp
    tp_rank: int
    dp_rank: int                # this rank's index in the data dimension (data loader shard)
    ep_rank: int
    tp_group: Optional[object] = None
    dp_group: Optional[object] = None
    ep_group: Optional[object] = None
    expert_dp_group: Optional[object] = None
    tp_ranks: Optional[List[int]] = None
    dp_ranks: Optional[List[int]] = None
    ep_ranks: Optional[List[int]] = None
    expert_dp_ranks: Optional[List[int]] = None

    @property
    def expert_dp(self) -> int:
        return self.dp // self.ep

    def layout(self) -> dict:
        """Plain-value description stored in checkpoints (resume must match it)."""
        return {"world": self.world, "tp": self.tp, "ep": self.ep, "dp": self.dp}


def layout_ranks(world: int, tp: int = 1, ep: int = 1):
    """Pure rank arithmetic (no process group): lists of rank lists per group kind."""
    if world % tp:
        raise ValueError(f"tp={tp} must divide world={world}")
    data = world // tp
    if data % ep:
        raise ValueError(f"ep={ep} must divide the data dimension world/tp={data}")
    rank_of = lambda t, d: d * tp + t  # noqa: E731  (tp innermost: TP peers adjacent)
    tp_groups = [[rank_of(t, d) for t in range(tp)] for d in range(data)]
    dp_groups = [[rank_of(t, d) for d in range(data)] for t in range(tp)]
    ep_groups = [[rank_of(t, g * ep + k) for k in range(ep)] for t in range(tp) for g in range(data // ep)]
    edp_groups = [[rank_of(t, g * ep + k) for g in range(data // ep)] for t in range(tp) for k in range(ep)]
    return {"tp": tp_groups, "dp": dp_groups, "ep": ep_groups, "expert_dp": edp_groups}


def _hp_options(kind):
    """RCCL options for the TP / EP communicators: their collectives sit between compute on the
    critical path (or between the two chunks of an overlapped pair), so their internal stream is high
    priority (parallel/comm.py COMM_PRIORITY); DP buckets keep the default."""
    from .comm import COMM_PRIORITY
    if kind in ("dp", "expert_dp") or COMM_PRIORITY >= 0 or dist.get_backend() != "nccl":
        return None
    try:
        o = dist.ProcessGroupNCCL.Options()
        o.is_high_priority_stream = True
        return o
    except (AttributeError, RuntimeError):
        return None


def build_groups(tp: int = 1, ep: int = 1) -> ProcessGroups:
    initialized = dist.is_available() and dist.is_initialized()
    world = dist.get_world_size() if initialized else 1
    rank = dist.get_rank() if initialized else 0
    lay = layout_ranks(world, tp, ep)
    mine = {}
    for kind in ("tp", "dp", "ep", "expert_dp"):
        for ranks in lay[kind]:
            # new_group is collective over the WORLD: create every group on every rank, in order
            g = dist.new_group(ranks, pg_options=_hp_options(kind)) if (initialized and len(ranks) > 1) else None
            if rank in ranks:
                mine[kind] = (g, ranks)
    tp_ranks, dp_ranks, ep_ranks = mine["tp"][1], mine["dp"][1], mine["ep"][1]
    return ProcessGroups(
        world=world, rank=rank, tp=tp, ep=ep, dp=world // tp,
        tp_rank=tp_ranks.index(rank), dp_rank=dp_ranks.index(rank), ep_rank=ep_ranks.index(rank),
        tp_group=mine["tp"][0], dp_group=mine["dp"][0], ep_group=mine["ep"][0],
        expert_dp_group=mine["expert_dp"][0],
        tp_ranks=tp_ranks, dp_ranks=dp_ranks, ep_ranks=ep_ranks, expert_dp_ranks=mine["expert_dp"][1])
