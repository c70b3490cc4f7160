"""Context parallelism for long sequences: all-to-all (Ulysses-style) sequence <-> head exchange.

The reference has no long-context support (max context 256, materialised (B,H,T,T) scores;
SURVEY.md §5 "Long context"). Here each of P ranks holds a contiguous T/P slice of the
sequence. Attention needs every key, so q/k/v are re-sharded from [B, T/P, H, hd] to
[B, T, H/P, hd] by one all-to-all each, the flash kernel runs on full-length sequences for
H/P heads (causal masking is exact: every rank sees all of T), and one all-to-all returns the
output to the sequence layout. Everything outside attention (norms, projections, FFN) runs on
T/P tokens per rank, so activation memory per GPU falls by P.

Per layer the traffic is 4 all-to-alls of B·T·H·hd/P elements per rank (q, k, v, o; the same
again in backward): on xGMI every pair of GPUs has a direct link, so an all-to-all uses all 7
links at once instead of a ring's 2. K/V heads are exchanged before any replication when
Hkv % P == 0 (GQA keeps its bandwidth saving); MQA / small Hkv replicate K/V to P heads first.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from ..ops.attention import flash_attention


def _a2a(x: torch.Tensor, group) -> torch.Tensor:
    out = torch.empty_like(x)
    dist.all_to_all_single(out, x.contiguous(), group=group)
    return out


def _seq_to_head(x, P, group):
    """[B, Tl, H, d] (sequence shard) -> [B, Tl*P, H/P, d] (head shard)."""
    B, Tl, H, d = x.shape
    # chunk j of dim 0 goes to rank j: put the head groups first
    send = x.reshape(B, Tl, P, H // P, d).permute(2, 0, 1, 3, 4).contiguous()
    recv = _a2a(send, group)                                 # [P(src = seq chunk), B, Tl, H/P, d]
    return recv.permute(1, 0, 2, 3, 4).reshape(B, P * Tl, H // P, d)


def _head_to_seq(x, P, group):
    """[B, T, Hl, d] (head shard) -> [B, T/P, Hl*P, d] (sequence shard)."""
    B, T, Hl, d = x.shape
    send = x.reshape(B, P, T // P, Hl, d).permute(1, 0, 2, 3, 4).contiguous()
    recv = _a2a(send, group)                                 # [P(src = head group), B, T/P, Hl, d]
    return recv.permute(1, 2, 0, 3, 4).reshape(B, T // P, P * Hl, d)


class _SeqToHead(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, P, group):
        ctx.P, ctx.group = P, group
        return _seq_to_head(x, P, group)

    @staticmethod
    def backward(ctx, g):
        return _head_to_seq(g, ctx.P, ctx.group), None, None


class _HeadToSeq(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, P, group):
        ctx.P, ctx.group = P, group
        return _head_to_seq(x, P, group)

    @staticmethod
    def backward(ctx, g):
        return _seq_to_head(g, ctx.P, ctx.group), None, None


def context_parallel_attention(q, k, v, group=None, causal=True, scale=None):
    """q [B, T/P, H, hd], k/v [B, T/P, Hkv, hd] -> o [B, T/P, H, hd]: attention over the full
    sequence of P ranks, each holding the T/P slice at offset rank*T/P."""
    P = dist.get_world_size(group) if dist.is_initialized() else 1
    if P == 1:
        return flash_attention(q, k, v, causal, scale)
    H, Hkv = q.shape[2], k.shape[2]
    assert H % P == 0, f"context parallel needs heads ({H}) divisible by ranks ({P})"
    if Hkv % P:
        # MQA / too few kv heads to split: expand kv to one head per query head, so the head
        # shards of q and kv line up one to one
        rep = H // Hkv
        k = k.repeat_interleave(rep, dim=2)
        v = v.repeat_interleave(rep, dim=2)
    qh = _SeqToHead.apply(q, P, group)
    kh = _SeqToHead.apply(k, P, group)
    vh = _SeqToHead.apply(v, P, group)
    o = flash_attention(qh, kh, vh, causal, scale)
    return _HeadToSeq.apply(o, P, group)
