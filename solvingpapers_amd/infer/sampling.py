"""Token sampling: greedy / categorical / top-k / top-p, with temperature.

Covers every sampler of the reference: greedy argmax (gpt/gpt-jax.ipynb:827), categorical
at T = 1 (llama3/LLaMA-jax.ipynb:508), softmax + multinomial (gemma/gemma.ipynb:620-622)
and top-k + temperature (deepseekv3/deepseekv3.ipynb:1861-1866); nucleus (top-p) is an
addition. Everything stays on the device: no ``.item()`` per token.
"""
from __future__ import annotations

from typing import Optional

import torch


def sample(logits: torch.Tensor, temperature: float = 1.0, top_k: Optional[int] = None,
           greedy: bool = False, generator: Optional[torch.Generator] = None,
           top_p: Optional[float] = None) -> torch.Tensor:
    """logits [B, V] -> next ids [B, 1]."""
    if greedy:
        return logits.argmax(-1, keepdim=True)
    logits = logits.float() / max(temperature, 1e-6)
    if top_k is not None:
        v, ix = torch.topk(logits, min(int(top_k), logits.shape[-1]), dim=-1)
        if top_p is not None:
            v = _nucleus(v, top_p)
        p = torch.softmax(v, dim=-1)
        j = torch.multinomial(p, 1, generator=generator)
        return ix.gather(-1, j)
    if top_p is not None:
        v, ix = torch.sort(logits, dim=-1, descending=True)
        p = torch.softmax(_nucleus(v, top_p), dim=-1)
        return ix.gather(-1, torch.multinomial(p, 1, generator=generator))
    p = torch.softmax(logits, dim=-1)
    return torch.multinomial(p, 1, generator=generator)


def _nucleus(sorted_logits: torch.Tensor, top_p: float) -> torch.Tensor:
    """Mask (to -inf) the tail of descending-sorted logits beyond cumulative mass top_p;
    the first token is always kept."""
    p = torch.softmax(sorted_logits, dim=-1)
    cum = p.cumsum(-1)
    drop = (cum - p) > top_p
    return sorted_logits.masked_fill(drop, float("-inf"))
