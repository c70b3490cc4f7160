"""Preallocated per-layer KV cache for GQA / MQA decoding.

One [B, Tmax, Hkv, hd] buffer per layer for K and for V, allocated once for the whole
generation (HBM is 288 GB per MI355X: a LLaMA3-8B cache at 8K tokens is 1 GB per
sequence), written in place at the current position and read as strided views by the
decode kernel -- no concatenation per token (the reference's unused cache path,
llama3/LLaMA-jax.ipynb:816-819, concatenates).
"""
from __future__ import annotations

from typing import List, Tuple

import torch


class KVCache(list):
    """``list`` of (k, v) pairs so models can index ``cache[layer]`` directly."""

    def __init__(self, n_layers: int, batch: int, max_len: int, n_kv_heads: int, head_dim: int,
                 device=None, dtype=torch.bfloat16):
        super().__init__(
            (torch.zeros(batch, max_len, n_kv_heads, head_dim, device=device, dtype=dtype),
             torch.zeros(batch, max_len, n_kv_heads, head_dim, device=device, dtype=dtype))
            for _ in range(n_layers))
        self.max_len = max_len
        self.pos = 0

    def write(self, layer: int, k: torch.Tensor, v: torch.Tensor, pos: int) -> Tuple[torch.Tensor, torch.Tensor]:
        """Store k/v [B, T, Hkv, hd] at [pos, pos+T) and return the [0, pos+T) views."""
        kc, vc = self[layer]
        T = k.shape[1]
        if pos + T > self.max_len:
            raise ValueError(f"KV cache overflow: {pos + T} > {self.max_len}")
        kc[:, pos:pos + T] = k
        vc[:, pos:pos + T] = v
        return kc[:, :pos + T], vc[:, :pos + T]

    def nbytes(self) -> int:
        return sum(k.numel() * k.element_size() * 2 for k, _ in self)

    @staticmethod
    def layers(cache) -> List:
        return list(cache)
