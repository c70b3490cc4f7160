"""Text data: char-level tokenizer (gpt/gpt-jax.ipynb:247-252, gemma/gemma.ipynb:95-106),
random-window batching (gpt-jax.ipynb:491-497, gemma.ipynb:116-129, done on-device here),
and the sliding-window CausalDataset (deepseekv3/deepseekv3.ipynb:715-726) with rank sharding."""
from __future__ import annotations

import random
from typing import Iterator, Optional, Tuple

import torch


class CharTokenizer:
    """sorted(set(text)) vocabulary; encode/decode as in the reference notebooks."""

    def __init__(self, text: str):
        self.chars = sorted(set(text))
        self.stoi = {c: i for i, c in enumerate(self.chars)}
        self.itos = {i: c for i, c in enumerate(self.chars)}

    @property
    def vocab_size(self):
        return len(self.chars)

    def encode(self, s: str):
        return [self.stoi[c] for c in s]

    def decode(self, ids):
        return "".join(self.itos[int(i)] for i in ids)


_WORDS = ("the king and queen of rome spoke to the people who came to hear what was said about war and "
          "peace love death honour time night day crown sword lord lady good noble heart mind world fair "
          "thou art thee thy shall not be nor ever more").split()


def synthetic_corpus(n_chars: int = 200_000, seed: int = 0) -> str:
    """Deterministic pseudo-Shakespeare text (65-ish symbol alphabet is not required;
    the char tokenizer adapts). Stands in for tinyshakespeare (no network)."""
    rng = random.Random(seed)
    out, n = [], 0
    while n < n_chars:
        speaker = rng.choice(["ROMEO", "JULIET", "KING", "LORD", "QUEEN", "DUKE"])
        line = speaker + ":\n" + " ".join(rng.choice(_WORDS) for _ in range(rng.randint(5, 14))).capitalize() + ".\n\n"
        out.append(line)
        n += len(line)
    return "".join(out)[:n_chars]


def synthetic_tokens(n: int, vocab: int, seed: int = 0, device=None) -> torch.Tensor:
    """Random token stream (the perf benchmarks use synthetic ids of the right shape)."""
    g = torch.Generator().manual_seed(seed)
    return torch.randint(0, vocab, (n,), generator=g).to(device)


def get_batch(data: torch.Tensor, batch_size: int, block_size: int, generator=None) -> Tuple[torch.Tensor, torch.Tensor]:
    """Random windows x = data[i:i+T], y = data[i+1:i+T+1]; gathered on data's device
    with one index op (the reference stacks B Python slices)."""
    n = data.numel() - block_size
    ix = torch.randint(0, n, (batch_size,), generator=generator, device="cpu").to(data.device)
    off = torch.arange(block_size + 1, device=data.device)
    win = data[ix[:, None] + off[None, :]]
    return win[:, :-1].contiguous(), win[:, 1:].contiguous()


class TokenWindowDataset:
    """Every sliding window of a flat token stream (len = N - block), sharded by rank:
    rank r sees windows r, r+world, ... (DistributedSampler-style)."""

    def __init__(self, tokens: torch.Tensor, block_size: int, rank: int = 0, world: int = 1):
        self.tokens, self.block, self.rank, self.world = tokens, block_size, rank, world

    def __len__(self):
        return (self.tokens.numel() - self.block - self.rank + self.world - 1) // self.world

    def __getitem__(self, i):
        j = i * self.world + self.rank
        return self.tokens[j:j + self.block], self.tokens[j + 1:j + self.block + 1]

    def batches(self, batch_size: int, shuffle=True, seed=0, drop_last=True) -> Iterator:
        order = list(range(len(self)))
        if shuffle:
            random.Random(seed).shuffle(order)
        for k in range(0, len(order) - (batch_size - 1 if drop_last else 0), batch_size):
            idx = order[k:k + batch_size]
            xs, ys = zip(*(self[i] for i in idx))
            yield torch.stack(xs), torch.stack(ys)
