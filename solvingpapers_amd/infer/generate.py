"""Generic autoregressive generation driver.

Protocol a model implements for cached decoding:
  ``new_cache(batch, max_len)``  -> cache object (KVCache or the model's latent cache)
  ``step(ids, cache, pos)``      -> logits [B, V] of the LAST position of ``ids``, after
                                    writing ``ids``' keys/values at cache rows [pos, pos+T)
  ``max_context`` (attribute, optional) -> the longest sequence the model accepts

The first call is the prompt prefill (flash attention over the whole prompt), every later
call feeds one token per sequence (split-K decode attention). Models without the protocol
(the reference-exact GPT / Gemma presets, whose notebooks crop to ``block_size`` and
re-run the window) are driven by re-forwarding the cropped window, as the reference does
(gpt/gpt-jax.ipynb:821-829, gemma/gemma.ipynb:608-630).
"""
from __future__ import annotations

import time
from dataclasses import dataclass
from typing import Optional

import torch

from .sampling import sample


@dataclass
class GenerationStats:
    prompt_tokens: int = 0
    new_tokens: int = 0
    prefill_s: float = 0.0
    decode_s: float = 0.0
    cached: bool = False

    @property
    def decode_tok_s(self) -> float:
        """Generated tokens per second over the decode phase (all sequences)."""
        return self.new_tokens / self.decode_s if self.decode_s > 0 else 0.0

    @property
    def prefill_tok_s(self) -> float:
        return self.prompt_tokens / self.prefill_s if self.prefill_s > 0 else 0.0


def _sync(t: torch.Tensor):
    if t.is_cuda:
        torch.cuda.synchronize(t.device)


@torch.no_grad()
def generate(model, ids: torch.Tensor, max_new_tokens: int, temperature: float = 1.0,
             top_k: Optional[int] = None, top_p: Optional[float] = None, greedy: bool = False,
             eos_token_id: Optional[int] = None, generator: Optional[torch.Generator] = None,
             stats: Optional[GenerationStats] = None, timed: bool = False) -> torch.Tensor:
    """ids [B, T0] -> [B, T0 + n] (n <= max_new_tokens; stops early once every sequence has
    produced ``eos_token_id``, checked every 16 tokens to keep the host out of the loop)."""
    was = model.training
    model.eval()
    timed = timed or stats is not None  # stats requested -> device-synchronised phase timings
    st = stats if stats is not None else GenerationStats()
    B, T0 = ids.shape
    limit = getattr(model, "max_context", None)
    out = ids
    done = torch.zeros(B, dtype=torch.bool, device=ids.device)
    try:
        if hasattr(model, "new_cache") and hasattr(model, "step"):
            st.cached = True
            total = T0 + max_new_tokens
            if limit is not None:
                total = min(total, limit)
            prompt = ids[:, -total:] if T0 > total else ids
            cache = model.new_cache(B, total)
            if timed:
                _sync(ids)
            t0 = time.perf_counter()
            logits = model.step(prompt, cache, 0)
            pos = prompt.shape[1]
            if timed:
                _sync(ids)
            t1 = time.perf_counter()
            st.prompt_tokens += B * prompt.shape[1]
            st.prefill_s += t1 - t0
            n = 0
            while n < max_new_tokens:
                nxt = sample(logits, temperature, top_k, greedy, generator, top_p)
                if eos_token_id is not None:
                    nxt = torch.where(done[:, None], torch.full_like(nxt, eos_token_id), nxt)
                    done |= nxt[:, 0] == eos_token_id
                out = torch.cat([out, nxt], 1)
                n += 1
                if pos >= total or n >= max_new_tokens:
                    break
                if eos_token_id is not None and n % 16 == 0 and bool(done.all()):
                    break
                logits = model.step(nxt, cache, pos)
                pos += 1
            if timed:
                _sync(ids)
            st.decode_s += time.perf_counter() - t1
            st.new_tokens += B * n
        else:
            block = limit or getattr(getattr(model, "c", None), "block_size", None)
            t1 = time.perf_counter()
            for n in range(max_new_tokens):
                window = out[:, -block:] if block else out
                lg = model(window)[:, -1].float()
                nxt = sample(lg, temperature, top_k, greedy, generator, top_p)
                out = torch.cat([out, nxt], 1)
            if timed:
                _sync(ids)
            st.decode_s += time.perf_counter() - t1
            st.new_tokens += B * max_new_tokens
    finally:
        model.train(was)
    return out
