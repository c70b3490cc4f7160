"""Inference: KV-cached generation for the language models of the catalogue.

* :func:`sample` -- greedy / categorical / top-k / top-p with temperature;
* :class:`KVCache` -- preallocated per-layer K/V buffers, written in place;
* :func:`generate` -- prompt prefill (flash attention) + token-by-token decode (split-K
  decode kernel, csrc/kernels/decode.hip) with the model's own cache layout, timing
  prefill and decode separately.

Reference entry points (all recompute the whole prefix per token, no cache):
gpt/gpt-jax.ipynb:821-829, llama3/LLaMA-jax.ipynb:499-511, gemma/gemma.ipynb:608-630,
deepseekv3/deepseekv3.ipynb:1849-1873.
"""
from .cache import KVCache
from .generate import GenerationStats, generate
from .graph import DecodeState, GraphDecoder
from .sampling import sample

__all__ = ["KVCache", "DecodeState", "GenerationStats", "GraphDecoder", "generate", "sample"]
