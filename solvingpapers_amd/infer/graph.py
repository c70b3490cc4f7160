"""HIP-graph decode: one captured launch per generated token.

A KV-cached decode step of LLaMA3-8B is ~450 short kernels (32 layers x norms, four
projections, RoPE, cache writes, decode attention, GLU) whose launch cost exceeds their
run time at batch 1. ``GraphDecoder`` captures one step with every position-dependent
value on the device:

* ``DecodeState.index``     -- the cache row written this step (long [1]);
* ``DecodeState.positions`` -- RoPE positions (int32 [B, 1]);
* ``DecodeState.kv_len``    -- valid cache rows (int32 [1]) read by the decode kernel.

The captured step ends by advancing that state on the device, and greedy sampling
(argmax into the static token buffer) is captured too, so ``n`` tokens are ``n`` graph
replays with no host work in between. Non-greedy sampling runs eagerly on the replay's
logits between replays (torch.multinomial).

Protocol a model implements: ``new_cache(B, max_len)``, ``step(ids, cache, pos)`` (eager
prefill) and ``step_graph(ids, cache, state)`` (graph-safe decode step: no host syncs).
"""
from __future__ import annotations

from typing import Optional

import torch

from .sampling import sample


class DecodeState:
    """Device-resident position state of a captured decode step (batch-uniform positions)."""

    def __init__(self, batch: int, max_len: int, device):
        self.batch, self.max_len = batch, max_len
        self.index = torch.zeros(1, dtype=torch.long, device=device)
        self.positions = torch.zeros(batch, 1, dtype=torch.int32, device=device)
        self.kv_len = torch.ones(1, dtype=torch.int32, device=device)

    def set(self, pos: int):
        """Host-side (re)position, outside the graph: the next step writes cache row ``pos``."""
        self.index.fill_(pos)
        self.positions.fill_(pos)
        self.kv_len.fill_(pos + 1)

    def advance(self):
        """Device-side increment (captured at the end of the step)."""
        self.index.add_(1)
        self.positions.add_(1)
        self.kv_len.add_(1)


class GraphDecoder:
    def __init__(self, model, batch: int, max_len: int, greedy: bool = True, warmup: int = 2):
        self.model, self.batch, self.max_len, self.greedy = model, batch, max_len, greedy
        dev = next(model.parameters()).device
        self.cache = model.new_cache(batch, max_len)
        self.state = DecodeState(batch, max_len, dev)
        self.ids = torch.zeros(batch, 1, dtype=torch.long, device=dev)
        self.logits: Optional[torch.Tensor] = None
        self._capture(warmup)

    def _body(self):
        lg = self.model.step_graph(self.ids, self.cache, self.state)
        if self.greedy:
            self.ids.copy_(lg.argmax(-1, keepdim=True))
        self.state.advance()
        return lg

    @torch.no_grad()
    def _capture(self, warmup):
        # warm-up outside the capture (lazy allocations, library handles, RoPE tables); it
        # scribbles on the first cache rows and advances the state, both reset by prefill()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(warmup):
                self._body()
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        self.state.set(0)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self.logits = self._body()
        self.state.set(0)

    @torch.no_grad()
    def prefill(self, ids: torch.Tensor) -> torch.Tensor:
        """Eager prompt pass: fills cache rows [0, T0), positions the state at T0 and returns
        the last position's logits."""
        T0 = ids.shape[1]
        if T0 >= self.max_len:
            raise ValueError(f"prompt of {T0} tokens leaves no room in a {self.max_len}-token cache")
        lg = self.model.step(ids, self.cache, 0)
        self.state.set(T0)
        return lg

    @torch.no_grad()
    def generate(self, ids: torch.Tensor, max_new_tokens: int, temperature: float = 1.0, top_k=None,
                 top_p=None, generator=None, stats=None) -> torch.Tensor:
        import time
        if stats is not None:
            torch.cuda.synchronize()
        t0 = time.perf_counter()
        lg = self.prefill(ids)
        if stats is not None:
            torch.cuda.synchronize()
        t1 = time.perf_counter()
        n = min(max_new_tokens, self.max_len - ids.shape[1] + 1)
        out = torch.empty(self.batch, n, dtype=torch.long, device=ids.device)
        if self.greedy:
            self.ids.copy_(lg.argmax(-1, keepdim=True))
        else:
            self.ids.copy_(sample(lg, temperature, top_k, False, generator, top_p))
        for i in range(n):
            out[:, i:i + 1].copy_(self.ids)
            if i + 1 == n:
                break
            self.graph.replay()  # feeds the token at row T0 + i; greedy leaves the next one in self.ids
            if not self.greedy:
                self.ids.copy_(sample(self.logits, temperature, top_k, False, generator, top_p))
        if stats is not None:
            torch.cuda.synchronize()
            stats.cached = True
            stats.prompt_tokens += ids.numel()
            stats.new_tokens += self.batch * n
            stats.prefill_s += t1 - t0
            stats.decode_s += time.perf_counter() - t1
        return torch.cat([ids, out], 1)
