"""LLaMA3 (GQA + RoPE + RMSNorm + SwiGLU), MI355X-native.

Reference: llama3/LLaMA-jax.ipynb (pure functional JAX). Component map:
  L6 rms_norm :536-538 -> ops.rms_norm (HIP, fused residual add)
  L7/L8 RoPE :563-601 -> ops.rope_packed_ (HIP, in place on the packed qkv buffer)
  L9 repeat_kv :626-627 -> not materialised (GQA head mapping inside the flash kernel)
  L11 GQA attention :809-829 -> ops.attention_packed (HIP flash fwd/bwd)
  L12 SwiGLU :854-855 -> one fused [gate|up] GEMM + ops.glu (HIP)
  L14 model_forward :916-931, L15 loss :956-968 -> ops.cross_entropy (HIP, in-place grad)
  L10 init :652-783 (N(0,1)/sqrt(fan_in), norm weights N(0,1) in the ref preset)
  L5 generate :499-511 -> generate() here, with a KV cache (the ref re-forwards the
     whole prefix per token; its cache path :816-819 was never exercised).
The reference's parameter pytree layout (§2.6 of SURVEY.md) is produced by
``to_reference_params`` / consumed by ``from_reference_params``.

Presets: ``llama3_ref`` (the notebook's 2-layer d256 config) and ``llama3_8b``
(the BASELINE.json north-star shape: D4096 L32 H32 KV8 FFN14336 V128256 theta 5e5).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field, replace
from typing import List, Optional

import torch
import torch.nn as nn

from ..infer.cache import KVCache
from ..infer.graph import DecodeState
from ..infer.sampling import sample  # noqa: F401  (re-exported: reference-style sampling)
from ..ops import _ext, attention_packed, embedding, linear, linear_cross_entropy, rms_norm, rope_packed_
from ..ops.linear import swiglu_mlp
from ..ops.attention import decode_attention
from ..ops.rope import RopeCache, apply_rope
from ..utils.grad import mark_ready


@dataclass
class LlamaConfig:
    vocab_size: int = 50257
    dim: int = 256
    n_layers: int = 2
    n_heads: int = 4
    n_kv_heads: int = 2
    ffn_hidden: int = 1024
    max_seq_len: int = 128
    norm_eps: float = 1e-6
    rope_theta: float = 10000.0
    gate: str = "w3"            # reference quirk (Q10): SwiGLU gate on w3; Meta uses w1
    ref_freqs: bool = True      # reference quirk: RoPE freq theta^(-i/hd) (LLaMA-jax.ipynb:563-567)
    init: str = "ref"           # "ref": N(0,1)/sqrt(fan_in) & N(0,1) norms; "std": N(0,0.02) & ones
    tie_embeddings: bool = False
    batch_size: int = 16
    lr: float = 3e-4

    @property
    def head_dim(self):
        return self.dim // self.n_heads


PRESETS = {
    # llama3/LLaMA-jax.ipynb:349-358 (+ ffn 4D :713-718)
    "llama3_ref": LlamaConfig(),
    # BASELINE.json north-star shape (public LLaMA3-8B card)
    "llama3_8b": LlamaConfig(vocab_size=128256, dim=4096, n_layers=32, n_heads=32, n_kv_heads=8, ffn_hidden=14336,
                             max_seq_len=8192, norm_eps=1e-5, rope_theta=500000.0, gate="w1", init="std",
                             ref_freqs=False, batch_size=1, lr=3e-4),
    # small GPU smoke shape with the 8B's head geometry
    "llama3_tiny": LlamaConfig(vocab_size=1024, dim=512, n_layers=2, n_heads=4, n_kv_heads=2, ffn_hidden=1536,
                               max_seq_len=256, norm_eps=1e-5, rope_theta=500000.0, gate="w1", init="std",
                               ref_freqs=False, batch_size=2),
}


def config(name: str, **kw) -> LlamaConfig:
    return replace(PRESETS[name], **kw)


class LlamaBlock(nn.Module):
    def __init__(self, c: LlamaConfig, **fk):
        super().__init__()
        hd = c.head_dim
        self.c = c
        self.cp_group = None  # context parallelism: this rank holds a T/P slice of the sequence
        self.attention_norm = nn.Parameter(torch.ones(c.dim, **fk))
        self.wqkv = nn.Parameter(torch.empty((c.n_heads + 2 * c.n_kv_heads) * hd, c.dim, **fk))
        self.wo = nn.Parameter(torch.empty(c.dim, c.n_heads * hd, **fk))
        self.ffn_norm = nn.Parameter(torch.ones(c.dim, **fk))
        self.w13 = nn.Parameter(torch.empty(2 * c.ffn_hidden, c.dim, **fk))  # [gate ; up]
        self.w2 = nn.Parameter(torch.empty(c.dim, c.ffn_hidden, **fk))

    @torch.no_grad()
    def reset_parameters(self, gen=None):
        c = self.c
        if c.init == "ref":
            for w in (self.wqkv, self.wo, self.w13, self.w2):
                nn.init.normal_(w, 0.0, 1.0, generator=gen).div_(math.sqrt(w.shape[1]))
            nn.init.normal_(self.attention_norm, 0.0, 1.0, generator=gen)
            nn.init.normal_(self.ffn_norm, 0.0, 1.0, generator=gen)
        else:
            for w in (self.wqkv, self.wo, self.w13, self.w2):
                nn.init.normal_(w, 0.0, 0.02, generator=gen)
            nn.init.ones_(self.attention_norm)
            nn.init.ones_(self.ffn_norm)

    def attn(self, n1, kv_cache=None, pos=0):
        c = self.c
        B, T, _ = n1.shape
        hd = c.head_dim
        qkv = linear(n1, self.wqkv)  # [B, T, (H+2Hkv)*hd]
        if isinstance(pos, DecodeState):  # graph-capturable decode step: positions on the device
            H, KV = c.n_heads, c.n_kv_heads
            x4 = qkv.view(B, T, H + 2 * KV, hd)
            cos, sin = RopeCache.get(pos.max_len, hd, c.rope_theta, qkv.device, c.ref_freqs)
            kc, vc = kv_cache
            # one launch: RoPE on q (in place) and k, k/v rows into the cache at pos.index
            _ext.ops().rope_kv_write_(x4, cos, sin, pos.positions, pos.index, kc, vc, H, KV, 0)
            o = decode_attention(x4[:, :, :H], kc, vc, causal=True, kv_len=pos.kv_len)
            return linear(o.reshape(B, T, H * hd), self.wo)
        if kv_cache is None and self.cp_group is not None:
            # sequence slice at offset rank*T: RoPE at global positions, attention over all
            # ranks' tokens via the all-to-all sequence <-> head exchange
            import torch.distributed as dist
            from ..parallel.context_parallel import context_parallel_attention
            H, KV = c.n_heads, c.n_kv_heads
            off = dist.get_rank(self.cp_group) * T
            qkv = rope_packed_(qkv, H + KV, c.rope_theta, off, head_dim=hd, ref_freqs=c.ref_freqs)
            x4 = qkv.view(B, T, H + 2 * KV, hd)
            o = context_parallel_attention(x4[:, :, :H], x4[:, :, H:H + KV], x4[:, :, H + KV:], self.cp_group)
        elif kv_cache is None:
            qkv = rope_packed_(qkv, c.n_heads + c.n_kv_heads, c.rope_theta, 0, head_dim=hd, ref_freqs=c.ref_freqs)
            o = attention_packed(qkv, c.n_heads, c.n_kv_heads, causal=True, head_dim=hd)
        else:
            qkv = qkv.view(B, T, c.n_heads + 2 * c.n_kv_heads, hd)
            q = apply_rope(qkv[:, :, :c.n_heads], c.rope_theta, pos, ref_freqs=c.ref_freqs)
            k = apply_rope(qkv[:, :, c.n_heads:c.n_heads + c.n_kv_heads], c.rope_theta, pos, ref_freqs=c.ref_freqs)
            v = qkv[:, :, c.n_heads + c.n_kv_heads:]
            kc, vc = kv_cache
            kc[:, pos:pos + T] = k
            vc[:, pos:pos + T] = v
            # decode steps: split-K decode kernel; prompt prefill: flash (decode_attention routes)
            o = decode_attention(q, kc[:, :pos + T], vc[:, :pos + T], causal=True)
        return linear(o.reshape(B, T, c.n_heads * hd), self.wo)

    def forward(self, res, delta, kv_cache=None, pos=0):
        """Pre-norm block on a split residual stream: h = res + delta (fused in the norm)."""
        c = self.c
        if res is None:
            n1 = rms_norm(delta, self.attention_norm, c.norm_eps)
            h = delta
        else:
            n1, h = rms_norm(delta, self.attention_norm, c.norm_eps, residual=res)
        a = self.attn(n1, kv_cache, pos)
        n2, h2 = rms_norm(a, self.ffn_norm, c.norm_eps, residual=h)
        return h2, swiglu_mlp(n2, self.w13, self.w2, "silu")


class Llama3(nn.Module):
    def __init__(self, c: LlamaConfig, device=None, dtype=torch.float32, seed: int = 0):
        super().__init__()
        self.c = c
        fk = dict(device=device, dtype=dtype)  # build in place on the target device (8B: no host copy)
        self.tok_embeddings = nn.Parameter(torch.empty(c.vocab_size, c.dim, **fk))
        self.layers = nn.ModuleList([LlamaBlock(c, **fk) for _ in range(c.n_layers)])
        self.norm_f = nn.Parameter(torch.ones(c.dim, **fk))
        self.output = None if c.tie_embeddings else nn.Parameter(torch.empty(c.vocab_size, c.dim, **fk))
        self.grad_ready_cb = None   # DP: launch gradient bucket i when its layer's backward is done
        self.param_wait_cb = None   # optimizer overlap: wait for bucket i's update before using it
        self.reset_parameters(seed)

    @torch.no_grad()
    def reset_parameters(self, seed=0):
        dev = self.tok_embeddings.device
        g = torch.Generator(device=dev).manual_seed(seed)
        c = self.c
        if c.init == "ref":
            nn.init.normal_(self.tok_embeddings, 0.0, 1.0, generator=g).div_(math.sqrt(c.vocab_size))
            nn.init.normal_(self.norm_f, 0.0, 1.0, generator=g)
            if self.output is not None:
                nn.init.normal_(self.output, 0.0, 1.0, generator=g).div_(math.sqrt(c.dim))
        else:
            nn.init.normal_(self.tok_embeddings, 0.0, 0.02, generator=g)
            nn.init.ones_(self.norm_f)
            if self.output is not None:
                nn.init.normal_(self.output, 0.0, 0.02, generator=g)
        for blk in self.layers:
            blk.reset_parameters(g)

    # bucket order for FlatParams / DP: embedding, layer0..N-1, head
    def param_groups(self) -> List[List[nn.Parameter]]:
        head = [self.norm_f] + ([self.output] if self.output is not None else [])
        return [[self.tok_embeddings]] + [list(l.parameters()) for l in self.layers] + [head]

    def hidden(self, ids, kv_caches=None, pos=0):
        c = self.c
        wait = self.param_wait_cb or (lambda i: None)
        wait(0)
        x = embedding(self.tok_embeddings, ids)
        res, delta = None, x
        cb = self.grad_ready_cb
        for i, layer in enumerate(self.layers):
            wait(i + 1)
            delta = mark_ready(delta, cb, i + 1)
            res, delta = layer(res, delta, None if kv_caches is None else kv_caches[i], pos)
        wait(len(self.layers) + 1)
        delta = mark_ready(delta, cb, len(self.layers) + 1)
        n, _ = rms_norm(delta, self.norm_f, c.norm_eps, residual=res)
        return n

    def set_context_parallel(self, group):
        """Train on sequence slices: rank r of ``group`` feeds tokens [r*T, (r+1)*T) of each
        sequence. Gradients are then summed over ``group`` like data parallelism (e.g.
        ``DataParallel(model, flat, group=group)``): the mean of the ranks' local losses is the
        full-sequence loss."""
        for l in self.layers:
            l.cp_group = group
        return self

    def logits(self, n):
        w = self.output if self.output is not None else self.tok_embeddings
        return linear(n, w)

    def forward(self, ids, targets=None):
        n = self.hidden(ids)
        if targets is None:
            return self.logits(n)
        w = self.output if self.output is not None else self.tok_embeddings
        return linear_cross_entropy(n.reshape(-1, n.shape[-1]), w, targets.reshape(-1))

    def loss(self, ids, targets):
        return self.forward(ids, targets)

    def num_params(self):
        return sum(p.numel() for p in self.parameters())

    def flops_per_token(self, T):
        """Training FLOPs/token: 6*N_matmul + causal attention 6*L*D*T (fwd+bwd, causal half)."""
        c = self.c
        hd = c.head_dim
        per_layer = c.dim * (c.n_heads + 2 * c.n_kv_heads) * hd + c.dim * c.n_heads * hd + 3 * c.dim * c.ffn_hidden
        n_mm = c.n_layers * per_layer + c.vocab_size * c.dim
        attn = 6 * c.n_layers * c.n_heads * hd * T  # 2 matmuls x 2 flop x T/2 (causal) x 3 (fwd+bwd)
        return 6 * n_mm + attn

    # ---------------------------------------------------------------- inference
    @property
    def max_context(self):
        return self.c.max_seq_len

    def new_cache(self, B, Tmax):
        c = self.c
        return KVCache(c.n_layers, B, Tmax, c.n_kv_heads, c.head_dim, device=self.tok_embeddings.device,
                       dtype=self.tok_embeddings.dtype)

    def step(self, ids, cache, pos):
        """Write ids' K/V at cache rows [pos, pos+T), return the last position's logits [B, V]."""
        n = self.hidden(ids, cache, pos)
        return self.logits(n[:, -1:]).float()[:, -1]

    def step_graph(self, ids, cache, state: DecodeState):
        """One-token decode step with every position on the device (HIP-graph capturable;
        infer/graph.py): one fused launch rotates q/k and writes the cache row at
        ``state.index``, RoPE reads device positions, the decode kernel reads the cache
        length from ``state.kv_len``."""
        n = self.hidden(ids, cache, state)
        return self.logits(n).float()[:, -1]

    @torch.no_grad()
    def generate(self, ids, max_new_tokens, temperature=1.0, top_k=None, greedy=False, generator=None,
                 top_p=None, eos_token_id=None, stats=None):
        """KV-cached sampling (reference: llama3/LLaMA-jax.ipynb:499-511, categorical at T=1,
        full re-forward per token; its cache path :816-819 was never exercised)."""
        from ..infer.generate import generate
        return generate(self, ids, max_new_tokens, temperature, top_k, top_p, greedy, eos_token_id, generator, stats)

    # ------------------------------------------------------- reference layout I/O
    def to_reference_params(self):
        """Nested dict in the notebook's layout (matrices (in, out))."""
        c = self.c
        H, KV, hd, F = c.n_heads, c.n_kv_heads, c.head_dim, c.ffn_hidden
        out = {"token_embedding": self.tok_embeddings.detach().float().clone(),
               "norm_f": self.norm_f.detach().float().clone(),
               "output": (self.output if self.output is not None else self.tok_embeddings).detach().float().t().clone(),
               "blocks": []}
        for l in self.layers:
            wqkv = l.wqkv.detach().float()
            wq, wk, wv = wqkv[:H * hd], wqkv[H * hd:(H + KV) * hd], wqkv[(H + KV) * hd:]
            gate, up = l.w13.detach().float()[:F], l.w13.detach().float()[F:]
            w1, w3 = (up, gate) if c.gate == "w3" else (gate, up)
            out["blocks"].append({
                "attention": {"wq": wq.t().clone(), "wk": wk.t().clone(), "wv": wv.t().clone(),
                              "wo": l.wo.detach().float().t().clone()},
                "ffn": {"w1": w1.t().clone(), "w2": l.w2.detach().float().t().clone(), "w3": w3.t().clone()},
                "attention_norm": l.attention_norm.detach().float().clone(),
                "ffn_norm": l.ffn_norm.detach().float().clone(),
            })
        return out

    @torch.no_grad()
    def from_reference_params(self, ref):
        c = self.c
        t = lambda x: torch.as_tensor(x, dtype=torch.float32)
        self.tok_embeddings.copy_(t(ref["token_embedding"]))
        self.norm_f.copy_(t(ref["norm_f"]))
        if self.output is not None:
            self.output.copy_(t(ref["output"]).t())
        for l, b in zip(self.layers, ref["blocks"]):
            a, f = b["attention"], b["ffn"]
            l.wqkv.copy_(torch.cat([t(a["wq"]).t(), t(a["wk"]).t(), t(a["wv"]).t()], 0))
            l.wo.copy_(t(a["wo"]).t())
            gate, up = (f["w3"], f["w1"]) if c.gate == "w3" else (f["w1"], f["w3"])
            l.w13.copy_(torch.cat([t(gate).t(), t(up).t()], 0))
            l.w2.copy_(t(f["w2"]).t())
            l.attention_norm.copy_(t(b["attention_norm"]))
            l.ffn_norm.copy_(t(b["ffn_norm"]))
        return self
