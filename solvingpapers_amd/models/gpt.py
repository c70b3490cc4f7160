"""GPT (decoder-only char-LM) — MI355X-native re-implementation of gpt/gpt-jax.ipynb.

Reference components: CausalSelfAttention :321-357 (fused QKV Dense(3D, no bias),
-1e4 causal mask, softmax, attention-weight dropout, proj Dense with bias),
MLP :376-389 (Dense 4D -> GELU tanh-approx (flax default) -> dropout -> Dense D),
DecoderBlock :408-422 (pre-LN, flax LayerNorm eps 1e-6), GPT :441-472 (token Embed +
learned pos_embed N(0,0.02), emb dropout, 8 blocks, ln_f, untied lm_head), training
:528-552,791-802 (AdamW 3e-4 wd 0.01, eval every 100 steps), greedy generate :821-829.

Here: packed QKV GEMM -> causal flash attention (HIP; materialised path only when
training with attention dropout p>0), fused LayerNorm + residual kernels, GELU-tanh
kernel, fused token+position embedding gather, fused LM-head cross-entropy.
Parameter names follow the Flax pytree (``to_reference_params``), kernels (in, out).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, replace
from typing import Dict, Optional

import torch
import torch.nn as tnn

from .. import nn as snn
from ..ops import act, attention_packed, embedding, layer_norm, linear, linear_cross_entropy
from ..ops.attention import attention_dropout, decode_attention
from ..ops.misc import dropout
from ..utils.grad import mark_ready


@dataclass
class GPTConfig:
    vocab_size: int = 65
    block_size: int = 256
    emb_dim: int = 256
    num_heads: int = 1
    num_layers: int = 8
    dropout_rate: float = 0.1
    ln_eps: float = 1e-6
    lr: float = 3e-4
    weight_decay: float = 0.01
    batch_size: int = 128
    total_steps: int = 1000
    eval_iters: int = 100


PRESETS = {
    "gpt_ref": GPTConfig(),                                        # gpt-jax.ipynb:293-302
    "gpt_tiny_cpu": GPTConfig(num_layers=2, block_size=64, batch_size=16, emb_dim=128, num_heads=2),  # BASELINE config #1
}


def config(name, **kw):
    return replace(PRESETS[name], **kw)


class Block(tnn.Module):
    def __init__(self, c: GPTConfig, **fk):
        super().__init__()
        D = c.emb_dim
        self.c = c
        self.ln1 = snn.LayerNorm(D, c.ln_eps, **fk)
        self.qkv = tnn.Parameter(torch.empty(3 * D, D, **fk))          # Dense(3D, use_bias=False)
        self.proj = snn.Linear(D, D, **fk)
        self.ln2 = snn.LayerNorm(D, c.ln_eps, **fk)
        self.fc1 = snn.Linear(D, 4 * D, **fk)
        self.fc2 = snn.Linear(4 * D, D, **fk)

    @torch.no_grad()
    def reset_parameters(self, g):
        for w in (self.qkv, self.proj.weight, self.fc1.weight, self.fc2.weight):  # lecun_normal (flax Dense)
            w.normal_(0.0, 1.0 / math.sqrt(w.shape[1]), generator=g)
        for b in (self.proj.bias, self.fc1.bias, self.fc2.bias):
            b.zero_()

    def attn(self, x, cache=None, pos=0):
        c = self.c
        B, T, D = x.shape
        qkv = linear(x, self.qkv)
        hd = D // c.num_heads
        if cache is not None:
            # cached decoding (inference): K/V rows [pos, pos+T) into the preallocated cache, the
            # queries attend to every cached row (causal with offset) -- split-K decode kernel for
            # single tokens, flash for the prompt (ops/attention.py decode_attention)
            H = c.num_heads
            q4 = qkv.view(B, T, 3 * H, hd)
            kc, vc = cache
            kc[:, pos:pos + T] = q4[:, :, H:2 * H]
            vc[:, pos:pos + T] = q4[:, :, 2 * H:]
            o = decode_attention(q4[:, :, :H], kc[:, :pos + T], vc[:, :pos + T], causal=True)
            return self.proj(o.reshape(B, T, D))
        p = c.dropout_rate if self.training else 0.0
        if p > 0:
            q4 = qkv.view(B, T, 3 * c.num_heads, hd)
            H = c.num_heads
            o = attention_dropout(q4[:, :, :H], q4[:, :, H:2 * H], q4[:, :, 2 * H:], True, None, p, True, -1e4)
            o = o.reshape(B, T, D)
        else:
            o = attention_packed(qkv, c.num_heads, c.num_heads, causal=True, head_dim=hd)
        return dropout(self.proj(o), p, self.training)

    def forward(self, x, cache=None, pos=0):
        c = self.c
        p = c.dropout_rate if self.training else 0.0
        a = self.attn(self.ln1(x), cache, pos)
        n2, h = self.ln2(a, residual=x)
        m = self.fc2(dropout(act(self.fc1(n2), "gelu_tanh"), p, self.training))
        return h + m


class GPT(tnn.Module):
    def __init__(self, c: GPTConfig = GPTConfig(), device=None, dtype=None, seed=42):
        super().__init__()
        fk = dict(device=device, dtype=dtype)
        self.c = c
        self.token_embed = tnn.Parameter(torch.empty(c.vocab_size, c.emb_dim, **fk))
        self.pos_embed = tnn.Parameter(torch.empty(1, c.block_size, c.emb_dim, **fk))
        self.layers = tnn.ModuleList([Block(c, **fk) for _ in range(c.num_layers)])
        self.ln_f = snn.LayerNorm(c.emb_dim, c.ln_eps, **fk)
        self.lm_head = tnn.Parameter(torch.empty(c.vocab_size, c.emb_dim, **fk))
        self.grad_ready_cb = None
        self.reset_parameters(seed)

    @torch.no_grad()
    def reset_parameters(self, seed):
        g = torch.Generator(device=self.token_embed.device).manual_seed(seed)
        self.token_embed.normal_(0.0, 1.0 / math.sqrt(self.c.emb_dim), generator=g)  # flax Embed default
        self.pos_embed.normal_(0.0, 0.02, generator=g)
        self.lm_head.normal_(0.0, 1.0 / math.sqrt(self.c.emb_dim), generator=g)
        for l in self.layers:
            l.reset_parameters(g)

    def param_groups(self):
        return [[self.token_embed, self.pos_embed]] + [list(l.parameters()) for l in self.layers] + \
            [list(self.ln_f.parameters()) + [self.lm_head]]

    def hidden(self, idx, cache=None, pos=0):
        c = self.c
        T = idx.shape[1]
        assert pos + T <= c.block_size
        x = embedding(self.token_embed, idx, pos=self.pos_embed.view(c.block_size, c.emb_dim)[pos:pos + T])
        x = dropout(x, c.dropout_rate, self.training)
        for i, l in enumerate(self.layers):
            x = mark_ready(x, self.grad_ready_cb, i + 1)
            x = l(x, None if cache is None else cache[i], pos)
        x = mark_ready(x, self.grad_ready_cb, len(self.layers) + 1)
        return self.ln_f(x)

    def forward(self, idx, targets=None):
        h = self.hidden(idx)
        if targets is None:
            return linear(h, self.lm_head)
        return linear_cross_entropy(h.reshape(-1, h.shape[-1]), self.lm_head, targets.reshape(-1))

    # ------------------------------------------------------------ cached decoding
    @property
    def max_context(self):
        return self.c.block_size

    def new_cache(self, B, Tmax):
        from ..infer.cache import KVCache
        c = self.c
        return KVCache(c.num_layers, B, Tmax, c.num_heads, c.emb_dim // c.num_heads,
                       device=self.token_embed.device, dtype=self.token_embed.dtype)

    def step(self, ids, cache, pos):
        """Write ids' K/V at cache rows [pos, pos+T) (learned positions pos..pos+T-1), return the
        last position's logits [B, V]."""
        h = self.hidden(ids, cache, pos)
        return linear(h[:, -1:], self.lm_head).float()[:, -1]

    @torch.no_grad()
    def generate(self, idx, max_new_tokens, greedy=True, temperature=1.0, top_k=None, generator=None,
                 eos_token_id=None, stats=None):
        """gpt-jax.ipynb:821-829 (greedy by default). While prompt + new tokens fit the learned
        position table (block_size) this is KV-cached: one prefill, then one token per step. Past
        block_size the reference crops the window to the last block_size tokens, which shifts
        every token's position embedding, so no cache can stand in: that tail re-forwards the
        cropped window exactly as the reference does."""
        from ..infer.generate import generate
        from ..infer.sampling import sample
        was = self.training
        self.eval()
        n_cached = max(0, min(max_new_tokens, self.c.block_size - idx.shape[1]))
        if n_cached:
            idx = generate(self, idx, n_cached, temperature, top_k, None, greedy, eos_token_id, generator, stats)
        for _ in range(max_new_tokens - n_cached):
            lg = self(idx[:, -self.c.block_size:])[:, -1].float()
            idx = torch.cat([idx, sample(lg, temperature, top_k, greedy, generator)], 1)
        self.train(was)
        return idx

    # ------------------------------------------------------------ Flax pytree layout
    def to_reference_params(self, dtype=torch.float32) -> Dict[str, torch.Tensor]:
        """The Flax pytree (gpt-jax.ipynb GPT.init), kernels (in, out); ``dtype`` None keeps the
        model's (fp64 for the numeric parity test)."""
        d = {"token_embed/embedding": self.token_embed.detach(), "pos_embed": self.pos_embed.detach()}
        for i, l in enumerate(self.layers):
            p = f"layers_{i}/"
            d[p + "ln1/scale"], d[p + "ln1/bias"] = l.ln1.weight.detach(), l.ln1.bias.detach()
            d[p + "attn/qkv/kernel"] = l.qkv.detach().t()
            d[p + "attn/proj/kernel"], d[p + "attn/proj/bias"] = l.proj.weight.detach().t(), l.proj.bias.detach()
            d[p + "ln2/scale"], d[p + "ln2/bias"] = l.ln2.weight.detach(), l.ln2.bias.detach()
            d[p + "mlp/fc1/kernel"], d[p + "mlp/fc1/bias"] = l.fc1.weight.detach().t(), l.fc1.bias.detach()
            d[p + "mlp/fc2/kernel"], d[p + "mlp/fc2/bias"] = l.fc2.weight.detach().t(), l.fc2.bias.detach()
        d["ln_f/scale"], d["ln_f/bias"] = self.ln_f.weight.detach(), self.ln_f.bias.detach()
        d["lm_head/kernel"] = self.lm_head.detach().t()
        return {k: (v if dtype is None else v.to(dtype)).clone() for k, v in d.items()}

    @torch.no_grad()
    def from_reference_params(self, d):
        t = lambda k: torch.as_tensor(d[k], dtype=self.token_embed.dtype)
        self.token_embed.copy_(t("token_embed/embedding"))
        self.pos_embed.copy_(t("pos_embed"))
        for i, l in enumerate(self.layers):
            p = f"layers_{i}/"
            l.ln1.weight.copy_(t(p + "ln1/scale")); l.ln1.bias.copy_(t(p + "ln1/bias"))
            l.qkv.copy_(t(p + "attn/qkv/kernel").t())
            l.proj.weight.copy_(t(p + "attn/proj/kernel").t()); l.proj.bias.copy_(t(p + "attn/proj/bias"))
            l.ln2.weight.copy_(t(p + "ln2/scale")); l.ln2.bias.copy_(t(p + "ln2/bias"))
            l.fc1.weight.copy_(t(p + "mlp/fc1/kernel").t()); l.fc1.bias.copy_(t(p + "mlp/fc1/bias"))
            l.fc2.weight.copy_(t(p + "mlp/fc2/kernel").t()); l.fc2.bias.copy_(t(p + "mlp/fc2/bias"))
        self.ln_f.weight.copy_(t("ln_f/scale")); self.ln_f.bias.copy_(t("ln_f/bias"))
        self.lm_head.copy_(t("lm_head/kernel").t())
        return self

    def num_params(self):
        return sum(p.numel() for p in self.parameters())
