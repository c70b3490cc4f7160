"""Gemma: reference-parity model (gemma/gemma.ipynb) and a paper-style Gemma-7B-shape
MQA model with tensor parallelism (BASELINE.json config #4).

GemmaRef reproduces the notebook exactly:
  RMSNorm fp32 eps 1e-6 :139-159; the "rotary" per-position dense matrix :169-208 (here
  the fused gemma_ref mode of the HIP rope kernel — no (T, D, D) materialisation);
  MQA :218-259 with heads//kv_heads = 2 full-width (D) query projections, one shared
  K and V, -inf mask then /sqrt(D), dropout on the attention output, concat -> Linear
  (2D->D); GeGLU :269-286 (exact-erf GELU, hidden 4D) + dropout; pre-norm decoder
  :320-337; Embedding (no sqrt(D) scale) -> dropout -> 12 layers -> norm -> Linear
  with bias (untied) :347-368. State-dict keys are identical to the reference.

Gemma (paper-style): fused QKV GEMM, true RoPE, H query heads x hd 256 with ONE KV head
(MQA), GeGLU fused [gate|up] GEMM + HIP glu kernel, sqrt(D)-scaled tied embedding,
RMSNorm; ``tp`` > 1 shards query heads, GeGLU hidden and the vocabulary over a TP
process group (K/V replicated because Hkv = 1 < tp; see parallel/tensor_parallel.py).
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass, replace
from typing import Optional

import torch
import torch.nn as tnn

from .. import nn as snn
from ..infer.graph import DecodeState
from ..ops import _ext, attention_packed, embedding, glu, linear, linear_cross_entropy, rms_norm, rope_packed_
from ..ops.linear import swiglu_mlp
from ..ops.attention import decode_attention, flash_attention
from ..ops.linear import linear_rows
from ..ops.misc import dropout
from ..ops.rope import RopeCache, gemma_ref_rotate
from ..utils.grad import mark_ready


# =============================================================================== reference
@dataclass
class GemmaRefConfig:
    block_size: int = 128
    batch_size: int = 64
    embeddings_dims: int = 768
    attn_dropout: float = 0.1
    no_of_heads: int = 4
    dropout: float = 0.1
    max_lr: float = 2.5e-4
    no_of_decoder_layers: int = 12
    no_kv_heads: int = 2
    vocab_size: int = 65
    total_steps: int = 5000
    eval_iters: int = 100


class _RMS(tnn.Module):
    def __init__(self, D):
        super().__init__()
        self.rmsnorm_layer = snn.RMSNorm(D, 1e-6)

    def forward(self, x):
        return self.rmsnorm_layer(x)


def _stacked_state_alias(module, pname, pieces):
    """Keep the reference's state-dict keys for a parameter stored stacked: ``pname`` [sum rows, K]
    is saved as the reference's separate ``pieces`` = [(key, rows)] and rebuilt from them on
    load, so one GEMM runs where the notebook runs several (gemma.ipynb state dict)."""
    def save(mod, sd, prefix, _meta):
        w = sd.pop(prefix + pname)
        r = 0
        for key, n in pieces:
            sd[prefix + key] = w[r:r + n]
            r += n
        return sd

    def load(sd, prefix, *_):
        keys = [prefix + k for k, _ in pieces]
        if all(k in sd for k in keys):
            sd[prefix + pname] = torch.cat([sd.pop(k) for k in keys], 0)

    module._register_state_dict_hook(save)
    module._register_load_state_dict_pre_hook(load)


class MQARef(tnn.Module):
    """gemma.ipynb:218-259. The notebook's 2 query projections, key and value (four D x D
    Linears) run as ONE GEMM on a stacked [2D + 2D, D] weight; the state dict still holds
    ``multi_query.{j}.weight``, ``key.weight`` and ``value.weight``."""

    def __init__(self, c: GemmaRefConfig):
        super().__init__()
        D = c.embeddings_dims
        self.c = c
        self.no_of_q_heads = c.no_of_heads // c.no_kv_heads if c.no_kv_heads > 0 else 1
        Hq = self.no_of_q_heads
        self.wqkv = tnn.Parameter(torch.empty((Hq + 2) * D, D))
        with torch.no_grad():                               # nn.Linear's default init, per piece
            for i in range(Hq + 2):
                tnn.init.kaiming_uniform_(self.wqkv[i * D:(i + 1) * D], a=math.sqrt(5))
        _stacked_state_alias(self, "wqkv", [(f"multi_query.{j}.weight", D) for j in range(Hq)]
                             + [("key.weight", D), ("value.weight", D)])
        self.linear_layer = snn.Linear(D * Hq, D, bias=False)

    def forward(self, x):
        B, T, D = x.shape
        Hq = self.no_of_q_heads
        p = self.c.attn_dropout if self.training else 0.0
        qkv = linear(x, self.wqkv).view(B, T, Hq + 2, D)
        q, k, v = qkv[:, :, :Hq], qkv[:, :, Hq:Hq + 1], qkv[:, :, Hq + 1:]
        o = flash_attention(gemma_ref_rotate(q), gemma_ref_rotate(k), v, causal=True, scale=1.0 / math.sqrt(D))
        o = dropout(o, p, self.training)                                  # dropout on each head's output
        return dropout(self.linear_layer(o.reshape(B, T, -1)), p, self.training)


class GeGLURef(tnn.Module):
    """gemma.ipynb:269-286: gelu(l1 x) * (l2 x) -> l3. l1 and l2 are ONE GEMM on a stacked
    [8D, D] weight feeding the fused HIP glu kernel (state dict keeps ``linear_layer{1,2}``)."""

    def __init__(self, D):
        super().__init__()
        self.w12 = tnn.Parameter(torch.empty(8 * D, D))
        with torch.no_grad():
            for i in range(2):
                tnn.init.kaiming_uniform_(self.w12[i * 4 * D:(i + 1) * 4 * D], a=math.sqrt(5))
        _stacked_state_alias(self, "w12", [("linear_layer1.weight", 4 * D), ("linear_layer2.weight", 4 * D)])
        self.linear_layer3 = snn.Linear(4 * D, D, bias=False)

    def forward(self, x):
        return self.linear_layer3(glu(linear(x, self.w12), "gelu"))


class FFNRef(tnn.Module):
    def __init__(self, c):
        super().__init__()
        self.gglu = GeGLURef(c.embeddings_dims)
        self.p = c.dropout

    def forward(self, x):
        return dropout(self.gglu(x), self.p, self.training)


class DecoderLayerRef(tnn.Module):
    def __init__(self, c):
        super().__init__()
        self.feedforward_network = FFNRef(c)
        self.mqa = MQARef(c)
        self.norm1 = _RMS(c.embeddings_dims)
        self.norm2 = _RMS(c.embeddings_dims)

    def forward(self, x):
        x = x + self.mqa(self.norm1(x))
        return x + self.feedforward_network(self.norm2(x))


class GemmaRef(tnn.Module):
    def __init__(self, c: GemmaRefConfig = GemmaRefConfig()):
        super().__init__()
        self.c = c
        self.embeddings = snn.Embedding(c.vocab_size, c.embeddings_dims)
        self.decoder = tnn.Sequential(*[DecoderLayerRef(c) for _ in range(c.no_of_decoder_layers)])
        self.linear_layer = snn.Linear(c.embeddings_dims, c.vocab_size)
        self.norm = _RMS(c.embeddings_dims)

    def forward(self, x, targets=None):
        x = dropout(self.embeddings(x), self.c.dropout, self.training)
        x = self.norm(self.decoder(x))
        if targets is None:
            return self.linear_layer(x)
        return linear_cross_entropy(x.reshape(-1, x.shape[-1]), self.linear_layer.weight, targets.reshape(-1),
                                    bias=self.linear_layer.bias)

    @torch.no_grad()
    def generate(self, idx, max_new_tokens, generator=None):
        """gemma.ipynb:608-630: crop to block_size, softmax + multinomial."""
        was = self.training
        self.eval()
        for _ in range(max_new_tokens):
            lg = self(idx[:, -self.c.block_size:])[:, -1].float()
            idx = torch.cat([idx, torch.multinomial(torch.softmax(lg, -1), 1, generator=generator)], 1)
        self.train(was)
        return idx


# =============================================================================== paper-style
@dataclass
class GemmaConfig:
    vocab_size: int = 256000
    dim: int = 3072
    n_layers: int = 28
    n_heads: int = 16
    n_kv_heads: int = 1           # MQA (BASELINE.json config #4)
    head_dim: int = 256
    ffn_hidden: int = 24576
    max_seq_len: int = 8192
    norm_eps: float = 1e-6
    rope_theta: float = 10000.0
    batch_size: int = 1


PRESETS = {
    "gemma_ref": GemmaRefConfig(),
    "gemma_7b_mqa": GemmaConfig(),
    "gemma_tiny": GemmaConfig(vocab_size=1024, dim=512, n_layers=2, n_heads=8, n_kv_heads=1, head_dim=64,
                              ffn_hidden=1024, max_seq_len=256),
}


def config(name, **kw):
    return replace(PRESETS[name], **kw)


class GemmaBlock(tnn.Module):
    def __init__(self, c: GemmaConfig, tp_size: int = 1, **fk):
        super().__init__()
        self.c, self.tp = c, tp_size
        assert c.n_heads % tp_size == 0 and c.ffn_hidden % tp_size == 0
        self.hl = c.n_heads // tp_size                                   # local query heads
        self.attn_norm = tnn.Parameter(torch.ones(c.dim, **fk))
        self.wq = tnn.Parameter(torch.empty(self.hl * c.head_dim, c.dim, **fk))      # column-parallel
        self.wkv = tnn.Parameter(torch.empty(2 * c.n_kv_heads * c.head_dim, c.dim, **fk))  # replicated
        self.wo = tnn.Parameter(torch.empty(c.dim, self.hl * c.head_dim, **fk))      # row-parallel
        self.ffn_norm = tnn.Parameter(torch.ones(c.dim, **fk))
        self.w13 = tnn.Parameter(torch.empty(2 * c.ffn_hidden // tp_size, c.dim, **fk))  # column-parallel [gate|up]
        self.w2 = tnn.Parameter(torch.empty(c.dim, c.ffn_hidden // tp_size, **fk))       # row-parallel
        for p in (self.wkv, self.attn_norm, self.ffn_norm):
            p.tp_replicated = True

    @torch.no_grad()
    def reset_parameters(self, g, tp_rank: int = 0):
        """Draw the UNSHARDED tensors and keep this TP rank's slice, so a TP=n model starts
        as the exact shards of the TP=1 model (shard_gemma_from_full); drawing only the local
        shard from the shared generator would give every rank identical heads / FFN columns
        that stay symmetric through training."""
        c, tp = self.c, self.tp
        H, hd, F, D = c.n_heads, c.head_dim, c.ffn_hidden, c.dim
        full = {n: torch.empty(shape, device=self.wq.device, dtype=self.wq.dtype).normal_(0.0, 0.02, generator=g)
                for n, shape in (("wq", (H * hd, D)), ("wkv", tuple(self.wkv.shape)), ("wo", (D, H * hd)),
                                 ("w13", (2 * F, D)), ("w2", (D, F)))}
        hl, fl = self.hl * hd, F // tp
        r = tp_rank
        self.wq.copy_(full["wq"][r * hl:(r + 1) * hl])
        self.wkv.copy_(full["wkv"])
        self.wo.copy_(full["wo"][:, r * hl:(r + 1) * hl])
        self.w13.copy_(torch.cat([full["w13"][r * fl:(r + 1) * fl], full["w13"][F + r * fl:F + (r + 1) * fl]]))
        self.w2.copy_(full["w2"][:, r * fl:(r + 1) * fl])

    def forward(self, res, delta, tp_group=None, cache=None, pos=0):
        """Plain (replicated residual) TP layer; the sequence-parallel layer is sp_attn + sp_mlp
        (driven by Gemma._hidden_sp)."""
        from ..parallel.tensor_parallel import copy_to_tp, reduce_from_tp, reduce_grad_tp
        c = self.c
        if res is None:
            n1, h = rms_norm(delta, self.attn_norm, c.norm_eps), delta
        else:
            n1, h = rms_norm(delta, self.attn_norm, c.norm_eps, residual=res)
        hd, KV = c.head_dim, c.n_kv_heads
        if self.tp == 1:     # one GEMM over the adjacent q and K/V weights
            qkv = linear_rows(n1, (self.wq, self.wkv))
        else:
            q = linear(copy_to_tp(n1, tp_group), self.wq)                # [B, T, hl*hd]
            kv = reduce_grad_tp(linear(n1, self.wkv), tp_group)          # replicated K/V, grads summed over TP
            qkv = torch.cat([q, kv], dim=-1)
        B, T = qkv.shape[0], qkv.shape[1]
        if isinstance(pos, DecodeState):  # graph-capturable decode step: positions on the device
            x4 = qkv.view(B, T, self.hl + 2 * KV, hd)
            cos, sin = RopeCache.get(pos.max_len, hd, c.rope_theta, qkv.device)
            kc, vc = cache
            # one launch: rotate_half RoPE on q (in place) and k, k/v rows into the cache
            _ext.ops().rope_kv_write_(x4, cos, sin, pos.positions, pos.index, kc, vc, self.hl, KV, 1)
            o = decode_attention(x4[:, :, :self.hl], kc, vc, causal=True, kv_len=pos.kv_len)
            a = reduce_from_tp(linear(o.reshape(B, T, self.hl * hd), self.wo), tp_group)
            n2, h2 = rms_norm(a, self.ffn_norm, c.norm_eps, residual=h)
            f = glu(linear(copy_to_tp(n2, tp_group), self.w13), "gelu_tanh")
            return h2, reduce_from_tp(linear(f, self.w2), tp_group)
        qkv = rope_packed_(qkv, self.hl + KV, c.rope_theta, pos, interleaved=False, head_dim=hd)
        if cache is None:
            o = attention_packed(qkv, self.hl, KV, causal=True, head_dim=hd)
        else:  # KV-cached inference: write this step's K/V, attend over the cache
            x4 = qkv.view(B, T, self.hl + 2 * KV, hd)
            kc, vc = cache
            kc[:, pos:pos + T] = x4[:, :, self.hl:self.hl + KV]
            vc[:, pos:pos + T] = x4[:, :, self.hl + KV:]
            o = decode_attention(x4[:, :, :self.hl], kc[:, :pos + T], vc[:, :pos + T], causal=True)
            o = o.reshape(B, T, self.hl * hd)
        a = reduce_from_tp(linear(o, self.wo), tp_group)
        n2, h2 = rms_norm(a, self.ffn_norm, c.norm_eps, residual=h)
        return h2, reduce_from_tp(swiglu_mlp(copy_to_tp(n2, tp_group), self.w13, self.w2, "gelu_tanh"), tp_group)

    # ---- sequence-parallel pieces. Between the TP regions the residual stream is a [B, T/tp, D]
    # sequence shard h; each region starts from the all-gathered full sequence hf (its norm runs on
    # every rank) and ends with a TP-partial [B, T, D] product into which this rank's residual rows
    # were added, so the layer boundary is one reduce-scatter -> all-gather pair with no compute
    # between (tensor_parallel.rs_ag_start / rs_ag_finish) -- Gemma._forward_sp_pair runs one
    # chunk's pair under the other chunk's GEMMs.
    def sp_attn(self, h, hf, g, pos=0, kv_prefix=None, want_kv=False):
        """norm1 of the gathered input, q and K/V projections (MQA K/V of the full sequence on
        every rank: its activation gradient stays TP-partial and the boundary's reduce-scatter sums
        it with the q path's), RoPE, attention, o projection + this rank's residual rows.
        ``kv_prefix``: the packed (RoPE'd) qkv buffer of the earlier chunk of the same sequences,
        whose keys this chunk's queries also see (causal with offset). Returns the TP-partial
        [B, T, D] and, with ``want_kv``, this chunk's packed qkv buffer for the next chunk."""
        from ..ops.attention import attention_packed_prefix
        from ..parallel.tensor_parallel import add_owner_rows
        c = self.c
        hd, KV = c.head_dim, c.n_kv_heads
        n1f = rms_norm(hf, self.attn_norm, c.norm_eps)
        qkv = linear_rows(n1f, (self.wq, self.wkv))
        B, T = qkv.shape[0], qkv.shape[1]
        qkv = rope_packed_(qkv, self.hl + KV, c.rope_theta, pos, interleaved=False, head_dim=hd)
        if kv_prefix is None:
            o = attention_packed(qkv, self.hl, KV, causal=True, head_dim=hd)
        else:
            o = attention_packed_prefix(qkv, kv_prefix, self.hl, KV, hd)
        out = add_owner_rows(linear(o.reshape(B, T, self.hl * hd), self.wo), h, g)
        return out, (qkv if want_kv else None)

    def sp_mlp(self, h, hf, g):
        """norm2 of the gathered input, GeGLU, down projection + this rank's residual rows
        (TP-partial [B, T, D])."""
        from ..parallel.tensor_parallel import add_owner_rows
        n2f = rms_norm(hf, self.ffn_norm, self.c.norm_eps)
        return add_owner_rows(swiglu_mlp(n2f, self.w13, self.w2, "gelu_tanh"), h, g)


class Gemma(tnn.Module):
    def __init__(self, c: GemmaConfig, device=None, dtype=torch.float32, tp_group=None, seed=0,
                 sequence_parallel=None, tp_pipeline=None):
        """``sequence_parallel`` (default: on when TP > 1): Megatron sequence parallelism for
        training -- the residual stream between TP regions is a [B, T/tp, D] shard, each TP
        region opens with an all-gather over T and closes with a reduce-scatter.
        ``tp_pipeline`` (default on; env SPA_TP_PIPE=0 turns it off): under sequence parallelism a
        training forward with targets runs as two chunks (the batch halves, or the sequence
        halves when the batch is odd) whose collectives overlap each other's compute -- see
        _forward_sp_pair."""
        super().__init__()
        from ..parallel.tensor_parallel import tp_rank_size
        self.c = c
        self.tp_group = tp_group
        self.tp_rank, self.tp = tp_rank_size(tp_group)
        self.sp = (self.tp > 1) if sequence_parallel is None else (bool(sequence_parallel) and self.tp > 1)
        self.tp_pipeline = (os.environ.get("SPA_TP_PIPE", "1") != "0") if tp_pipeline is None else bool(tp_pipeline)
        assert c.vocab_size % self.tp == 0
        fk = dict(device=device, dtype=dtype)
        self.embed = tnn.Parameter(torch.empty(c.vocab_size // self.tp, c.dim, **fk))   # vocab-parallel, tied head
        self.layers = tnn.ModuleList([GemmaBlock(c, self.tp, **fk) for _ in range(c.n_layers)])
        self.norm_f = tnn.Parameter(torch.ones(c.dim, **fk))
        self.norm_f.tp_replicated = True
        self.grad_ready_cb = None
        self.param_wait_cb = None   # overlapped optimizer: wait for param group i's update before use
        with torch.no_grad():
            # unsharded draws sliced per TP rank: TP=n init == shards of the TP=1 init
            g = torch.Generator(device=self.embed.device).manual_seed(seed)
            vl = c.vocab_size // self.tp
            if self.tp == 1:
                self.embed.normal_(0.0, 0.02, generator=g)
            else:
                full = torch.empty(c.vocab_size, c.dim, **fk).normal_(0.0, 0.02, generator=g)
                self.embed.copy_(full[self.tp_rank * vl:(self.tp_rank + 1) * vl])
                del full
            gl = torch.Generator(device=self.embed.device).manual_seed(seed)
            for l in self.layers:
                l.reset_parameters(gl, self.tp_rank)

    def param_groups(self):
        return [[self.embed]] + [list(l.parameters()) for l in self.layers] + [[self.norm_f]]

    def _pair_split(self, ids):
        """'batch' / 'sequence' when a training forward runs as two overlapped chunks, else None."""
        if not (self.sp and self.tp_pipeline and self.training and torch.is_grad_enabled()):
            return None
        B, T = ids.shape
        if B % 2 == 0 and T % self.tp == 0:
            return "batch"
        if T % (2 * self.tp) == 0:
            return "sequence"
        return None

    def _embed_sp(self, ids):
        """Vocab-parallel embedding rows of ``ids`` (TP-partial [B, T, D]): the first layer
        boundary's reduce-scatter sums them into the residual shard."""
        from ..parallel.tensor_parallel import vocab_parallel_embedding
        return vocab_parallel_embedding(self.embed, ids, self.tp_group, scale=math.sqrt(self.c.dim),
                                        sequence_parallel=True, reduce=False)

    def _hidden_sp(self, ids):
        """Sequence-parallel forward (one chunk): the final norm of the gathered last residual,
        [B, T, D] on every rank."""
        from ..parallel.tensor_parallel import rs_ag
        c, g = self.c, self.tp_group
        wait = self.param_wait_cb or (lambda i: None)
        wait(0)
        h, hf = rs_ag(self._embed_sp(ids), g)
        for i, l in enumerate(self.layers):
            wait(i + 1)
            hf = mark_ready(hf, self.grad_ready_cb, i + 1)
            h, hf = rs_ag(l.sp_attn(h, hf, g)[0], g)
            h, hf = rs_ag(l.sp_mlp(h, hf, g), g)
        wait(len(self.layers) + 1)
        hf = mark_ready(hf, self.grad_ready_cb, len(self.layers) + 1)
        return rms_norm(hf, self.norm_f, c.norm_eps)

    def forward_pair(self, ids0, t0, ids1, t1):
        """loss(ids0, t0) + loss(ids1, t1) for two gradient-accumulation micro-batches. Under
        sequence-parallel TP they run as the overlapped chunk pair (each micro-batch at its own
        full shape: no GEMM is split); otherwise one after the other."""
        if self.sp and self.tp_pipeline and self.training and torch.is_grad_enabled():
            return self._forward_sp_pair(None, None, "micro", parts=(ids0, ids1), tps=(t0, t1))
        # one backward covers both micro-batches and autograd finishes micro-batch 1's before it
        # starts micro-batch 0's: a layer's DP bucket may launch only once BOTH passed its marker
        cb = self.grad_ready_cb
        if cb is None:
            return self(ids0, t0) + self(ids1, t1)
        from .deepseekv3 import _PairReady
        self.grad_ready_cb = _PairReady(cb)
        try:
            return self(ids0, t0) + self(ids1, t1)
        finally:
            self.grad_ready_cb = cb

    def pair_overlaps(self):
        """True when forward_pair overlaps something (the sequence-parallel TP chunk pair);
        otherwise pairing only keeps two micro-batches' activations alive (Trainer pairs only then)."""
        return bool(self.sp and self.tp_pipeline and self.training and torch.is_grad_enabled())

    def _forward_sp_pair(self, ids, targets, split, parts=None, tps=None):
        """Sequence-parallel TP training step as two chunks on one compute stream. Per layer the
        compute stream runs

            A.attn(l)  B.attn(l)  A.mlp(l)  B.mlp(l)  |  A.attn(l+1) ...

        (attn = norm1, q / K/V projections, attention, o projection of the gathered input; mlp =
        norm2, GeGLU, down projection), and after each piece its chunk's layer boundary -- the
        reduce-scatter of the partial output into the residual shard and the all-gather of that
        shard -- is issued to the communicator at once and waited for only before that chunk's next
        piece, so it runs under the other chunk's piece. No compute sits between the two
        collectives (the residual add is folded into the partial output, the norm runs on the
        gathered sequence), so no side compute stream is needed. The backward replays the pairs
        in reverse (launched at the finish node, waited at the start node), under the other
        chunk's backward pieces. ``split`` "sequence": chunk B is the second half of every
        sequence and attends to chunk A's K/V of the same layer (causal with offset), so the
        result equals the unsplit model."""
        from ..parallel.tensor_parallel import rs_ag_finish, rs_ag_start, vocab_parallel_cross_entropy
        c, g = self.c, self.tp_group
        if split == "micro":                 # two micro-batches (forward_pair)
            pos = (0, 0)
        elif split == "batch":
            B = ids.shape[0]
            parts, tps, pos = (ids[:B // 2], ids[B // 2:]), (targets[:B // 2], targets[B // 2:]), (0, 0)
        else:
            T = ids.shape[1]
            parts, tps, pos = (ids[:, :T // 2], ids[:, T // 2:]), (targets[:, :T // 2], targets[:, T // 2:]), (0, T // 2)
        cb = None
        if self.grad_ready_cb is not None:
            from .deepseekv3 import _PairReady
            cb = _PairReady(self.grad_ready_cb)
        wait = self.param_wait_cb or (lambda i: None)
        L = self.layers
        wait(0)
        pend = [rs_ag_start(self._embed_sp(parts[m]), g) for m in (0, 1)]
        for li, l in enumerate(L):
            wait(li + 1)
            kv = None
            for m in (0, 1):
                h, hf = rs_ag_finish(pend[m])
                hf = mark_ready(hf, cb, li + 1)
                o, kvo = l.sp_attn(h, hf, g, pos[m], kv_prefix=kv if (m == 1 and split == "sequence") else None,
                                   want_kv=(m == 0 and split == "sequence"))
                kv = kvo
                pend[m] = rs_ag_start(o, g)
            for m in (0, 1):
                h, hf = rs_ag_finish(pend[m])
                pend[m] = rs_ag_start(l.sp_mlp(h, hf, g), g)
        wait(len(L) + 1)
        ls, nv = [None, None], [None, None]
        for m in (0, 1):
            _, hf = rs_ag_finish(pend[m])
            hf = mark_ready(hf, cb, len(L) + 1)
            n = rms_norm(hf, self.norm_f, c.norm_eps)
            t = tps[m].reshape(-1)
            # the head's input gradient stays TP-partial: the boundary's reduce-scatter sums it
            ls[m] = vocab_parallel_cross_entropy(n.reshape(-1, c.dim), self.embed, t, g, reduce_dh=False)
            nv[m] = (t != -100).sum().clamp_min(1).to(ls[m].dtype)
        if split == "micro":
            return ls[0] + ls[1]
        return (ls[0] * nv[0] + ls[1] * nv[1]) / (nv[0] + nv[1])

    def hidden(self, ids, cache=None, pos=0):
        """Final-norm hidden states [B, T, D] (under sequence parallelism the full sequence on
        every rank)."""
        from ..parallel.tensor_parallel import vocab_parallel_embedding
        c = self.c
        if self.sp and cache is None:
            return self._hidden_sp(ids)
        wait = self.param_wait_cb or (lambda i: None)
        wait(0)
        x = vocab_parallel_embedding(self.embed, ids, self.tp_group, scale=math.sqrt(c.dim))
        res, delta = None, x
        for i, l in enumerate(self.layers):
            wait(i + 1)
            delta = mark_ready(delta, self.grad_ready_cb, i + 1)
            res, delta = l(res, delta, self.tp_group, None if cache is None else cache[i], pos)
        wait(len(self.layers) + 1)
        delta = mark_ready(delta, self.grad_ready_cb, len(self.layers) + 1)
        n, _ = rms_norm(delta, self.norm_f, c.norm_eps, residual=res)
        return n

    def forward(self, ids, targets=None):
        from ..parallel.tensor_parallel import vocab_parallel_cross_entropy
        c = self.c
        if targets is not None:
            split = self._pair_split(ids)
            if split is not None:
                return self._forward_sp_pair(ids, targets, split)
        n = self.hidden(ids)
        if targets is None:
            from ..parallel.tensor_parallel import gather_vocab_logits
            return gather_vocab_logits(linear(n, self.embed), self.tp_group)
        # under SP the head's input gradient stays TP-partial: the boundary's reduce-scatter sums it
        return vocab_parallel_cross_entropy(n.reshape(-1, c.dim), self.embed, targets.reshape(-1), self.tp_group,
                                            reduce_dh=not self.sp)

    def sync_sequence_parallel_grads(self):
        """Parameters used on sequence shards (norm weights, the replicated K/V projection) see
        only their shard's tokens: sum their grads over TP in one packed all-reduce (call after
        backward, before the optimizer)."""
        if self.sp:
            from ..parallel.tensor_parallel import sync_sequence_parallel_grads
            ps = [self.norm_f] + [p for l in self.layers for p in (l.attn_norm, l.ffn_norm, l.wkv)]
            sync_sequence_parallel_grads(ps, self.tp_group)

    # ---------------------------------------------------------------- inference
    @property
    def max_context(self):
        return self.c.max_seq_len

    def new_cache(self, B, Tmax):
        from ..infer.cache import KVCache
        c = self.c
        return KVCache(c.n_layers, B, Tmax, c.n_kv_heads, c.head_dim, device=self.embed.device, dtype=self.embed.dtype)

    def step(self, ids, cache, pos):
        from ..parallel.tensor_parallel import gather_vocab_logits
        n = self.hidden(ids, cache, pos)
        return gather_vocab_logits(linear(n[:, -1:], self.embed), self.tp_group).float()[:, -1]

    def step_graph(self, ids, cache, state):
        """One-token decode step with every position on the device (HIP-graph capturable,
        infer/graph.py): fused rotate_half RoPE + cache write at ``state.index``, MQA decode
        kernel over ``state.kv_len`` rows. Single TP rank (a captured step holds no collectives)."""
        if self.tp != 1:
            raise NotImplementedError("graph decode runs on one TP rank; use step() under tensor parallelism")
        n = self.hidden(ids, cache, state)
        return linear(n, self.embed).float()[:, -1]

    @torch.no_grad()
    def generate(self, ids, max_new_tokens, temperature=1.0, top_k=None, greedy=False, generator=None,
                 top_p=None, eos_token_id=None, stats=None):
        """KV-cached MQA decoding (the reference re-runs the window per token, gemma.ipynb:608-630)."""
        from ..infer.generate import generate
        return generate(self, ids, max_new_tokens, temperature, top_k, top_p, greedy, eos_token_id, generator, stats)

    def flops_per_token(self, T):
        c = self.c
        per = c.dim * (c.n_heads + 2 * c.n_kv_heads) * c.head_dim + c.dim * c.n_heads * c.head_dim + \
            3 * c.dim * c.ffn_hidden
        return 6 * (c.n_layers * per + c.vocab_size * c.dim) + 6 * c.n_layers * c.n_heads * c.head_dim * T
