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
from ..ops.attention import decode_attention, flash_attention
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

    def forward(self, res, delta, tp_group=None, cache=None, pos=0, sp=False, kv_prefix=None, want_kv=False):
        """``sp``: sequence parallel -- res/delta are [B, T/tp, D] shards; the TP regions
        open with an all-gather over T and close with a reduce-scatter over T.
        ``kv_prefix`` / ``want_kv`` (training, TP chunk pipelining in Gemma.hidden): this call
        holds tokens [pos, pos+T) of the sequence; its queries also attend to the (RoPE'd) K/V
        of the earlier tokens ``kv_prefix`` = (k, v), and ``want_kv`` returns this chunk's own
        (k, v) for the next chunk."""
        from ..parallel.tensor_parallel import (copy_to_tp, gather_seq, reduce_from_tp, reduce_grad_tp,
                                                reduce_scatter_seq, scale_grad)
        c = self.c
        if res is None:
            n1, h = rms_norm(delta, self.attn_norm, c.norm_eps), delta
        else:
            n1, h = rms_norm(delta, self.attn_norm, c.norm_eps, residual=res)
        hd, KV = c.head_dim, c.n_kv_heads
        if sp:
            assert cache is None, "sequence parallelism is a training layout"
            n1f = gather_seq(n1, tp_group)                               # [B, T, D]
            q = linear(n1f, self.wq)
            # the K/V activation grad is summed over TP below, so its input grad is complete on
            # every rank: scale by 1/tp before gather_seq's reduce-scatter sums the copies
            kv = reduce_grad_tp(linear(scale_grad(n1f, 1.0 / self.tp), self.wkv), tp_group)
        else:
            n1p = copy_to_tp(n1, tp_group)
            q = linear(n1p, self.wq)                                     # [B, T, hl*hd]
            kv = reduce_grad_tp(linear(n1, self.wkv), tp_group)          # replicated K/V, grads summed over TP
        B, T = q.shape[0], q.shape[1]
        qkv = torch.cat([q, kv], dim=-1)
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
        kv_out = None
        if cache is None and (kv_prefix is not None or want_kv):
            x4 = qkv.view(B, T, self.hl + 2 * KV, hd)
            k4, v4 = x4[:, :, self.hl:self.hl + KV], x4[:, :, self.hl + KV:]
            ev = None
            if want_kv and qkv.is_cuda:      # the next chunk waits for THIS point only, not for the
                ev = torch.cuda.Event()      # rest of the layer (its all-reduces) on this stream
                ev.record()
            kv_out = (k4, v4, ev)
            if kv_prefix is not None:     # causal with offset: query i sees keys <= prefix + i
                k4 = torch.cat([kv_prefix[0], k4], 1)
                v4 = torch.cat([kv_prefix[1], v4], 1)
            o = flash_attention(x4[:, :, :self.hl], k4, v4, causal=True).reshape(B, T, self.hl * hd)
        elif cache is None:
            o = attention_packed(qkv, self.hl, KV, causal=True, head_dim=hd)
        else:  # KV-cached inference: write this step's K/V, attend over the cache
            x4 = qkv.view(B, T, self.hl + 2 * KV, hd)
            kc, vc = cache
            kc[:, pos:pos + T] = x4[:, :, self.hl:self.hl + KV]
            vc[:, pos:pos + T] = x4[:, :, self.hl + KV:]
            o = decode_attention(x4[:, :, :self.hl], kc[:, :pos + T], vc[:, :pos + T], causal=True)
            o = o.reshape(B, T, self.hl * hd)
        close = reduce_scatter_seq if sp else reduce_from_tp
        a = close(linear(o, self.wo), tp_group)
        n2, h2 = rms_norm(a, self.ffn_norm, c.norm_eps, residual=h)
        f = glu(linear(gather_seq(n2, tp_group) if sp else copy_to_tp(n2, tp_group), self.w13), "gelu_tanh")
        out = close(linear(f, self.w2), tp_group)
        return (h2, out, kv_out) if want_kv else (h2, out)


    # ---- one-stream interleaved TP schedule (Gemma._hidden_interleaved): the layer in four
    # stages, each ending where a collective would block; the caller runs the other chunk's
    # stage between two stages of one chunk, so every collective has a stage to hide behind.
    def stage1(self, st, g):
        """norm1 on (res, delta | pending all-reduce of the previous layer's output)."""
        from ..parallel import comm
        c = self.c
        x = comm.ar_finish(st["out"]) if st.get("out") is not None else st["delta"]
        st["out"] = None
        if st["res"] is None:
            n1, h = rms_norm(x, self.attn_norm, c.norm_eps), x
        else:
            n1, h = rms_norm(x, self.attn_norm, c.norm_eps, residual=st["res"])
        st["n1"], st["h"] = n1, h
        st["sq"] = comm.grad_ar_start(n1, g)            # q path: gradient all-reduce (bwd)

    def stage2(self, st, g, pos, kv_prefix=None):
        """q / kv projections, RoPE, attention (queries of this chunk over kv_prefix + own K/V),
        o projection; starts its all-reduce. Returns this chunk's (k, v)."""
        from ..parallel import comm
        from ..parallel.tensor_parallel import reduce_grad_tp
        c = self.c
        hd, KV = c.head_dim, c.n_kv_heads
        q = linear(comm.grad_ar_finish(st.pop("sq")), self.wq)
        kv = reduce_grad_tp(linear(st.pop("n1"), self.wkv), g)
        B, T = q.shape[0], q.shape[1]
        qkv = rope_packed_(torch.cat([q, kv], dim=-1), self.hl + KV, c.rope_theta, pos, interleaved=False,
                           head_dim=hd)
        x4 = qkv.view(B, T, self.hl + 2 * KV, hd)
        k4, v4 = x4[:, :, self.hl:self.hl + KV], x4[:, :, self.hl + KV:]
        kk, vv = (k4, v4) if kv_prefix is None else (torch.cat([kv_prefix[0], k4], 1), torch.cat([kv_prefix[1], v4], 1))
        o = flash_attention(x4[:, :, :self.hl], kk, vv, causal=True).reshape(B, T, self.hl * hd)
        st["sa"] = comm.ar_start(linear(o, self.wo), g)
        return k4, v4

    def stage3(self, st, g):
        from ..parallel import comm
        n2, h2 = rms_norm(comm.ar_finish(st.pop("sa")), self.ffn_norm, self.c.norm_eps, residual=st.pop("h"))
        st["res"] = h2
        st["sm"] = comm.grad_ar_start(n2, g)

    def stage4(self, st, g):
        from ..parallel import comm
        f = glu(linear(comm.grad_ar_finish(st.pop("sm")), self.w13), "gelu_tanh")
        st["out"] = comm.ar_start(linear(f, self.w2), g)


class _Null:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


class _JoinStreams(torch.autograd.Function):
    """Identity at the end of the two-stream forward. Its backward runs first in the backward
    pass and queues an end-of-backward callback that makes the caller's stream wait for the
    side stream: weight gradients committed from it (utils/grad.py) are complete before the
    optimizer (or a DP bucket launched after backward) reads them."""

    @staticmethod
    def forward(ctx, x, side):
        ctx.side = side
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        side, main = ctx.side, torch.cuda.current_stream()
        torch.autograd.Variable._execution_engine.queue_callback(lambda: main.wait_stream(side))
        return g, None


class Gemma(tnn.Module):
    def __init__(self, c: GemmaConfig, device=None, dtype=torch.float32, tp_group=None, seed=0,
                 sequence_parallel=False, tp_group2=None, tp_schedule=None):
        """``tp_group2``: a second communicator over the SAME TP ranks. Given (TP > 1, no
        sequence parallelism), training splits each sequence into two halves that run as two
        pipelines -- half A on the current stream with ``tp_group``, half B on a second compute
        stream with ``tp_group2`` -- so every TP all-reduce of one half overlaps the other
        half's GEMMs / attention, forward AND backward (autograd runs each backward op on its
        forward's stream). Half B's queries attend to half A's K/V (causal with offset), so
        the result equals the unsplit model; see hidden()."""
        super().__init__()
        from ..parallel.tensor_parallel import tp_rank_size
        self.c = c
        self.tp_group = tp_group
        self.tp_rank, self.tp = tp_rank_size(tp_group)
        self.sp = bool(sequence_parallel) and self.tp > 1
        self.tp_group2 = tp_group2 if (self.tp > 1 and not self.sp) else None
        # "two_stream": half B on a second compute stream (_hidden_pipelined); "interleave": the
        # one-stream staged schedule (_hidden_interleaved). 1-GPU proxy, TP=8 Gemma-7B layers
        # (profiles/r3_overlap_proxy_tp_schedules.jsonl): two_stream hides 0.28-0.35 of the
        # collective time, interleave 0.19 at +17 % compute (its per-layer stages are two tiny
        # norms and two large blocks, so half of the collectives can only bracket a norm; and
        # every host-side stall of the one stream idles the GPU). SPA_TP_SCHEDULE overrides.
        self.tp_schedule = tp_schedule or os.environ.get("SPA_TP_SCHEDULE", "two_stream")
        assert self.tp_schedule in ("interleave", "two_stream"), self.tp_schedule
        self._side = None
        assert c.vocab_size % self.tp == 0
        fk = dict(device=device, dtype=dtype)
        self.embed = tnn.Parameter(torch.empty(c.vocab_size // self.tp, c.dim, **fk))   # vocab-parallel, tied head
        self.layers = tnn.ModuleList([GemmaBlock(c, self.tp, **fk) for _ in range(c.n_layers)])
        self.norm_f = tnn.Parameter(torch.ones(c.dim, **fk))
        self.norm_f.tp_replicated = True
        self.grad_ready_cb = None
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
        if self.tp_group2 is not None and self.tp_schedule == "two_stream":
            from ..utils.grad import mark_multi_stream
            mark_multi_stream(self.parameters())     # weight-grad commits come from two streams

    def param_groups(self):
        return [[self.embed]] + [list(l.parameters()) for l in self.layers] + [[self.norm_f]]

    def _pipelined(self, ids, cache):
        return (self.tp_group2 is not None and cache is None and torch.is_grad_enabled() and self.training
                and (ids.shape[0] % 2 == 0 or (ids.shape[1] % 2 == 0 and ids.shape[1] >= 2)))

    def _hidden_interleaved(self, ids, targets=None):
        """One-stream two-chunk TP schedule. Each layer is four stages per chunk (GemmaBlock
        stage1..4, each ending at a collective: the q-path and MLP-input gradient all-reduces of
        the backward, the o-projection and MLP-output all-reduces of the forward), issued as

            A.s1(l) B.s3(l-1) A.s2(l) B.s4(l-1) A.s3(l) B.s1(l) A.s4(l) B.s2(l) | A.s1(l+1) ...

        with every collective started at the end of one stage of its chunk and finished at the
        start of the next (parallel/comm ar_start / ar_finish, grad_ar_start / grad_ar_finish).
        Half B runs half a layer behind half A (its attention needs A's K/V of the same layer),
        so between the two halves of any collective the other chunk's stage runs -- in the
        forward, and, since autograd replays nodes in reverse creation order, in the backward.
        One compute stream: the chunks never share the CUs (the two-stream form's chunks fall
        into lockstep and their collectives coincide, profiles/r3_overlap_proxy_v2.jsonl)."""
        from ..parallel import comm
        from ..parallel.tensor_parallel import vocab_parallel_cross_entropy, vocab_parallel_embedding
        if ids.shape[1] % 2:             # an odd length with an even batch: the batch-split form
            return self._hidden_pipelined(ids, targets)
        c = self.c
        half = ids.shape[1] // 2
        g = (self.tp_group, self.tp_group2 if self.tp_group2 is not None else self.tp_group)
        st = [dict(res=None, delta=vocab_parallel_embedding(self.embed, ids[:, i * half:(i + 1) * half], g[i],
                                                            scale=math.sqrt(c.dim)), out=None) for i in range(2)]
        L = self.layers
        for i, l in enumerate(L):
            l.stage1(st[0], g[0])
            if i > 0:
                L[i - 1].stage3(st[1], g[1])
            kv = l.stage2(st[0], g[0], 0)
            if i > 0:
                L[i - 1].stage4(st[1], g[1])
            l.stage3(st[0], g[0])
            l.stage1(st[1], g[1])
            l.stage4(st[0], g[0])
            l.stage2(st[1], g[1], half, kv_prefix=kv)
        L[-1].stage3(st[1], g[1])
        outs, hs = [None, None], [None, None]
        for i in range(2):
            if i == 0:
                x = comm.ar_finish(st[0]["out"])
            else:
                L[-1].stage4(st[1], g[1])
                x = comm.ar_finish(st[1]["out"])
            outs[i], _ = rms_norm(x, self.norm_f, c.norm_eps, residual=st[i]["res"])
            if targets is not None:
                hs[i] = comm.grad_ar_start(outs[i], g[i])   # head input grads: all-reduced async
        if targets is None:
            return torch.cat(outs, 1)
        ls, nv = [None, None], [None, None]
        for i in range(2):
            t = targets[:, i * half:(i + 1) * half].reshape(-1)
            h = comm.grad_ar_finish(hs[i])
            ls[i] = vocab_parallel_cross_entropy(h.reshape(-1, c.dim), self.embed, t, g[i], reduce_dh=False)
            nv[i] = (t != -100).sum().clamp_min(1).to(ls[i].dtype)
        return (ls[0] * nv[0] + ls[1] * nv[1]) / (nv[0] + nv[1])

    def _hidden_pipelined(self, ids, targets=None):
        """Two-chunk TP pipeline (see __init__): per layer, half A runs on the current stream
        (``tp_group``), then half B on the side stream (``tp_group2``) once A's K/V exist.
        Each stream waits only on its own communicator, so while one half's all-reduce is on
        the wire the other half's kernels run; the backward replays the same two streams."""
        from ..parallel.tensor_parallel import vocab_parallel_embedding
        c = self.c
        T = ids.shape[1]
        half = T // 2
        # an even batch splits by SEQUENCES: the halves share no K/V and run as two independent
        # pipelines (B is offset by half a layer: it starts when A's first o-projection is done);
        # otherwise each sequence splits in halves and B's queries attend to A's K/V
        by_batch = ids.shape[0] % 2 == 0
        groups = (self.tp_group, self.tp_group2)
        cuda = ids.is_cuda
        main = torch.cuda.current_stream(ids.device) if cuda else None
        if cuda and self._side is None:
            from ..parallel.comm import side_stream
            self._side = side_stream(ids.device)
            from ..utils.grad import register_side_stream
            register_side_stream(self._side)
        side = self._side if cuda else None

        def on(i):
            return torch.cuda.stream(side) if (i == 1 and side is not None) else _Null()

        if side is not None:
            side.wait_stream(main)
        hb = ids.shape[0] // 2
        chunks = (ids[:hb], ids[hb:]) if by_batch else (ids[:, :half], ids[:, half:])
        delta = [None, None]
        for i in range(2):
            with on(i):
                delta[i] = vocab_parallel_embedding(self.embed, chunks[i], groups[i], scale=math.sqrt(c.dim))
        res = [None, None]
        for li, l in enumerate(self.layers):
            with on(0):
                res[0], delta[0], kv = l(res[0], delta[0], groups[0], None, 0, False, want_kv=True)
            if side is not None and (not by_batch or li == 0):
                side.wait_event(kv[2])       # half A's K/V are rope'd: half B may start its layer
                for t in kv[:2]:
                    t.record_stream(side)
            kv = kv[:2]
            with on(1):
                if by_batch:
                    res[1], delta[1] = l(res[1], delta[1], groups[1], None, 0, False)
                else:
                    res[1], delta[1] = l(res[1], delta[1], groups[1], None, half, False, kv_prefix=kv)
        outs = [None, None]
        for i in range(2):
            with on(i):
                outs[i], _ = rms_norm(delta[i], self.norm_f, c.norm_eps, residual=res[i])
        if targets is not None:
            # the vocab-parallel head + CE per chunk, each on its own stream and communicator: the
            # [T/2, D] hidden-gradient all-reduce of one chunk's head backward overlaps the other
            # chunk's head GEMMs (one [T, D] all-reduce here was the longest exposed collective)
            from ..parallel.tensor_parallel import vocab_parallel_cross_entropy
            tg = (targets[:hb], targets[hb:]) if by_batch else (targets[:, :half], targets[:, half:])
            ls, nv = [None, None], [None, None]
            for i in range(2):
                with on(i):
                    t = tg[i].reshape(-1)
                    ls[i] = vocab_parallel_cross_entropy(outs[i].reshape(-1, c.dim), self.embed, t, groups[i])
                    nv[i] = (t != -100).sum().clamp_min(1).to(ls[i].dtype)
            if side is not None:
                main.wait_stream(side)
                ls[1].record_stream(main)
                nv[1].record_stream(main)
            loss = (ls[0] * nv[0] + ls[1] * nv[1]) / (nv[0] + nv[1])
            return _JoinStreams.apply(loss, side) if side is not None else loss
        cat_dim = 0 if by_batch else 1
        if side is not None:
            main.wait_stream(side)
            outs[1].record_stream(main)
            return _JoinStreams.apply(torch.cat(outs, cat_dim), side)
        return torch.cat(outs, cat_dim)

    def hidden(self, ids, cache=None, pos=0):
        """Final-norm hidden states; a [B, T/tp, D] sequence shard under sequence parallelism."""
        from ..parallel.tensor_parallel import vocab_parallel_embedding
        c = self.c
        if self._pipelined(ids, cache):
            if self.tp_schedule == "interleave":
                return self._hidden_interleaved(ids)
            return self._hidden_pipelined(ids)
        sp = self.sp and cache is None
        x = vocab_parallel_embedding(self.embed, ids, self.tp_group, scale=math.sqrt(c.dim), sequence_parallel=sp)
        res, delta = None, x
        for i, l in enumerate(self.layers):
            delta = mark_ready(delta, self.grad_ready_cb, i + 1)
            res, delta = l(res, delta, self.tp_group, None if cache is None else cache[i], pos, sp)
        delta = mark_ready(delta, self.grad_ready_cb, len(self.layers) + 1)
        n, _ = rms_norm(delta, self.norm_f, c.norm_eps, residual=res)
        return n

    def forward(self, ids, targets=None):
        from ..parallel.tensor_parallel import gather_seq, scale_grad, vocab_parallel_cross_entropy
        c = self.c
        if targets is not None and self._pipelined(ids, None):
            if self.tp_schedule == "interleave":
                return self._hidden_interleaved(ids, targets)
            return self._hidden_pipelined(ids, targets)
        n = self.hidden(ids)
        if self.sp:  # the vocab-parallel head needs every token on every rank; its input grad is
            n = scale_grad(gather_seq(n, self.tp_group), 1.0 / self.tp)  # complete on each rank
        if targets is None:
            from ..parallel.tensor_parallel import gather_vocab_logits
            return gather_vocab_logits(linear(n, self.embed), self.tp_group)
        return vocab_parallel_cross_entropy(n.reshape(-1, c.dim), self.embed, targets.reshape(-1), self.tp_group)

    def sync_sequence_parallel_grads(self):
        """Norm weights see only their sequence shard under SP: sum their grads over TP
        (call after backward, before the optimizer)."""
        if self.sp:
            from ..parallel.tensor_parallel import sync_sequence_parallel_grads
            ps = [self.norm_f] + [p for l in self.layers for p in (l.attn_norm, l.ffn_norm)]
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
