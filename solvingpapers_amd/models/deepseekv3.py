"""DeepSeek-V3: multi-head latent attention + DeepSeekMoE (shared + routed experts with
aux-loss-free balancing) + multi-token prediction — deepseekv3/deepseekv3.ipynb.

One model class, two attention families selected by the config:

``attention="ref"`` (preset ``dsv3_ref``) reproduces the notebook exactly (SURVEY
Appendix A Q1-Q5): per-head latents ``W_dkv`` (:1143-1148), absorbed query
``x @ (query.W^T W_k.W)`` scored against the latent, values ``W_v(latent)``; the
``kv_cache`` threaded through every head and layer (:1256-1261,1406-1408) plus the
``tril(T, Tc)`` mask means every head of every layer attends ONLY to layer-0/head-0's
latent — so here that latent ``L0`` is computed once and all layers attend to it with
a single H-head / 1-KV-head flash attention (``k = v = L0``, hd = latent) followed by
the per-head ``W_v`` up-projection (the absorbed-V form, identical math). Sinusoidal
PE (:836-842), tied embedding/LM head (:1393,1501), ``x * 2 * L^-0.5`` before the final
RMSNorm (:1411), torch RMSNorm with eps = finfo(fp32).eps (:914), MoE with
softmax-over-(logits+bias)-top-k gating and the SOFT-mass bias update (:1041-1086).

``attention="mla"`` (presets ``dsv3_style`` / ``dsv3_tiny``) is the paper's MLA: one
shared compressed KV latent per layer (kv_lora) + a decoupled RoPE key shared across
heads, optional low-rank query, per-head nope/rope/v dims; training runs the flash
kernel on the up-projected heads, cached decoding runs in latent space with the
up-projections absorbed (cache = kv_lora + rope floats per token per layer). Routing
bias steers selection only and is updated from token COUNTS all-reduced over the
data/expert-parallel group; MTP depth-k modules predict token i+k+1.

Routed experts run through ops/moe.py (HIP router, counting-sort permute, MFMA grouped
GEMMs, weighted combine) or parallel/expert_parallel.py under EP. Expert hidden sizes
are padded to a multiple of 8 internally (zero rows/cols: exact, gradients stay zero)
so the reference's 1365 runs on the vectorised kernels; the reference state-dict
exporter slices the padding off.
"""
from __future__ import annotations

import contextlib
import math
import os
from dataclasses import dataclass, replace
from typing import Dict, List, Optional

import torch
import torch.distributed as dist
import torch.nn as tnn
from types import SimpleNamespace

from ..ops import apply_rope, embedding, glu, layer_norm, linear, linear_cross_entropy, rms_norm
from ..ops.attention import attention_dropout, flash_attention, mla_attention, split_last
from ..ops.misc import dropout
from ..ops.moe import route, router_logits
from ..utils.grad import mark_ready
from ..infer.sampling import sample

FP32_EPS = float(torch.finfo(torch.float32).eps)


@dataclass
class DSV3Config:
    vocab_size: int = 50257
    block_size: int = 256
    dim: int = 512
    n_layers: int = 6
    n_heads: int = 8
    attention: str = "ref"          # "ref" (notebook latent heads) | "mla" (paper MLA)
    latent_dim: int = 64            # ref: per-head latent width
    q_lora_rank: int = 0            # mla
    kv_lora_rank: int = 512
    qk_nope_dim: int = 64
    qk_rope_dim: int = 64
    v_head_dim: int = 128
    rope_theta: float = 10000.0
    pos_emb: str = "sinusoidal"     # "sinusoidal" (ref) | "none"
    n_experts: int = 8
    top_k: int = 2
    n_shared: int = 1
    expert_hidden: int = 0          # 0 -> (2*D*4)//3 (reference SWiGLUExpert)
    n_dense_layers: int = 0         # leading layers with a dense SwiGLU FFN
    dense_hidden: int = 0
    moe_fp8: bool = False           # routed-expert fwd/dX GEMMs in OCP e4m3 (BASELINE config #5)
    # EP dispatch: 0 = exact split sizes (one host sync per MoE layer per micro-batch); > 0 = the
    # host-sync-free padded dispatch with this capacity factor (parallel/expert_parallel.py)
    ep_capacity: float = 0.0
    fp8_linears: bool = False       # dense projections too (MLA, shared / dense FFN): the V3 recipe
    noisy_topk: bool = False        # ref (deepseekv3.ipynb:390,1026-1039): + softplus(noise(x)) * N(0,1)
    aux_free: bool = True
    bias_update_rate: float = 1e-3
    bias_in_weights: bool = True    # ref: softmax over (logits + bias); paper: bias steers selection only
    balance_stat: str = "soft"      # "soft" (ref Q4: probability mass) | "counts" (tokens, all-reduced)
    dropout: float = 0.1
    attn_dropout: float = 0.1
    final_scale: bool = True        # x * 2 * L^-0.5 before the final norm
    norm_eps: float = FP32_EPS
    mtp_heads: int = 0
    mtp_lambda: float = 0.3
    init_std: float = 0.02
    # reference training hyper-parameters (deepseekv3.ipynb:369-396,1923-1934)
    batch_size: int = 16
    max_lr: float = 6e-4
    min_lr: float = 6e-5
    warmup_iters: int = 400
    total_iters: int = 10000
    weight_decay: float = 0.1
    beta1: float = 0.9
    beta2: float = 0.95
    eps: float = 1e-8
    clip: float = 1.0

    @property
    def head_size(self):
        return self.dim // self.n_heads

    @property
    def ffn_hidden(self):
        return self.expert_hidden or (self.dim * 2 * 4) // 3

    @property
    def qk_head_dim(self):
        return self.qk_nope_dim + self.qk_rope_dim


PRESETS = {
    "dsv3_ref": DSV3Config(),
    # the notebook's stale checkpoint copy (SURVEY D23,
    # deepseekv3/.ipynb_checkpoints/deepseekv3-checkpoint.ipynb:53-80): block 512, batch 32 and one
    # MTP head, everything else as dsv3_ref
    "dsv3_ref_stale": DSV3Config(block_size=512, batch_size=32, mtp_heads=1),
    "dsv3_tiny": DSV3Config(vocab_size=512, block_size=128, dim=256, n_layers=2, n_heads=4, attention="mla",
                            kv_lora_rank=64, qk_nope_dim=32, qk_rope_dim=32, v_head_dim=64, n_experts=8, top_k=2,
                            n_shared=1, expert_hidden=128, n_dense_layers=1, dense_hidden=512, pos_emb="none",
                            bias_in_weights=False, balance_stat="counts", final_scale=False, norm_eps=1e-6,
                            dropout=0.0, attn_dropout=0.0, mtp_heads=1),
    # DeepSeek-V2-Lite-like widths (D2048, 16 heads, kv_lora 512, 64 routed experts top-6 +
    # 2 shared, hidden 1408, 1 dense layer), qk = 64 nope + 64 rope = 128 = v so attention
    # stays on the hd-128 flash kernel. Depth is a bench knob.
    "dsv3_style": DSV3Config(vocab_size=102400, block_size=4096, dim=2048, n_layers=12, n_heads=16,
                             attention="mla", q_lora_rank=0, kv_lora_rank=512, qk_nope_dim=64, qk_rope_dim=64,
                             v_head_dim=128, n_experts=64, top_k=6, n_shared=2, expert_hidden=1408,
                             n_dense_layers=1, dense_hidden=10944, pos_emb="none", bias_in_weights=False,
                             balance_stat="counts", final_scale=False, norm_eps=1e-6, dropout=0.0,
                             attn_dropout=0.0, mtp_heads=1, batch_size=1),
    # DeepSeek-V3 (arXiv 2412.19437) widths: D7168, 128 heads, q_lora 1536, kv_lora 512,
    # qk 128 nope + 64 rope = 192 and v 128 (native (192, 128) flash kernels, no padding), 256 routed
    # experts top-8 + 1 shared of hidden 2048, 3 dense layers of 18432, V 129280. 61 layers is
    # the model card; benches override depth and (for 1 GPU) the expert count.
    "dsv3_v3": DSV3Config(vocab_size=129280, block_size=4096, dim=7168, n_layers=61, n_heads=128,
                          attention="mla", q_lora_rank=1536, kv_lora_rank=512, qk_nope_dim=128,
                          qk_rope_dim=64, v_head_dim=128, n_experts=256, top_k=8, n_shared=1,
                          expert_hidden=2048, n_dense_layers=3, dense_hidden=18432, pos_emb="none",
                          bias_in_weights=False, balance_stat="counts", final_scale=False, norm_eps=1e-6,
                          dropout=0.0, attn_dropout=0.0, mtp_heads=1, batch_size=1),
}


def config(name, **kw):
    return replace(PRESETS[name], **kw)


def _pad8(n):
    return (n + 7) // 8 * 8


def sinusoidal_pe(block_size, dim, device=None):
    """deepseekv3.ipynb:836-842 (fp32, [1, T, D])."""
    pe = torch.zeros(block_size, dim, device=device)
    pos = torch.arange(0, block_size, dtype=torch.float, device=device).unsqueeze(1)
    div = torch.exp(torch.arange(0, dim, 2, dtype=torch.float, device=device) * (-math.log(10000.0) / dim))
    pe[:, 0::2] = torch.sin(pos * div)
    pe[:, 1::2] = torch.cos(pos * div)
    return pe.unsqueeze(0)


# =============================================================================== attention
class RefLatentAttention(tnn.Module):
    """MHLA of the notebook (:1135-1265) with its per-head parameters stacked."""

    def __init__(self, c: DSV3Config, **fk):
        super().__init__()
        H, D, L, hs = c.n_heads, c.dim, c.latent_dim, c.head_size
        self.c = c
        self.wdkv = tnn.Parameter(torch.empty(H, L, D, **fk))   # heads.h.W_dkv
        self.wk = tnn.Parameter(torch.empty(H, hs, L, **fk))    # heads.h.W_k
        self.wv = tnn.Parameter(torch.empty(H, hs, L, **fk))    # heads.h.W_v
        self.wq = tnn.Parameter(torch.empty(H, hs, D, **fk))    # heads.h.query
        self.wo = tnn.Parameter(torch.empty(D, D, **fk))        # linear

    def params(self):
        return [self.wdkv, self.wk, self.wv, self.wq, self.wo]

    def latent0(self, xn):
        return linear(xn, self.wdkv[0])                          # [B, T, latent]

    def forward(self, xn, L0, cache=None, pos=0):
        c = self.c
        B, T, D = xn.shape
        H, L, hs = c.n_heads, c.latent_dim, c.head_size
        # absorbed query weights A_h = query_h^T W_k_h  -> one [D, H*L] GEMM
        A = torch.einsum("hsd,hsl->hld", self.wq, self.wk).reshape(H * L, D)
        q = linear(xn, A).view(B, T, H, L)
        kv = L0.unsqueeze(2)                                     # one shared "head": k = v = L0
        if cache is not None:
            kv = cache[:, :pos + T].unsqueeze(2)
        p = c.attn_dropout if self.training else 0.0
        o = attention_dropout(q, kv, kv, causal=True, scale=hs ** -0.5, p=p, training=self.training)
        o = torch.einsum("bthl,hsl->bths", o, self.wv).reshape(B, T, H * hs)
        return dropout(linear(o, self.wo), p, self.training)


class MLA(tnn.Module):
    """Paper MLA: c_kv = norm(W_dkv x)[:kv_lora], k_rope = RoPE(W_dkv x)[kv_lora:] shared by all
    heads; [k_nope | v] = W_ukv c_kv; q = W_uq norm(W_dq x) (or W_q x)."""

    def __init__(self, c: DSV3Config, **fk):
        super().__init__()
        H, D = c.n_heads, c.dim
        self.c = c
        qd = H * c.qk_head_dim
        if c.q_lora_rank:
            self.wdq = tnn.Parameter(torch.empty(c.q_lora_rank, D, **fk))
            self.q_norm = tnn.Parameter(torch.ones(c.q_lora_rank, **fk))
            self.wuq = tnn.Parameter(torch.empty(qd, c.q_lora_rank, **fk))
        else:
            self.wq = tnn.Parameter(torch.empty(qd, D, **fk))
        self.wdkv = tnn.Parameter(torch.empty(c.kv_lora_rank + c.qk_rope_dim, D, **fk))
        self.kv_norm = tnn.Parameter(torch.ones(c.kv_lora_rank, **fk))
        self.wukv = tnn.Parameter(torch.empty(H * (c.qk_nope_dim + c.v_head_dim), c.kv_lora_rank, **fk))
        self.wo = tnn.Parameter(torch.empty(D, H * c.v_head_dim, **fk))

    def params(self):
        return list(self.parameters())

    def _q(self, xn):
        c = self.c
        if c.q_lora_rank:
            return linear(rms_norm(linear(xn, self.wdq, fp8=c.fp8_linears), self.q_norm, c.norm_eps), self.wuq,
                          fp8=c.fp8_linears)
        return linear(xn, self.wq, fp8=c.fp8_linears)

    def _rope(self, x, pos):
        from ..infer.graph import DecodeState
        if isinstance(pos, DecodeState):   # device positions: graph-capture safe
            return apply_rope(x, self.c.rope_theta, positions=pos.positions.expand(x.shape[0], x.shape[1]),
                              max_len=pos.max_len)
        return apply_rope(x, self.c.rope_theta, pos)

    def _latent(self, xn, pos):
        c = self.c
        B, T, _ = xn.shape
        ckr = linear(xn, self.wdkv, fp8=c.fp8_linears)
        ckv = rms_norm(ckr[..., :c.kv_lora_rank].contiguous(), self.kv_norm, c.norm_eps)
        kr = self._rope(ckr[..., c.kv_lora_rank:].reshape(B, T, 1, c.qk_rope_dim), pos)
        return ckv, kr

    def forward(self, xn, L0=None, cache=None, pos=0):
        c = self.c
        B, T, _ = xn.shape
        H, dn, dr, dv = c.n_heads, c.qk_nope_dim, c.qk_rope_dim, c.v_head_dim
        scale = 1.0 / math.sqrt(dn + dr)
        q = self._q(xn).view(B, T, H, dn + dr)
        if cache is None and isinstance(pos, int):
            # training / prefill: head assembly fused around the flash kernels (ops.mla_attention)
            ckv_in, kr = split_last(linear(xn, self.wdkv, fp8=c.fp8_linears), c.kv_lora_rank)
            ckv = rms_norm(ckv_in, self.kv_norm, c.norm_eps)
            kv = linear(ckv, self.wukv, fp8=c.fp8_linears).view(B, T, H, dn + dv)
            o = mla_attention(q, kv, kr.view(B, T, 1, dr), dn, scale, c.rope_theta, pos)
            return linear(o.reshape(B, T, H * dv), self.wo, fp8=c.fp8_linears)
        qr = self._rope(q[..., dn:], pos)
        ckv, kr = self._latent(xn, pos)
        if cache is not None:
            return self._decode(q[..., :dn], qr, ckv, kr, cache, pos, scale)
        kv = linear(ckv, self.wukv, fp8=c.fp8_linears).view(B, T, H, dn + dv)
        qf = torch.cat([q[..., :dn], qr], dim=-1)
        k = torch.cat([kv[..., :dn], kr.expand(B, T, H, dr)], dim=-1)
        v = kv[..., dn:]
        # the flash kernels take (q/k, v) head dims (64,64) / (128,128) / (192,128) -- V3's MLA
        # heads -- directly, reading v as a strided view of the up-projection output
        o = flash_attention(qf, k, v, causal=True, scale=scale)
        return linear(o.reshape(B, T, H * dv), self.wo, fp8=c.fp8_linears)

    def _decode(self, qn, qr, ckv, kr, cache, pos, scale):
        """Latent-space attention over the compressed cache (W_uk absorbed into q, W_uv applied
        after): per token the cache holds kv_lora + rope values instead of 2*H*hd. The scores
        and the latent output come from one HIP launch (csrc/kernels/mla_decode.hip: 576-wide
        single-head MQA, split-K flash-decoding); the absorptions are two batched GEMMs.
        ``pos`` is an int (eager) or a DecodeState (HIP-graph decode: write row and valid
        length on the device)."""
        from ..infer.graph import DecodeState
        from ..ops.attention import mla_decode_attention
        c = self.c
        B, T, H, dn = qn.shape
        C, dv = c.kv_lora_rank, c.v_head_dim
        cc, cr = cache
        if isinstance(pos, DecodeState):
            cc.index_copy_(1, pos.index, ckv.to(cc.dtype))
            cr.index_copy_(1, pos.index, kr.reshape(B, T, -1).to(cr.dtype))
            kv_len, kv_len_t = 0, pos.kv_len
        else:
            cc[:, pos:pos + T] = ckv.to(cc.dtype)
            cr[:, pos:pos + T] = kr.reshape(B, T, -1).to(cr.dtype)
            kv_len, kv_len_t = pos + T, None
        w = self.wukv.view(H, dn + dv, C)
        # q_abs[b, t, h] = q_nope[b, t, h] @ W_uk[h]  (one batched GEMM over heads)
        q_abs = torch.bmm(qn.permute(2, 0, 1, 3).reshape(H, B * T, dn), w[:, :dn]).view(H, B, T, C)
        o_lat = mla_decode_attention(q_abs.permute(1, 2, 0, 3), qr, cc, cr, scale, kv_len, kv_len_t)
        o = torch.bmm(o_lat.permute(2, 0, 1, 3).reshape(H, B * T, C), w[:, dn:].transpose(1, 2))
        return linear(o.view(H, B, T, dv).permute(1, 2, 0, 3).reshape(B, T, H * dv), self.wo)


# =============================================================================== FFN / MoE
class DenseFFN(tnn.Module):
    def __init__(self, D, F, fp8=False, **fk):
        super().__init__()
        self.F, self.Fp, self.fp8 = F, _pad8(F), fp8
        self.w13 = tnn.Parameter(torch.zeros(2 * self.Fp, D, **fk))    # [gate ; up], padded rows zero
        self.w2 = tnn.Parameter(torch.zeros(D, self.Fp, **fk))

    @torch.no_grad()
    def reset_parameters(self, std, g):
        F, Fp = self.F, self.Fp
        self.w13.zero_()
        self.w2.zero_()
        self.w13[:F].normal_(0, std, generator=g)
        self.w13[Fp:Fp + F].normal_(0, std, generator=g)
        self.w2[:, :F].normal_(0, std, generator=g)

    def forward(self, x):
        return linear(glu(linear(x, self.w13, fp8=self.fp8), "silu"), self.w2, fp8=self.fp8)


class _PairReady:
    """grad_ready_cb for two micro-batches in one backward: a layer's gradients are complete
    (the DP bucket may launch) only when BOTH micro-batches' backward passed its marker."""

    def __init__(self, cb):
        self.cb, self.seen = cb, {}

    def __call__(self, key):
        n = self.seen.get(key, 0) + 1
        if n == 2:
            self.seen.pop(key, None)
            self.cb(key)
        else:
            self.seen[key] = n


class MoE(tnn.Module):
    """DeepSeekMoE: shared experts + top-k routed experts with aux-free load balancing.
    Under EP (``ep_group`` of size P) this rank holds experts [r*E/P, (r+1)*E/P)."""

    def __init__(self, c: DSV3Config, ep_group=None, **fk):
        """One forward is four stages (expert_parallel.EPStage): prepare (routing, count exchange,
        fp8 payload) -> shared expert -> dispatch (the one host sync; the all-to-all starts right
        after the payload, so the shared expert queued before the sync runs beside it) -> experts +
        combine. DeepSeekV3.forward_pair interleaves the stages of two micro-batches so every
        exchange also overlaps the other micro-batch's attention / experts. (Splitting one layer's
        tokens into chunks instead cost grouped-GEMM efficiency -- fewer rows per expert -- and
        was removed in round 4.)"""
        super().__init__()
        from ..parallel.expert_parallel import ep_rank_size
        self.c = c
        self.ep_group = ep_group
        self.ep_rank, self.ep = ep_rank_size(ep_group)
        assert c.n_experts % self.ep == 0
        El = c.n_experts // self.ep
        D, F = c.dim, c.ffn_hidden
        self.F, self.Fp = F, _pad8(F)
        self.gate = tnn.Parameter(torch.empty(c.n_experts, D, **fk))
        # noisy top-k gating (deepseekv3.ipynb:1026-1027): a second router GEMM whose softplus
        # scales the per-(token, expert) Gaussian noise added to the gate logits
        self.noise = tnn.Parameter(torch.empty(c.n_experts, D, **fk)) if c.noisy_topk else None
        self.w13 = tnn.Parameter(torch.zeros(El, 2 * self.Fp, D, **fk))
        self.w2 = tnn.Parameter(torch.zeros(El, D, self.Fp, **fk))
        self.w13.expert_parallel = self.ep > 1
        self.w2.expert_parallel = self.ep > 1
        self.shared = DenseFFN(D, F * c.n_shared, fp8=c.fp8_linears, **fk) if c.n_shared else None
        self.register_buffer("routing_bias", torch.zeros(c.n_experts, device=fk.get("device")))
        self.balance_group = None      # DP group for the counts all-reduce (set by the trainer)
        self.last_counts = None
        self._pending_bias = []        # (work, load): bias updates whose counts all-reduce is in flight
        self.cap_state = SimpleNamespace(rows=None)   # capacity-mode EP: this layer's block rows
        # EP dispatch override (DeepSeekV3.ep_dispatch): None -> DSV3Config.ep_capacity; "exact" ->
        # split-size dispatch; "bound" -> host-sync-free blocks at the exact per-peer bound (cannot
        # overflow, no flag: HIP-graph decode)
        self.dispatch_mode = None

    @torch.no_grad()
    def reset_parameters(self, std, g):
        F, Fp = self.F, self.Fp
        self.gate.normal_(0, std, generator=g)
        if self.noise is not None:
            self.noise.normal_(0, std, generator=g)
        # under EP draw all E experts exactly as the unsharded model does and keep this rank's
        # slice: every EP rank then holds distinct experts, and rank r's shard equals
        # shard_experts(unsharded init, r, P) (a per-rank E/P draw from the shared generator
        # sequence would give every rank the same experts)
        w13 = self.w13 if self.ep == 1 else self.w13.new_zeros((self.c.n_experts,) + tuple(self.w13.shape[1:]))
        w2 = self.w2 if self.ep == 1 else self.w2.new_zeros((self.c.n_experts,) + tuple(self.w2.shape[1:]))
        w13.zero_()
        w2.zero_()
        w13[:, :F].normal_(0, std, generator=g)
        w13[:, Fp:Fp + F].normal_(0, std, generator=g)
        w2[:, :, :F].normal_(0, std, generator=g)
        if self.ep > 1:
            El = self.w13.shape[0]
            self.w13.copy_(w13[self.ep_rank * El:(self.ep_rank + 1) * El])
            self.w2.copy_(w2[self.ep_rank * El:(self.ep_rank + 1) * El])
        if self.shared is not None:
            self.shared.reset_parameters(std, g)

    def expert_params(self):
        return [self.w13, self.w2]

    def _logits(self, x2):
        logits = router_logits(x2, self.gate)
        if self.noise is not None:
            # deepseekv3.ipynb:1037-1039 -- applied in eval too, exactly as the reference does;
            # the fp32 logits keep the noise draw at full precision
            logits = logits + torch.nn.functional.softplus(router_logits(x2, self.noise)) * torch.randn_like(logits)
        return logits

    def _fp8(self, x2):
        return self.c.moe_fp8 and x2.is_cuda and self.Fp % 16 == 0

    # ---- stages (expert_parallel.EPStage); forward() runs them in order, forward_pair interleaves
    def stage_prepare(self, x2):
        from ..parallel.expert_parallel import ep_stage_prepare
        c = self.c
        self.finish_pending()                   # last step's bias updates before this routing
        idx, w = route(self._logits(x2), c.top_k, self.routing_bias if c.aux_free else None, c.bias_in_weights)
        st = ep_stage_prepare(x2, idx, w, c.n_experts, self.ep_group, self._fp8(x2), self.w13,
                              capacity=self._capacity(), cap_state=self.cap_state)
        st.x2, st.idx, st.sh = x2, idx, None
        if c.aux_free and self.training:
            # the bias moves right after this routing (the reference updates it after every
            # forward, deepseekv3.ipynb:1082-1086): under forward_pair micro-batch 1 then routes
            # this layer with micro-batch 0's update applied, exactly as two forward() calls do
            self._update_bias(idx, w, st.prep.plan)
        return st

    def _capacity(self):
        if self.dispatch_mode == "exact":
            return 0.0
        if self.dispatch_mode == "bound":
            return math.inf
        return self.c.ep_capacity

    def stage_shared(self, st):
        if self.shared is not None:
            st.sh = self.shared(st.x2)

    def stage_dispatch(self, st):
        from ..parallel.expert_parallel import ep_stage_dispatch
        ep_stage_dispatch(st)

    def stage_experts(self, st):
        from ..parallel.expert_parallel import ep_stage_experts
        ep_stage_experts(st, self.w13, self.w2)

    def stage_finish(self, st):
        from ..parallel.expert_parallel import ep_stage_finish
        plan = st.prep.plan
        y = ep_stage_finish(st)
        if st.sh is not None:
            y = y + st.sh
        self.last_counts = plan.counts
        st.x2 = st.sh = None
        return y

    def forward(self, x):
        B, T, D = x.shape
        x2 = x.reshape(-1, D)
        st = self.stage_prepare(x2)
        self.stage_shared(st)                   # queued before the dispatch's host sync
        self.stage_dispatch(st)
        self.stage_experts(st)
        return self.stage_finish(st).view(B, T, D)

    @torch.no_grad()
    def _update_bias(self, idx, w, plan):
        """Aux-loss-free balancing (deepseekv3.ipynb:1082-1086): bias += rate * sign(mean - load).
        "counts": the load is summed over the DP group with an ASYNC all-reduce, applied by
        finish_pending() -- at the layer's next routing, or before a checkpoint / eval -- so the
        forward never blocks on it; the update still lands before the next use of the bias."""
        c = self.c
        if c.balance_stat == "soft":            # deepseekv3.ipynb:1082-1086
            load = torch.zeros(idx.shape[0], c.n_experts, device=w.device).scatter_(1, idx.long(), w).sum(0)
            self._apply_bias(load)
            return
        load = (plan.counts if plan is not None else
                torch.bincount(idx.reshape(-1).long(), minlength=c.n_experts)).float()
        grp = self.balance_group
        from ..parallel.dist import is_dist
        if grp is not None or is_dist():
            self._pending_bias.append((dist.all_reduce(load, group=grp, async_op=True), load))
        else:
            self._apply_bias(load)

    @torch.no_grad()
    def _apply_bias(self, load):
        err = load.mean() - load
        self.routing_bias.add_(self.c.bias_update_rate * torch.sign(err))

    @torch.no_grad()
    def finish_pending(self):
        """Apply the bias updates whose load all-reduce was in flight (in issue order)."""
        while self._pending_bias:
            work, load = self._pending_bias.pop(0)
            work.wait()
            self._apply_bias(load)


# =============================================================================== layers
class DSV3Layer(tnn.Module):
    def __init__(self, c: DSV3Config, dense: bool, ep_group=None, **fk):
        super().__init__()
        self.c = c
        self.attn_norm = tnn.Parameter(torch.ones(c.dim, **fk))
        self.ffn_norm = tnn.Parameter(torch.ones(c.dim, **fk))
        self.attn = RefLatentAttention(c, **fk) if c.attention == "ref" else MLA(c, **fk)
        if dense:
            self.ffn = DenseFFN(c.dim, c.dense_hidden or c.ffn_hidden, fp8=c.fp8_linears, **fk)
        else:
            self.ffn = MoE(c, ep_group, **fk)

    @torch.no_grad()
    def reset_parameters(self, g):
        std = self.c.init_std
        for n, p in self.attn.named_parameters():
            if n.endswith("norm"):
                p.fill_(1.0)
            else:
                p.normal_(0, std, generator=g)
        self.ffn.reset_parameters(std, g)
        self.attn_norm.fill_(1.0)
        self.ffn_norm.fill_(1.0)

    def dense_params(self):
        ex = {id(p) for p in self.expert_params()}
        return [p for p in self.parameters() if id(p) not in ex]

    def expert_params(self):
        return self.ffn.expert_params() if isinstance(self.ffn, MoE) else []

    def attn_part(self, res, delta, L0=None, cache=None, pos=0):
        """norm -> attention -> residual -> FFN norm: returns (h2, n2, L0), the FFN's input n2."""
        c = self.c
        if res is None:
            xn, h = rms_norm(delta, self.attn_norm, c.norm_eps), delta
        else:
            xn, h = rms_norm(delta, self.attn_norm, c.norm_eps, residual=res)
        if c.attention == "ref" and L0 is None:
            L0 = self.attn.latent0(xn)                 # the only latent anybody attends to (Q1)
            if cache is not None:
                cache[:, pos:pos + xn.shape[1]] = L0.to(cache.dtype)
        a = self.attn(xn, L0, cache, pos)
        n2, h2 = rms_norm(a, self.ffn_norm, c.norm_eps, residual=h)
        return h2, n2, L0

    def forward_split(self, res, delta, L0=None, cache=None, pos=0):
        """Pre-norm layer on a split residual stream (as LlamaBlock): the input is res + delta and
        the output (h, f) means h + f; both residual adds happen inside the fused RMSNorms, so
        neither the forward nor the backward launches a separate add."""
        h2, n2, L0 = self.attn_part(res, delta, L0, cache, pos)
        return h2, self.ffn(n2), L0

    def forward(self, x, L0=None, cache=None, pos=0):
        h, f, L0 = self.forward_split(None, x, L0, cache, pos)
        return h + f, L0


class DeepSeekV3(tnn.Module):
    def __init__(self, c: DSV3Config, device=None, dtype=torch.float32, seed: int = 0, ep_group=None):
        super().__init__()
        self.c = c
        fk = dict(device=device, dtype=dtype)
        self.embed = tnn.Parameter(torch.empty(c.vocab_size, c.dim, **fk))     # tied LM head
        self.layers = tnn.ModuleList([DSV3Layer(c, i < c.n_dense_layers, ep_group, **fk)
                                      for i in range(c.n_layers)])
        self.norm_f = tnn.Parameter(torch.ones(c.dim, **fk))
        # MTP (deepseekv3.ipynb:1466-1485): norm1 on the shifted-token embedding, norm2 on the
        # previous depth's hidden state, linear_layer [2D -> D], one decoder layer per depth.
        D = c.dim
        self.mtp_norm1_w = tnn.Parameter(torch.ones(D, **fk))
        self.mtp_norm1_b = tnn.Parameter(torch.zeros(D, **fk))
        self.mtp_norm2_w = tnn.Parameter(torch.ones(D, **fk))
        self.mtp_norm2_b = tnn.Parameter(torch.zeros(D, **fk))
        self.mtp_proj = tnn.Parameter(torch.empty(D, 2 * D, **fk))
        self.mtp_heads = tnn.ParameterList([tnn.Parameter(torch.empty(D, D, **fk)) for _ in range(c.mtp_heads)])
        self.mtp_layers = tnn.ModuleList([DSV3Layer(c, False, ep_group, **fk) for _ in range(c.mtp_heads)])
        if c.pos_emb == "sinusoidal":
            self.register_buffer("pe", sinusoidal_pe(c.block_size, c.dim, device=device).to(dtype))
        else:
            self.pe = None
        self.grad_ready_cb = None
        self.param_wait_cb = None
        self.reset_parameters(seed)

    @torch.no_grad()
    def reset_parameters(self, seed=0):
        g = torch.Generator(device=self.embed.device).manual_seed(seed)
        std = self.c.init_std
        self.embed.normal_(0, std, generator=g)
        self.norm_f.fill_(1.0)
        for l in list(self.layers) + list(self.mtp_layers):
            l.reset_parameters(g)
        self.mtp_proj.normal_(0, std, generator=g)
        for h in self.mtp_heads:
            h.normal_(0, std, generator=g)

    def moe_layers(self) -> List[MoE]:
        return [l.ffn for l in list(self.layers) + list(self.mtp_layers) if isinstance(l.ffn, MoE)]

    def pair_overlaps(self):
        """True when forward_pair hides something (expert-parallel exchanges). At EP 1 the pair
        only keeps two micro-batches' activations alive, so the Trainer runs them one by one."""
        return bool(self.training and torch.is_grad_enabled() and any(m.ep > 1 for m in self.moe_layers()))

    def param_groups(self):
        """Buckets: [embed], per-layer dense params, [head + MTP dense], then the expert
        buckets (kept apart so DP skips them under EP)."""
        head = [self.norm_f, self.mtp_norm1_w, self.mtp_norm1_b, self.mtp_norm2_w, self.mtp_norm2_b,
                self.mtp_proj] + list(self.mtp_heads)
        for l in self.mtp_layers:
            head += l.dense_params()
        groups = [[self.embed]] + [l.dense_params() for l in self.layers] + [head]
        return groups + [l.expert_params() for l in list(self.layers) + list(self.mtp_layers) if l.expert_params()]

    # ------------------------------------------------------------------ forward
    def _embed(self, ids, pos=0):
        T = ids.shape[1]
        pe = None if self.pe is None else self.pe[0, pos:pos + T]
        return embedding(self.embed, ids, pe)

    def _expert_buckets(self):
        """layer index (main layers, then MTP layers) -> index of its expert group in
        param_groups() (the index param_wait_cb receives; FlatParams.group_waiter maps it to the
        bucket that group landed in). The overlapped optimizer updates the expert buckets after
        every dense bucket, so each MoE layer waits for its own before it reads its experts."""
        eb = getattr(self, "_ebk", None)
        if eb is None:
            eb, k = {}, len(self.layers) + 2
            for j, l in enumerate(list(self.layers) + list(self.mtp_layers)):
                if l.expert_params():
                    eb[j] = k
                    k += 1
            self._ebk = eb
        return eb

    def hidden(self, ids, caches=None, pos=0):
        c = self.c
        wait = self.param_wait_cb or (lambda i: None)
        eb = self._expert_buckets() if self.param_wait_cb is not None else {}
        wait(0)
        x = self._embed(ids, pos)
        x0 = x
        L0 = None
        cb = self.grad_ready_cb
        res, delta = None, x
        for i, layer in enumerate(self.layers):
            wait(i + 1)
            if i in eb:
                wait(eb[i])
            delta = mark_ready(delta, cb, i + 1)
            if c.attention == "ref":
                res, delta, L0 = layer.forward_split(res, delta, L0, None if caches is None else caches[0], pos)
            else:
                res, delta, _ = layer.forward_split(res, delta, None, None if caches is None else caches[i], pos)
        wait(len(self.layers) + 1)
        delta = mark_ready(delta, cb, len(self.layers) + 1)
        return self._final(res, delta), x0

    def hidden_pair(self, ids0, ids1):
        """Two micro-batches through the main layers, interleaved so every expert-parallel
        all-to-all of one runs under the other's compute (DualPipe-style micro-batch overlap; no
        layer's tokens are split, so every grouped GEMM keeps its full rows per expert). Per MoE
        layer l, host order (each exchange is issued right after its producer, expert_parallel
        EPStage):

            finish combine_0(l-1) | attn_0 | prepare_0 | shared_0 | dispatch_0 (host sync)
            finish combine_1(l-1) | attn_1 | prepare_1 | shared_1 | dispatch_1 (host sync)
            experts_0 + combine_0 | experts_1 + combine_1

        so dispatch_0 overlaps shared_0 and attn_1, dispatch_1 overlaps shared_1 and experts_0,
        combine_0 overlaps experts_1 and combine_1 overlaps the next layer's attn_0; autograd
        replays the nodes in reverse creation order, which interleaves the backward the same way.
        Returns (final, [x0_0, x0_1]): final(m) finishes micro-batch m (its last combine, final
        norm) and returns its hidden state; call final(0), use it, then final(1), so micro-batch
        1's last combine overlaps micro-batch 0's head."""
        c = self.c
        wait = self.param_wait_cb or (lambda i: None)
        eb = self._expert_buckets() if self.param_wait_cb is not None else {}
        wait(0)
        xs = [self._embed(ids0), self._embed(ids1)]
        x0s = list(xs)
        cb = _PairReady(self.grad_ready_cb) if self.grad_ready_cb is not None else None
        S = [{"res": None, "delta": xs[0], "L0": None}, {"res": None, "delta": xs[1], "L0": None}]
        pend = [None, None]

        def settle(m):
            if pend[m] is not None:
                moe, st = pend[m]
                S[m]["delta"] = moe.stage_finish(st).view(st.shape)
                pend[m] = None

        for i, layer in enumerate(self.layers):
            wait(i + 1)
            if i in eb:
                wait(eb[i])
            is_moe = isinstance(layer.ffn, MoE)
            sts = [None, None]
            for m in (0, 1):
                settle(m)
                sm = S[m]
                sm["delta"] = mark_ready(sm["delta"], cb, i + 1)
                h2, n2, L0 = layer.attn_part(sm["res"], sm["delta"], sm["L0"] if c.attention == "ref" else None)
                sm["res"] = h2
                if c.attention == "ref":
                    sm["L0"] = L0
                if not is_moe:
                    sm["delta"] = layer.ffn(n2)
                    continue
                st = layer.ffn.stage_prepare(n2.reshape(-1, n2.shape[-1]))
                st.shape = n2.shape
                layer.ffn.stage_shared(st)        # queued before the dispatch's host sync
                layer.ffn.stage_dispatch(st)
                sts[m] = st
            if is_moe:
                layer.ffn.stage_experts(sts[0])
                layer.ffn.stage_experts(sts[1])
                pend = [(layer.ffn, sts[0]), (layer.ffn, sts[1])]
        wait(len(self.layers) + 1)

        def final(m):
            """micro-batch m's last combine, then its final norm: called for m = 0 before m = 1,
            with micro-batch 0's head in between, micro-batch 1's last combine overlaps it"""
            settle(m)
            delta = mark_ready(S[m]["delta"], cb, len(self.layers) + 1)
            return self._final(S[m]["res"], delta)
        return final, x0s

    def _final(self, res, delta):
        c = self.c
        if (c.dropout > 0 and self.training) or c.final_scale or res is None:
            x = delta if res is None else res + delta
            x = dropout(x, c.dropout, self.training)
            if c.final_scale:
                x = x * (2.0 * c.n_layers ** -0.5)
            return rms_norm(x, self.norm_f, c.norm_eps)
        n, _ = rms_norm(delta, self.norm_f, c.norm_eps, residual=res)
        return n

    # ---- capacity-mode EP (DSV3Config.ep_capacity > 0): no host sync inside the layers; one read
    # of the overflow flags per forward. On overflow the forward re-runs with every layer's block
    # rows set from the load it saw (x margin); a layer downstream of an overflow saw perturbed
    # inputs, so that re-run can overflow again -- then the last attempt takes the exact split-size
    # dispatch (one host sync per layer), which cannot overflow. Training never stops on capacity.
    _CAP_ATTEMPTS = 2

    def _capacity_run(self, fn, *args):
        if not self.c.ep_capacity > 0:
            return fn(*args)
        from ..parallel.expert_parallel import capacity_overflowed
        capacity_overflowed()                   # flags of work outside this forward are not ours
        snap = self._routing_snapshot()
        for _ in range(self._CAP_ATTEMPTS):
            out = fn(*args)
            if not capacity_overflowed():
                return out
            self._routing_restore(snap)         # the failed attempt's graph is dropped with `out`
        with self.ep_dispatch("exact"):
            return fn(*args)

    @contextlib.contextmanager
    def ep_dispatch(self, mode):
        """Every MoE layer on EP dispatch ``mode`` ("exact" | "bound", MoE.dispatch_mode) for the duration."""
        layers = list(self.moe_layers())
        prev = [m.dispatch_mode for m in layers]
        for m in layers:
            m.dispatch_mode = mode
        try:
            yield
        finally:
            for m, p in zip(layers, prev):
                m.dispatch_mode = p

    def _routing_snapshot(self):
        # outstanding bias updates of the previous step land first (each layer's routing would
        # apply them anyway), so the snapshot is the bias every attempt starts from
        self.finish_pending_updates()
        rng = (torch.get_rng_state(), torch.cuda.get_rng_state() if torch.cuda.is_available() and
               self.embed.is_cuda else None)
        return [(m, m.routing_bias.clone()) for m in self.moe_layers()], rng

    @torch.no_grad()
    def _routing_restore(self, snap):
        layers, (cpu_rng, gpu_rng) = snap
        for m, bias in layers:
            while m._pending_bias:                    # the failed attempt's async load all-reduces
                work, _ = m._pending_bias.pop()
                work.wait()
            m.routing_bias.copy_(bias)
        torch.set_rng_state(cpu_rng)
        if gpu_rng is not None:
            torch.cuda.set_rng_state(gpu_rng)

    def forward_pair(self, ids0, targets0, ids1, targets1):
        """loss(micro-batch 0) + loss(micro-batch 1) with the two run layer-interleaved
        (hidden_pair): the same values and gradients as two forward() calls, with each MoE
        layer's all-to-alls overlapped by the other micro-batch's compute. Training only.
        Aux-free balancing keeps the sequential semantics: each MoE layer moves its routing bias
        right after micro-batch 0's routing (MoE.stage_prepare), before micro-batch 1 routes."""
        return self._capacity_run(self._forward_pair, ids0, targets0, ids1, targets1)

    def _forward_pair(self, ids0, targets0, ids1, targets1):
        final, x0s = self.hidden_pair(ids0, ids1)
        D = self.c.dim
        loss = None
        for m, (x0, t) in enumerate(zip(x0s, (targets0, targets1))):
            n = final(m)
            l = linear_cross_entropy(n.reshape(-1, D), self.embed, t.reshape(-1))
            if self.c.mtp_heads and self.training:
                l = l + self.mtp_loss(n, x0, t)
            loss = l if loss is None else loss + l
        return loss

    def finish_pending_updates(self):
        """Apply routing-bias updates whose DP all-reduce is still in flight (before a checkpoint,
        an evaluation, or reading the buffers)."""
        for m in self.moe_layers():
            m.finish_pending()

    def logits(self, n):
        return linear(n, self.embed)

    def forward(self, ids, targets=None):
        return self._capacity_run(self._forward, ids, targets)

    def _forward(self, ids, targets=None):
        n, x0 = self.hidden(ids)
        if targets is None:
            return self.logits(n)
        D = self.c.dim
        loss = linear_cross_entropy(n.reshape(-1, D), self.embed, targets.reshape(-1))
        if self.c.mtp_heads and self.training:
            loss = loss + self.mtp_loss(n, x0, targets)
        return loss

    def mtp_loss(self, h, emb, targets):
        """DeepSeek-V3 MTP: depth k combines h^{k-1}_i with Emb(t_{i+k}) and predicts t_{i+k+1}
        through the shared head; loss = lambda * mean_k CE_k (targets[:, i] = t_{i+1})."""
        c = self.c
        B, T, D = h.shape
        tot = 0.0
        wait = self.param_wait_cb or (lambda i: None)
        eb = self._expert_buckets() if self.param_wait_cb is not None else {}
        for k, layer in enumerate(self.mtp_layers, start=1):
            if T - k <= 0:
                break
            if len(self.layers) + k - 1 in eb:
                wait(eb[len(self.layers) + k - 1])
            e = layer_norm(emb[:, k:], self.mtp_norm1_w, self.mtp_norm1_b, 1e-6)
            hp = layer_norm(h[:, :T - k], self.mtp_norm2_w, self.mtp_norm2_b, 1e-6)
            hk = linear(torch.cat([e, hp], dim=-1), self.mtp_proj)
            hk, _ = layer(hk)
            hk = rms_norm(hk, self.norm_f, c.norm_eps)
            tgt = targets[:, k:]
            tot = tot + linear_cross_entropy(hk.reshape(-1, D), self.embed, tgt.reshape(-1))
            h = hk
        return c.mtp_lambda * tot / max(1, len(self.mtp_layers))

    # ---------------------------------------------------------------- inference
    def new_cache(self, B, Tmax):
        c = self.c
        dev, dt = self.embed.device, self.embed.dtype
        if c.attention == "ref":
            return [torch.zeros(B, Tmax, c.latent_dim, device=dev, dtype=dt)]
        return [(torch.zeros(B, Tmax, c.kv_lora_rank, device=dev, dtype=dt),
                 torch.zeros(B, Tmax, c.qk_rope_dim, device=dev, dtype=dt)) for _ in self.layers]

    @property
    def max_context(self):
        return self.c.block_size if self.c.pos_emb == "sinusoidal" else None

    def step(self, ids, cache, pos):
        """Write ids' latents at cache rows [pos, pos+T), return the last position's logits [B, V].
        Always the exact EP dispatch: capacity mode's overflow re-run exists only for forward()."""
        with self.ep_dispatch("exact"):
            n, _ = self.hidden(ids, cache, pos)
        return self.logits(n[:, -1:]).float()[:, -1]

    def step_graph(self, ids, cache, state):
        """One-token decode step with every position on the device (HIP-graph capturable,
        infer/graph.py GraphDecoder): RoPE at ``state.positions``, latent cache rows written at
        ``state.index``, the MLA decode kernel reads the valid length from ``state.kv_len``; the
        MoE routing / permutation / grouped GEMMs never read device values on the host."""
        if self.c.attention == "ref":
            raise NotImplementedError("graph decode needs the paper MLA (the ref preset adds sinusoidal PE by position)")
        # EP > 1: fixed blocks at the exact per-peer bound (no host read, no overflow, no flag)
        with self.ep_dispatch("bound"):
            n, _ = self.hidden(ids, cache, state)
        return self.logits(n).float()[:, -1]

    @torch.no_grad()
    def generate(self, ids, max_new_tokens, temperature=1.0, top_k=None, greedy=False, generator=None,
                 top_p=None, eos_token_id=None, stats=None):
        """Cached decoding (ref: one latent cache, Q1; mla: per-layer compressed cache).
        Reference sampling (deepseekv3.ipynb:1850-1873) recomputes the whole prefix per token
        with top-k + temperature; results are identical, the cache removes the recompute."""
        from ..infer.generate import generate
        return generate(self, ids, max_new_tokens, temperature, top_k, top_p, greedy, eos_token_id, generator, stats)

    # ------------------------------------------------------------------- metrics
    def num_params(self, active=False):
        n = sum(p.numel() for p in self.parameters())
        if active:
            for m in self.moe_layers():
                per = (m.w13.numel() + m.w2.numel()) // m.w13.shape[0]
                n -= (m.w13.shape[0] - self.c.top_k) * per
        return n

    def flops_per_token(self, T):
        """6 x active matmul params (routed: top-k experts) + causal attention."""
        c = self.c
        n_mm = self.num_params(active=True) - sum(p.numel() for n, p in self.named_parameters() if p.dim() == 1)
        if c.attention == "ref":
            attn = 6 * c.n_layers * c.n_heads * c.latent_dim * T
        else:
            attn = 3 * c.n_layers * c.n_heads * (c.qk_head_dim + c.v_head_dim) * T
        return 6 * n_mm + attn

    # --------------------------------------------------------- reference layout I/O
    def to_reference_state_dict(self) -> Dict[str, torch.Tensor]:
        """Keys/shapes of the notebook's ``DeepSeekV3.state_dict()`` (ref attention only)."""
        c = self.c
        assert c.attention == "ref", "reference layout exists only for attention='ref'"
        sd = {}
        sd["embedding.weight"] = self.embed
        sd["decoder.embeddings.weight"] = self.embed
        sd["decoder.linear_layer.weight"] = self.embed
        sd["decoder.norm.rmsnorm_layer.weight"] = self.norm_f
        sd["norm1.weight"], sd["norm1.bias"] = self.mtp_norm1_w, self.mtp_norm1_b
        sd["norm2.weight"], sd["norm2.bias"] = self.mtp_norm2_w, self.mtp_norm2_b
        sd["linear_layer.weight"] = self.mtp_proj
        for k, h in enumerate(self.mtp_heads):
            sd[f"heads.{k}.weight"] = h
        for i, l in enumerate(self.layers):
            sd.update(_layer_to_ref(l, f"decoder.decoder.{i}."))
        for k, l in enumerate(self.mtp_layers):
            sd.update(_layer_to_ref(l, f"unilayer.{k}."))
        if self.pe is not None:
            sd["pe"] = self.pe
        return {k: v.detach().float().cpu().clone() for k, v in sd.items()}

    @torch.no_grad()
    def from_reference_state_dict(self, sd):
        self.embed.copy_(sd["decoder.embeddings.weight"])
        self.norm_f.copy_(sd["decoder.norm.rmsnorm_layer.weight"])
        self.mtp_norm1_w.copy_(sd["norm1.weight"])
        self.mtp_norm1_b.copy_(sd["norm1.bias"])
        self.mtp_norm2_w.copy_(sd["norm2.weight"])
        self.mtp_norm2_b.copy_(sd["norm2.bias"])
        self.mtp_proj.copy_(sd["linear_layer.weight"])
        for k, h in enumerate(self.mtp_heads):
            h.copy_(sd[f"heads.{k}.weight"])
        for i, l in enumerate(self.layers):
            _layer_from_ref(l, sd, f"decoder.decoder.{i}.")
        for k, l in enumerate(self.mtp_layers):
            _layer_from_ref(l, sd, f"unilayer.{k}.")
        return self


def _ffn_to_ref(f, F, prefix, sd, e=None):
    w13 = f.w13 if e is None else f.w13[e]
    w2 = f.w2 if e is None else f.w2[e]
    Fp = w13.shape[0] // 2
    sd[prefix + "w1.weight"] = w13[:F]
    sd[prefix + "w2.weight"] = w13[Fp:Fp + F]
    sd[prefix + "w3.weight"] = w2[:, :F]


def _ffn_from_ref(w13, w2, F, sd, prefix):
    Fp = w13.shape[0] // 2
    w13.zero_()
    w2.zero_()
    w13[:F].copy_(sd[prefix + "w1.weight"])
    w13[Fp:Fp + F].copy_(sd[prefix + "w2.weight"])
    w2[:, :F].copy_(sd[prefix + "w3.weight"])


def _layer_to_ref(l: DSV3Layer, p):
    sd = {p + "norm1.rmsnorm_layer.weight": l.attn_norm, p + "norm2.rmsnorm_layer.weight": l.ffn_norm}
    a = l.attn
    for h in range(l.c.n_heads):
        q = f"{p}mhla.heads.{h}."
        sd[q + "W_dkv.weight"] = a.wdkv[h]
        sd[q + "W_k.weight"] = a.wk[h]
        sd[q + "W_v.weight"] = a.wv[h]
        sd[q + "query.weight"] = a.wq[h]
    sd[p + "mhla.linear.weight"] = a.wo
    m = l.ffn
    sd[p + "moe_block.gate.weight"] = m.gate
    if m.noise is not None:
        sd[p + "moe_block.noise.weight"] = m.noise
    sd[p + "moe_block.routing_bias"] = m.routing_bias
    for e in range(m.w13.shape[0]):
        _ffn_to_ref(m, m.F, f"{p}moe_block.experts.{e}.", sd, e)
    if m.shared is not None:
        _ffn_to_ref(m.shared, m.shared.F, p + "moe_block.shared_expert.", sd)
    return sd


def _layer_from_ref(l: DSV3Layer, sd, p):
    l.attn_norm.copy_(sd[p + "norm1.rmsnorm_layer.weight"])
    l.ffn_norm.copy_(sd[p + "norm2.rmsnorm_layer.weight"])
    a = l.attn
    for h in range(l.c.n_heads):
        q = f"{p}mhla.heads.{h}."
        a.wdkv[h].copy_(sd[q + "W_dkv.weight"])
        a.wk[h].copy_(sd[q + "W_k.weight"])
        a.wv[h].copy_(sd[q + "W_v.weight"])
        a.wq[h].copy_(sd[q + "query.weight"])
    a.wo.copy_(sd[p + "mhla.linear.weight"])
    m = l.ffn
    m.gate.copy_(sd[p + "moe_block.gate.weight"])
    if m.noise is not None:
        m.noise.copy_(sd[p + "moe_block.noise.weight"])
    m.routing_bias.copy_(sd[p + "moe_block.routing_bias"])
    for e in range(m.w13.shape[0]):
        _ffn_from_ref(m.w13[e], m.w2[e], m.F, sd, f"{p}moe_block.experts.{e}.")
    if m.shared is not None:
        _ffn_from_ref(m.shared.w13, m.shared.w2, m.shared.F, sd, p + "moe_block.shared_expert.")


def estimate_loss(model, batches):
    """deepseekv3.ipynb:2098-2125 (mean CE over eval batches, eval mode, no grad)."""
    was = model.training
    model.eval()
    with torch.inference_mode():
        ls = [float(model(x, y)) for x, y in batches]
    model.train(was)
    return sum(ls) / max(1, len(ls))
