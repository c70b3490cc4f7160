"""Faithful re-statements of the reference notebooks' math (jax is not installed),
used by the parity tests. Each function mirrors the cited reference cell line by
line in float64 torch; nothing here is used by the framework itself."""
import math

import torch


# --- llama3/LLaMA-jax.ipynb cells 15-28 ------------------------------------
def ll_rms_norm(x, w, eps=1e-6):  # :536-538
    var = (x * x).mean(-1, keepdim=True)
    return x * w * (1.0 / torch.sqrt(var + eps))


def ll_freqs_cis(dim, end, theta=10000.0):  # :563-567  (arange(0, dim//2)/dim)
    freqs = 1.0 / (theta ** (torch.arange(0, dim // 2, dtype=torch.float64) / dim))
    t = torch.arange(end, dtype=torch.float64)
    return torch.polar(torch.ones(end, dim // 2, dtype=torch.float64), torch.outer(t, freqs))


def ll_apply_rotary(xq, xk, fc):  # :592-601
    def rot(x):
        xr = x.reshape(*x.shape[:-1], -1, 2)
        xc = torch.complex(xr[..., 0], xr[..., 1])
        out = xc * fc.reshape(1, fc.shape[0], 1, fc.shape[1])
        return torch.stack([out.real, out.imag], -1).reshape(x.shape)
    return rot(xq), rot(xk)


def ll_attention(p, x, mask, fc, H, KV):  # :809-829
    B, T, C = x.shape
    hd = C // H
    q = (x @ p["wq"]).reshape(B, T, H, hd)
    k = (x @ p["wk"]).reshape(B, T, KV, hd)
    v = (x @ p["wv"]).reshape(B, T, KV, hd)
    q, k = ll_apply_rotary(q, k, fc[:T])
    k = k.repeat_interleave(H // KV, dim=2)
    v = v.repeat_interleave(H // KV, dim=2)
    q, k, v = (t.transpose(1, 2) for t in (q, k, v))
    s = q @ k.transpose(-1, -2) / math.sqrt(hd) + mask[:, :, :T, :T]
    o = torch.softmax(s, -1) @ v
    return o.transpose(1, 2).reshape(B, T, -1) @ p["wo"]


def ll_forward(params, ids, H, KV, max_seq_len):  # :916-931
    h = params["token_embedding"][ids]
    D = h.shape[-1]
    fc = ll_freqs_cis(D // H, max_seq_len)
    mask = torch.tril(torch.ones(max_seq_len, max_seq_len, dtype=torch.float64))
    mask = torch.where(mask == 0, -1e9, 0.0)[None, None]
    for b in params["blocks"]:
        a = ll_attention(b["attention"], ll_rms_norm(h, b["attention_norm"]), mask, fc, H, KV)
        h = h + a
        f = b["ffn"]
        n = ll_rms_norm(h, b["ffn_norm"])
        h = h + (torch.nn.functional.silu(n @ f["w3"]) * (n @ f["w1"])) @ f["w2"]  # :854-855 (gate = w3)
    return ll_rms_norm(h, params["norm_f"]) @ params["output"]


def to64(tree):
    if isinstance(tree, dict):
        return {k: to64(v) for k, v in tree.items()}
    if isinstance(tree, list):
        return [to64(v) for v in tree]
    return tree.double()


# --- gpt/gpt-jax.ipynb cells 13-16 (:321-472) and the loss (:499-503) -------
def gpt_layer_norm(x, scale, bias, eps=1e-6):  # flax nn.LayerNorm defaults (eps 1e-6, biased variance)
    mu = x.mean(-1, keepdim=True)
    var = ((x - mu) ** 2).mean(-1, keepdim=True)
    return (x - mu) / torch.sqrt(var + eps) * scale + bias


def gpt_gelu(x):  # flax nn.gelu: approximate=True (tanh form)
    return 0.5 * x * (1.0 + torch.tanh(math.sqrt(2.0 / math.pi) * (x + 0.044715 * x ** 3)))


def gpt_attention(p, x, H):  # :321-357 (deterministic: no dropout)
    B, T, D = x.shape
    hd = D // H
    qkv = x @ p["qkv/kernel"]                                       # Dense(3D, use_bias=False)
    q, k, v = qkv[..., :D], qkv[..., D:2 * D], qkv[..., 2 * D:]     # jnp.split(qkv, 3, axis=-1)
    q, k, v = (t.reshape(B, T, H, hd).permute(0, 2, 1, 3) for t in (q, k, v))
    w = q @ k.transpose(-1, -2) / math.sqrt(hd)
    mask = torch.tril(torch.ones(T, T, dtype=torch.float64)).reshape(1, 1, T, T)
    w = torch.where(mask == 0, torch.full_like(w, -1e4), w)         # jnp.where(mask == 0, -1e4, w)
    w = torch.softmax(w, -1)
    o = (w @ v).permute(0, 2, 1, 3).reshape(B, T, D)
    return o @ p["proj/kernel"] + p["proj/bias"]


def gpt_forward(d, ids, H, L):  # :441-472, parameters in the Flax pytree layout (to_reference_params)
    B, T = ids.shape
    x = d["token_embed/embedding"][ids] + d["pos_embed"][:, :T, :]
    for i in range(L):
        p = {k[len(f"layers_{i}/"):]: v for k, v in d.items() if k.startswith(f"layers_{i}/")}
        x = x + gpt_attention({k[5:]: v for k, v in p.items() if k.startswith("attn/")},
                              gpt_layer_norm(x, p["ln1/scale"], p["ln1/bias"]), H)
        n = gpt_layer_norm(x, p["ln2/scale"], p["ln2/bias"])
        x = x + (gpt_gelu(n @ p["mlp/fc1/kernel"] + p["mlp/fc1/bias"]) @ p["mlp/fc2/kernel"] + p["mlp/fc2/bias"])
    x = gpt_layer_norm(x, d["ln_f/scale"], d["ln_f/bias"])
    return x @ d["lm_head/kernel"]                                   # Dense(V, use_bias=False)


def gpt_loss(logits, targets):  # :499-503 optax.softmax_cross_entropy_with_integer_labels(...).mean()
    V = logits.shape[-1]
    lp = torch.log_softmax(logits.reshape(-1, V), -1)
    return -lp.gather(1, targets.reshape(-1, 1)).mean()
