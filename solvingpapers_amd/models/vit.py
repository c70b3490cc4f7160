"""Vision Transformer (Dosovitskiy et al.).

Reference: vision transformer/ViT.ipynb (MNIST 28x28, patch 7, D64, 4 heads, 4 blocks,
MLP 2x, randn cls/pos init :262-263, pre-LN blocks with nn.MultiheadAttention :202-227,
LN + Linear head on the CLS token :238-247, Adam 1e-3, 5 epochs, batch 64).
State-dict keys match the reference (patch_embedding.patch_embed.*, cls_token,
pos_embedding, transformer_blocks.{i}.{layer_norm1,layer_norm2,multihead_attention.
{in_proj_weight,in_proj_bias,out_proj.*},mlp.{0,2}.*}, mlp_head.{layer_norm1,mlp_head}.*).

Hot path: implicit-GEMM MFMA patch embedding (bf16: patches gathered straight from the
NCHW image when patch and width are multiples of 8 -- ViT-B/16 -- else from an NHWC copy;
the NHWC output is the token matrix), fused LayerNorm(+residual),
non-causal flash attention (hd 64 for ViT-B/16; T = 197 ragged tile), GELU kernel.
Presets: ``vit_mnist_ref`` and ``vit_b16`` (224^2, patch 16, D768, L12, H12, MLP 3072).
"""
from __future__ import annotations

from dataclasses import dataclass, replace
from typing import Optional

import torch
import torch.nn as tnn

from .. import nn as snn
from ..ops import act, attention_packed, cross_entropy, layer_norm, linear
from ..ops.linear import mlp
from ..ops.misc import patch_embed
from ..utils.grad import mark_ready


@dataclass
class ViTConfig:
    image_size: int = 28
    patch_size: int = 7
    num_channels: int = 1
    embedding_dim: int = 64
    attention_heads: int = 4
    transformer_blocks: int = 4
    mlp_hidden: int = 128
    num_classes: int = 10
    ln_eps: float = 1e-5
    batch_size: int = 64
    lr: float = 1e-3
    epochs: int = 5

    @property
    def num_patches(self):
        return (self.image_size // self.patch_size) ** 2


PRESETS = {
    "vit_mnist_ref": ViTConfig(),  # ViT.ipynb:121-132
    "vit_b16": ViTConfig(image_size=224, patch_size=16, num_channels=3, embedding_dim=768, attention_heads=12,
                         transformer_blocks=12, mlp_hidden=3072, num_classes=1000, ln_eps=1e-6, batch_size=256),
}


def config(name, **kw):
    return replace(PRESETS[name], **kw)


class PatchEmbedding(tnn.Module):
    def __init__(self, c: ViTConfig, **fk):
        super().__init__()
        self.patch = c.patch_size
        self.patch_embed = snn.Conv2d(c.num_channels, c.embedding_dim, c.patch_size, stride=c.patch_size, **fk)

    def forward(self, x):
        return patch_embed(x, self.patch_embed.weight, self.patch_embed.bias, self.patch)


class MHA(tnn.Module):
    """nn.MultiheadAttention-compatible parameters (in_proj_weight [3D, D], out_proj)."""

    def __init__(self, D, H, **fk):
        super().__init__()
        self.H = H
        self.in_proj_weight = tnn.Parameter(torch.empty(3 * D, D, **fk))
        self.in_proj_bias = tnn.Parameter(torch.zeros(3 * D, **fk))
        self.out_proj = snn.Linear(D, D, **fk)
        tnn.init.xavier_uniform_(self.in_proj_weight)
        tnn.init.zeros_(self.out_proj.bias)

    def forward(self, x):
        B, T, D = x.shape
        qkv = linear(x, self.in_proj_weight, self.in_proj_bias)       # [B, T, 3D] = [q | k | v]
        o = attention_packed(qkv, self.H, self.H, causal=False, head_dim=D // self.H)
        return self.out_proj(o.reshape(B, T, D))


class TransformerEncoder(tnn.Module):
    def __init__(self, c: ViTConfig, **fk):
        super().__init__()
        D = c.embedding_dim
        self.eps = c.ln_eps
        self.layer_norm1 = snn.LayerNorm(D, c.ln_eps, **fk)
        self.layer_norm2 = snn.LayerNorm(D, c.ln_eps, **fk)
        self.multihead_attention = MHA(D, c.attention_heads, **fk)
        self.mlp = tnn.Sequential(snn.Linear(c.embedding_dim, c.mlp_hidden, **fk), snn.GELU(),
                                  snn.Linear(c.mlp_hidden, c.embedding_dim, **fk))

    def forward(self, x):
        h, m = self.forward_pair(x, None)
        return h + m

    def forward_pair(self, h, m):
        """Block on the unsummed residual pair (input x = h + m; m None: x = h) -> (h', m') with
        output h' + m'. The sum happens inside the next LayerNorm (one fused pass that also
        returns x), so the chain has no standalone residual add in either direction."""
        if m is None:
            x, n1 = h, self.layer_norm1(h)
        else:
            n1, x = self.layer_norm1(m, residual=h)
        a = self.multihead_attention(n1)
        n2, h2 = self.layer_norm2(a, residual=x)     # h2 = x + attn, n2 = LN2(h2)
        fc1, gelu, fc2 = self.mlp
        # ops.linear.mlp: hipBLASLt fc1 (+ bias) and a GELU pass forward; backward GELU' and fc1's bias
        # gradient in one pass (GEMM-epilogue forms measured slower, profiles/r5_vit_mlp_epilogue_and_fast_erf_rejected.txt)
        return h2, mlp(n2, fc1.weight, fc1.bias, fc2.weight, fc2.bias, gelu.kind, gelu.alpha)


class MLPHead(tnn.Module):
    def __init__(self, c: ViTConfig, **fk):
        super().__init__()
        self.layer_norm1 = snn.LayerNorm(c.embedding_dim, c.ln_eps, **fk)
        self.mlp_head = snn.Linear(c.embedding_dim, c.num_classes, **fk)

    def forward(self, x):
        return self.mlp_head(self.layer_norm1(x))


class ViT(tnn.Module):
    def __init__(self, c: ViTConfig = ViTConfig(), device=None, dtype=None):
        super().__init__()
        fk = dict(device=device, dtype=dtype)
        self.c = c
        self.patch_embedding = PatchEmbedding(c, **fk)
        self.cls_token = tnn.Parameter(torch.randn(1, 1, c.embedding_dim, **fk))
        self.pos_embedding = tnn.Parameter(torch.randn(1, c.num_patches + 1, c.embedding_dim, **fk))
        self.transformer_blocks = tnn.Sequential(*[TransformerEncoder(c, **fk) for _ in range(c.transformer_blocks)])
        self.mlp_head = MLPHead(c, **fk)
        self.grad_ready_cb = None

    def param_groups(self):
        return ([[self.cls_token, self.pos_embedding] + list(self.patch_embedding.parameters())] +
                [list(b.parameters()) for b in self.transformer_blocks] + [list(self.mlp_head.parameters())])

    def forward(self, x, targets=None):
        x = self.patch_embedding(x)
        x = torch.cat([self.cls_token.expand(x.shape[0], -1, -1), x], dim=1) + self.pos_embedding
        h, m = x, None
        for i, blk in enumerate(self.transformer_blocks):
            h = mark_ready(h, self.grad_ready_cb, i + 1)
            h, m = blk.forward_pair(h, m)
        h = mark_ready(h, self.grad_ready_cb, len(self.transformer_blocks) + 1)
        logits = self.mlp_head(h[:, 0] + m[:, 0] if m is not None else h[:, 0])
        if targets is None:
            return logits
        return cross_entropy(logits, targets)


def train(cfg: ViTConfig = PRESETS["vit_mnist_ref"], epochs=None, device=None, n_train=6000, n_test=1000,
          mnist_root: Optional[str] = None, log=print, seed=0):
    """Adam + CE loop with per-batch accuracy (ViT.ipynb:286-288,365-394) and test
    accuracy (:412-426) on MNIST IDX files or synthetic MNIST-like data."""
    from ..data.images import ImageBatches, mnist_or_synthetic
    from ..train.optim import FlatAdam
    from ..utils.flat import FlatParams
    device = device or ("cuda" if torch.cuda.is_available() else "cpu")
    torch.manual_seed(seed)
    (xtr, ytr), (xte, yte) = mnist_or_synthetic(mnist_root, n_train, n_test, seed)
    model = ViT(cfg, device=device)
    flat = FlatParams(model, groups=model.param_groups())
    opt = FlatAdam(flat, lr=cfg.lr)
    tl = ImageBatches(xtr, ytr, cfg.batch_size, True, device, seed)
    vl = ImageBatches(xte, yte, cfg.batch_size, False, device)
    accs = []
    for ep in range(epochs or cfg.epochs):
        correct = total = 0
        for x, y in tl:
            opt.zero_grad()
            logits = model(x)
            correct += int((logits.argmax(1) == y).sum())
            total += y.numel()
            cross_entropy(logits, y).backward()
            opt.step()
        acc = evaluate(model, vl)
        accs.append(acc)
        log(f"epoch {ep + 1}: train acc {100 * correct / total:.2f}% test acc {acc:.2f}%")
    return model, accs


@torch.inference_mode()
def evaluate(model, loader):
    model.eval()
    c = t = 0
    for x, y in loader:
        c += int((model(x).argmax(1) == y).sum())
        t += y.numel()
    model.train()
    return 100.0 * c / max(t, 1)
