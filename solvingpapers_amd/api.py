"""The reference's per-model entry-point names, so notebook users find them here.

    gpt/gpt-jax.ipynb            get_batch, estimate_loss, generate (greedy)
    llama3/LLaMA-jax.ipynb       get_batch, save_params / load_params, generate (categorical)
    gemma/gemma.ipynb            get_batch, estimate_loss, generate (multinomial)
    deepseekv3/deepseekv3.ipynb  get_lr, compute_mtp_loss, estimate_loss, topk_sampling,
                                 save_checkpoint / load_checkpoint, save_text
    vision transformer / AE / VAE / kd.py: train / evaluate / vae_loss / distillation_loss

All are thin wrappers over the framework (models/*, train/*, ops/*). Serialisation is
pickle-free: ``save_params`` writes the LLaMA reference pytree (nested dict of arrays,
llama3/LLaMA-jax.ipynb:433-443) to safetensors with '/'-joined keys.
"""
from __future__ import annotations

import math
from typing import Dict, Iterable, Optional

import torch

from .data.text import get_batch  # noqa: F401  (gpt-jax.ipynb:491-497, gemma.ipynb:116-129, LLaMA :468-474)
from .models.autoencoder import train as train_autoencoder  # noqa: F401
from .models.kd import evaluate as kd_evaluate, train as kd_train  # noqa: F401
from .models.vit import evaluate as vit_evaluate, train as vit_train  # noqa: F401
from .ops.misc import distillation_loss, vae_loss  # noqa: F401
from .train.optim import cosine_lr


# ------------------------------------------------------------------ generic
@torch.no_grad()
def estimate_loss(model, splits: Dict[str, torch.Tensor], eval_iters: int, batch_size: int, block_size: int,
                  generator=None) -> Dict[str, float]:
    """Mean loss over ``eval_iters`` random batches per split (gpt-jax.ipynb:542-552,
    gemma.ipynb:522-538). ``splits`` maps name -> flat token tensor."""
    was = model.training
    model.eval()
    out = {}
    for name, data in splits.items():
        tot = 0.0
        for _ in range(eval_iters):
            x, y = get_batch(data, batch_size, block_size, generator)
            tot += float(model(x, y))
        out[name] = tot / eval_iters
    model.train(was)
    return out


# ------------------------------------------------------------------ LLaMA pytree I/O
def _flatten(tree, prefix=""):
    if isinstance(tree, dict):
        out = {}
        for k, v in tree.items():
            out.update(_flatten(v, f"{prefix}{k}/"))
        return out
    if isinstance(tree, (list, tuple)):
        out = {}
        for i, v in enumerate(tree):
            out.update(_flatten(v, f"{prefix}{i}/"))
        return out
    return {prefix[:-1]: torch.as_tensor(tree).detach().cpu().contiguous()}


def _unflatten(flat):
    root: dict = {}
    for key, v in flat.items():
        parts = key.split("/")
        d = root
        for p in parts[:-1]:
            d = d.setdefault(p, {})
        d[parts[-1]] = v

    def fix(d):
        if isinstance(d, dict):
            d = {k: fix(v) for k, v in d.items()}
            if d and all(k.isdigit() for k in d):
                return [d[str(i)] for i in range(len(d))]
        return d
    return fix(root)


def save_params(params, path: str):
    """LLaMA-jax.ipynb:433-437 (pickle of the param pytree) -> safetensors, no pickle."""
    from safetensors.torch import save_file
    save_file(_flatten(params), path)


def load_params(path: str):
    """LLaMA-jax.ipynb:439-443; returns the nested pytree of tensors."""
    from safetensors.torch import load_file
    return _unflatten(load_file(path))


# ------------------------------------------------------------------ DeepSeek-V3
def get_lr(step, max_lr=6e-4, warmup_iters=400, lr_decay_iters=10000, min_lr=6e-5):
    """deepseekv3.ipynb:1976-1986."""
    return cosine_lr(step, max_lr, warmup_iters, lr_decay_iters, min_lr)


def compute_mtp_loss(logits, targets, ignore_index: int = -100):
    """deepseekv3.ipynb:2030-2056: logits [B, T, D, C] (D prediction depths); depth k at
    position i predicts token i+k+1 (clamped to the last target)."""
    B, T, D, C = logits.shape
    i = torch.arange(T, device=targets.device)[:, None]
    k = torch.arange(D, device=targets.device)[None, :]
    idx = (i + k + 1).clamp(max=targets.size(1) - 1).reshape(1, T * D).expand(B, -1)
    tgt = torch.gather(targets, 1, idx)
    return torch.nn.functional.cross_entropy(logits.reshape(-1, C).float(), tgt.reshape(-1),
                                             ignore_index=ignore_index)


@torch.no_grad()
def topk_sampling(model, input_ids, max_length=50, top_k=50, temperature=1.0, eos_token_id: Optional[int] = None,
                  generator=None):
    """deepseekv3.ipynb:1849-1873 (softmax -> top-k -> multinomial until max_length or EOS) as ONE
    cached ``generate`` call: the prompt is prefilled once and every further token is a single
    decode step against the model's KV / latent cache (the reference re-runs the whole prefix
    per token). With ``eos_token_id`` a finished sequence is padded with EOS; a single sequence
    is cut right after its first EOS, exactly where the reference's loop breaks."""
    remaining = max(0, max_length - input_ids.shape[1])
    if remaining == 0:
        return input_ids
    out = model.generate(input_ids, remaining, temperature=temperature, top_k=top_k, greedy=False,
                         generator=generator, eos_token_id=eos_token_id)
    if eos_token_id is not None and out.shape[0] == 1:
        gen = out[0, input_ids.shape[1]:]
        hit = (gen == eos_token_id).nonzero()
        if hit.numel():
            out = out[:, :input_ids.shape[1] + int(hit[0, 0]) + 1]
    return out


def save_checkpoint(model, optimizer_state, step, loss, path):
    """deepseekv3.ipynb:2167-2178 format ({step, model_state_dict, optimizer_state_dict, loss})."""
    from .train.checkpoint import save_reference_dsv3
    save_reference_dsv3(path, model, step, loss, optimizer_state)


def load_checkpoint(path, model):
    """deepseekv3.ipynb:2181-2188: returns the step to resume at (saved step + 1)."""
    from .train.checkpoint import load_reference_dsv3
    return load_reference_dsv3(path, model)


def save_text(path, step, text):
    """deepseekv3.ipynb:2224-2226."""
    with open(path, "w") as f:
        f.write(f"step {step}\n{text}\n")


def perplexity(loss: float) -> float:
    return math.exp(loss)
