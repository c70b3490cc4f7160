"""Trainer metric hooks with the reference's W&B metric names.

The DeepSeek notebook logs ``{train_loss, train_perplexity, lr, grad_norm, tokens, step}``
per step and ``{val_loss, val_perplexity}`` per eval to Weights & Biases
(deepseekv3/deepseekv3.ipynb:2323-2336, 2380, 2451-2458). The Trainer's records are
``{step, loss, lr, grad_norm, tok_per_s, tokens, mfu, mem_gb, ...}`` / ``{step, val_loss}``; ``reference_names``
maps one to the other. ``WandbHook`` forwards them to wandb when that package exists
(it is not installed here: constructing the hook then raises, nothing is silently dropped);
``JsonlHook`` writes the same renamed records to a file, for offline dashboards.
"""
from __future__ import annotations

import json
import math
from typing import Optional


def reference_names(rec: dict, tokens_per_step: Optional[int] = None) -> dict:
    """Trainer record -> the reference's W&B keys (perplexity = exp(loss))."""
    out = {"step": rec["step"]}
    if "loss" in rec and rec["loss"] is not None:
        out["train_loss"] = float(rec["loss"])
        out["train_perplexity"] = math.exp(min(float(rec["loss"]), 80.0))
    if rec.get("val_loss") is not None:
        out["val_loss"] = float(rec["val_loss"])
        out["val_perplexity"] = math.exp(min(float(rec["val_loss"]), 80.0))
    for k in ("lr", "grad_norm", "tok_per_s", "mfu", "mem_gb"):
        if rec.get(k) is not None:
            out[k] = float(rec[k])
    if tokens_per_step is not None:
        out["tokens"] = (rec["step"] + 1) * tokens_per_step
    elif rec.get("tokens") is not None:            # the Trainer's own cumulative count
        out["tokens"] = int(rec["tokens"])
    return out


class JsonlHook:
    def __init__(self, path: str, tokens_per_step: Optional[int] = None):
        self.f = open(path, "a")
        self.tps = tokens_per_step

    def __call__(self, rec: dict):
        self.f.write(json.dumps(reference_names(rec, self.tps)) + "\n")
        self.f.flush()

    def close(self):
        self.f.close()


class WandbHook:
    def __init__(self, project: str, config: Optional[dict] = None, tokens_per_step: Optional[int] = None, **kw):
        try:
            import wandb
        except ImportError as e:
            raise RuntimeError("WandbHook needs the 'wandb' package (not installed in this image); "
                               "use JsonlHook for offline metrics") from e
        self.wandb = wandb
        self.run = wandb.init(project=project, config=config or {}, **kw)
        self.tps = tokens_per_step

    def __call__(self, rec: dict):
        self.wandb.log(reference_names(rec, self.tps), step=rec["step"])

    def close(self):
        self.wandb.finish()
