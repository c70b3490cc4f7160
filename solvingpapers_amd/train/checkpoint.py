"""Checkpoint / resume.

Reference mechanisms (SURVEY §5 "Checkpoint / resume"): LLaMA pickles the JAX param
pytree (llama3/LLaMA-jax.ipynb:433-443), Gemma ``torch.save(state_dict)`` every 100
steps (gemma/gemma.ipynb:557), DeepSeek saves ``{step, model_state_dict,
optimizer_state_dict, loss}`` to ``checkpoint_latest.pt`` and resumes at step+1
(deepseekv3/deepseekv3.ipynb:2167-2199). None saves RNG / data position / LR state.

Here each rank writes its own file (its ZeRO shard of the optimizer, its experts under
EP) holding a handful of large flat tensors:

    <dir>/step_000123/rank00000.pt   {step, flat params, optimizer state, RNG, extra}
    <dir>/latest                     "step_000123" (written last, atomically)

Every file is written to ``*.tmp`` and ``os.replace``'d, ``latest`` only after a barrier
when every rank's file exists, so a crash mid-save never corrupts the previous
checkpoint. Files hold only tensors and plain Python values and load with
``torch.load(weights_only=True)``. ``keep`` prunes old step directories.
"""
from __future__ import annotations

import os
import shutil
from typing import Any, Dict, Optional

import torch
import torch.distributed as dist


def _rank_world():
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def _barrier():
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.barrier()


def _atomic_save(obj, path):
    tmp = path + ".tmp"
    torch.save(obj, tmp)
    os.replace(tmp, path)


def _rng_state():
    st = {"cpu": torch.get_rng_state()}
    if torch.cuda.is_available() and torch.cuda.is_initialized():
        st["cuda"] = torch.cuda.get_rng_state()
    return st


def _set_rng_state(st):
    torch.set_rng_state(st["cpu"])
    if "cuda" in st and torch.cuda.is_available():
        torch.cuda.set_rng_state(st["cuda"])


def _to_cpu(x):
    if isinstance(x, torch.Tensor):
        return x.detach().cpu()
    if isinstance(x, dict):
        return {k: _to_cpu(v) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return type(x)(_to_cpu(v) for v in x)
    return x


def save(ckpt_dir: str, step: int, flat, optimizer=None, buffers: Optional[Dict[str, torch.Tensor]] = None,
         extra: Optional[Dict[str, Any]] = None, keep: int = 2) -> str:
    """Save this rank's training state for ``step``; returns the step directory."""
    rank, world = _rank_world()
    name = f"step_{step:09d}"
    sdir = os.path.join(ckpt_dir, name)
    os.makedirs(sdir, exist_ok=True)
    obj = {
        "step": int(step),
        "world_size": world,
        "param": flat.param.detach().cpu(),
        "optimizer": _to_cpu(optimizer.state_dict()) if optimizer is not None else None,
        "buffers": _to_cpu(buffers or {}),
        "rng": _rng_state(),
        "extra": extra or {},
    }
    _atomic_save(obj, os.path.join(sdir, f"rank{rank:05d}.pt"))
    _barrier()
    if rank == 0:
        with open(os.path.join(ckpt_dir, "latest.tmp"), "w") as f:
            f.write(name)
        os.replace(os.path.join(ckpt_dir, "latest.tmp"), os.path.join(ckpt_dir, "latest"))
        olds = sorted(d for d in os.listdir(ckpt_dir) if d.startswith("step_") and d != name)
        for d in olds[:max(0, len(olds) - (keep - 1))] if keep > 0 else []:
            shutil.rmtree(os.path.join(ckpt_dir, d), ignore_errors=True)
    _barrier()
    return sdir


def latest(ckpt_dir: str) -> Optional[str]:
    p = os.path.join(ckpt_dir, "latest")
    if not os.path.exists(p):
        return None
    with open(p) as f:
        name = f.read().strip()
    d = os.path.join(ckpt_dir, name)
    return d if os.path.isdir(d) else None


def load(path: str, flat, optimizer=None, buffers: Optional[Dict[str, torch.Tensor]] = None,
         restore_rng: bool = True) -> Dict[str, Any]:
    """Load this rank's file from a step directory (or a checkpoint root with ``latest``).
    Returns {"step", "extra"}; training resumes at step + 1."""
    rank, world = _rank_world()
    if os.path.exists(os.path.join(path, "latest")):
        path = latest(path)
    obj = torch.load(os.path.join(path, f"rank{rank:05d}.pt"), map_location="cpu", weights_only=True)
    if obj["world_size"] != world:
        raise RuntimeError(f"checkpoint written with world size {obj['world_size']}, running {world}")
    with torch.no_grad():
        flat.param.copy_(obj["param"].to(flat.param.device))
    from ..ops.linear import invalidate_weight_caches
    invalidate_weight_caches()          # written through the flat buffer (ops/linear.py CONTRACT)
    if optimizer is not None and obj["optimizer"] is not None:
        dev = flat.param.device
        optimizer.load_state_dict({k: (v.to(dev) if isinstance(v, torch.Tensor) else v)
                                   for k, v in obj["optimizer"].items()})
    for k, t in (buffers or {}).items():
        if k in obj["buffers"]:
            with torch.no_grad():
                t.copy_(obj["buffers"][k].to(t.device))
    if restore_rng:
        _set_rng_state(obj["rng"])
    return {"step": obj["step"], "extra": obj["extra"]}


# ------------------------------------------------------------- reference formats
def save_reference_dsv3(path: str, model, step: int, loss=None, optimizer_state=None):
    """deepseekv3.ipynb:2167-2178 layout: {step, model_state_dict, optimizer_state_dict, loss}."""
    _atomic_save({"step": step, "model_state_dict": model.to_reference_state_dict(),
                  "optimizer_state_dict": optimizer_state or {}, "loss": loss}, path)


def load_reference_dsv3(path: str, model):
    """Resume semantics of deepseekv3.ipynb:2181-2188 (returns step + 1). Loads with
    weights_only=True: only tensors / plain values are accepted."""
    ck = torch.load(path, map_location="cpu", weights_only=True)
    model.from_reference_state_dict(ck["model_state_dict"])
    return ck["step"] + 1


def save_state_dict(path: str, state: Dict[str, torch.Tensor]):
    """Gemma-style ``torch.save(model.state_dict())`` (gemma.ipynb:557)."""
    _atomic_save({k: v.detach().cpu() for k, v in state.items()}, path)
