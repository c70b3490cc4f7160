"""Loader for the in-tree gfx950 extension (``solvingpapers_amd/_C.so``).

The HIP kernels are registered as ``torch.ops.spa.*`` (TORCH_LIBRARY). CPU
tensors use the pure-PyTorch oracles in :mod:`solvingpapers_amd.ops.reference`;
a GPU tensor NEVER silently falls back — if the extension is missing or fails
to load, :func:`ops` raises so a GPU test cannot pass on an eager fallback.
"""
from __future__ import annotations

import os
from pathlib import Path

import torch

# SPA_EXT_SO: load another build of the extension (kernel A/B experiments on one box)
_SO = Path(os.environ.get("SPA_EXT_SO") or Path(__file__).resolve().parent.parent / "_C.so")
_loaded = False
_err: str | None = None


def load() -> bool:
    global _loaded, _err
    if _loaded:
        return True
    if not _SO.exists():
        _err = f"{_SO} not built (run `python -m solvingpapers_amd._build`)"
        return False
    try:
        torch.ops.load_library(str(_SO))
        _loaded = True
    except Exception as e:  # pragma: no cover - depends on the box
        _err = f"failed to load {_SO}: {e}"
    return _loaded


def available() -> bool:
    return load()


def ops():
    """Return the ``torch.ops.spa`` namespace or raise loudly."""
    if not load():
        raise RuntimeError(f"solvingpapers_amd HIP extension unavailable: {_err}")
    return torch.ops.spa


def so_path() -> str:
    return str(_SO)


def on_gpu(t: torch.Tensor) -> bool:
    return t.is_cuda


def debug_sync(name: str):
    """SPA_DEBUG_SYNC=1 -> synchronise after every HIP op (fault localisation)."""
    if os.environ.get("SPA_DEBUG_SYNC") == "1" and torch.cuda.is_available():
        torch.cuda.synchronize()
