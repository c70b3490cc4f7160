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
    """Return the ``torch.ops.spa`` namespace or raise loudly.

    With SPA_DEBUG_SYNC=1 the namespace is wrapped so every op call is followed by a device
    synchronise (a fault surfaces at the op that caused it) and, in a debug-bounds build
    (``tools/build_variant.sh dbg -DSPA_DEBUG_BOUNDS=1``, loaded through SPA_EXT_SO), by a read of the
    kernels' bounds-guard records: a violation raises :class:`BoundsViolation` naming the op and the
    kernel file:line, block, thread, index and limit."""
    if not load():
        raise RuntimeError(f"solvingpapers_amd HIP extension unavailable: {_err}")
    if os.environ.get("SPA_DEBUG_SYNC") == "1":
        return _checked_ops()
    return torch.ops.spa


class BoundsViolation(RuntimeError):
    """A device-side bounds guard of the debug build fired (csrc/include/spa_debug.h)."""


def debug_bounds_enabled() -> bool:
    """True when the loaded extension was built with -DSPA_DEBUG_BOUNDS=1."""
    return load() and bool(torch.ops.spa.debug_bounds_enabled())


def debug_bounds_report(reset: bool = True) -> str:
    """Violations recorded by the device guards since the last reset ("" when clean or release)."""
    if not load():
        return ""
    return str(torch.ops.spa.debug_bounds_report(reset))


class _CheckedOp:
    __slots__ = ("_op", "_name")

    def __init__(self, op, name):
        self._op, self._name = op, name

    def __call__(self, *a, **k):
        out = self._op(*a, **k)
        # inside a HIP-graph capture a device sync is illegal: the guard records are read after
        # replay instead (debug_sync / debug_bounds_report by the caller)
        if torch.cuda.is_available() and torch.cuda.is_initialized() and \
                not torch.cuda.is_current_stream_capturing():
            torch.cuda.synchronize()
            if _DEBUG_BOUNDS[0]:
                rep = debug_bounds_report(True)
                if rep:
                    raise BoundsViolation(f"spa.{self._name}: device bounds guard fired\n{rep}")
        return out

    def __getattr__(self, attr):
        return getattr(self._op, attr)


class _CheckedNamespace:
    def __getattr__(self, name):
        op = getattr(torch.ops.spa, name)
        return _CheckedOp(op, name) if callable(op) else op


_DEBUG_BOUNDS = [False]
_CHECKED = []


def _checked_ops():
    if not _CHECKED:
        _DEBUG_BOUNDS[0] = debug_bounds_enabled()
        _CHECKED.append(_CheckedNamespace())
    return _CHECKED[0]


def so_path() -> str:
    return str(_SO)


def on_gpu(t: torch.Tensor) -> bool:
    return t.is_cuda


def debug_sync(name: str):
    """SPA_DEBUG_SYNC=1 -> synchronise here (and, in a debug-bounds build, check the guards) -- for
    code that launches kernels outside :func:`ops` (e.g. hipBLASLt GEMMs between two HIP ops)."""
    if os.environ.get("SPA_DEBUG_SYNC") == "1" and torch.cuda.is_available() and \
            not torch.cuda.is_current_stream_capturing():
        torch.cuda.synchronize()
        if debug_bounds_enabled():
            rep = debug_bounds_report(True)
            if rep:
                raise BoundsViolation(f"{name}: device bounds guard fired\n{rep}")
