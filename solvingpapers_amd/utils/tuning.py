"""GEMM solution tables (PyTorch TunableOp over hipBLASLt + rocBLAS) shipped with the repo.

The dense projections stay library GEMMs; which hipBLASLt / rocBLAS solution
runs for a shape is what TunableOp measures. ``tools/tune_gemms.py`` tunes the recorded
shapes of a workload on an MI355X and ``tuning/*.csv`` keeps the winners (their validator
lines pin the PyTorch / ROCm / hipBLASLt / rocBLAS versions and the gfx950 arch; TunableOp
ignores a file whose validators do not match, so a stale table falls back to the default
heuristics instead of failing). ``load_gemm_tuning()`` enables lookup-only mode: shapes in
the table use the tuned solution, every other GEMM the library default; nothing is tuned
at run time and nothing is written back into the repo.
"""
from __future__ import annotations

import os
from typing import Optional

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
DEFAULT_TABLE = os.path.join(ROOT, "tuning", "tunableop_llama8b.csv")


def load_gemm_tuning(path: Optional[str] = None) -> bool:
    """Use the tuned GEMM table at ``path`` (default: tuning/tunableop_llama8b.csv).
    SPA_GEMM_TUNING=0 disables it; SPA_GEMM_RECORD_UNTUNED=<csv> records the GEMMs it misses.
    Returns True if the table was loaded."""
    if os.environ.get("SPA_GEMM_TUNING", "1") == "0" or not torch.cuda.is_available():
        return False
    path = path or DEFAULT_TABLE
    if not os.path.exists(path):
        return False
    import torch.cuda.tunable as tunable
    tunable.enable(True)
    tunable.tuning_enable(False)
    # SPA_GEMM_RECORD_UNTUNED=<csv>: list the GEMMs the table does not cover (table-coverage check)
    untuned = os.environ.get("SPA_GEMM_RECORD_UNTUNED")
    if untuned:
        os.environ["PYTORCH_TUNABLEOP_UNTUNED_FILENAME"] = untuned
    tunable.record_untuned_enable(bool(untuned))
    # results of this process (none: tuning is off) go to a scratch file, never the repo table
    tunable.set_filename(os.path.join(os.environ.get("TMPDIR", "/tmp"), "spa_tunableop_out.csv"), True)
    return bool(tunable.read_file(path))
