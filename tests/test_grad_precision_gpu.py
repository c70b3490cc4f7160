"""Bounds the headline's bf16 gradient accumulation against fp32 main gradients at LLaMA3-8B
widths (2 layers, T 8192, accum 4; tools/grad_precision.py): the bf16 buffer
is rounded once per micro-batch, so its error must stay within a few bf16 roundings of the
exact (fp32-accumulated) sum, and the update direction must be unchanged."""
import os
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))


def test_bf16_grad_accumulation_within_bf16_roundings_at_8b_widths():
    from grad_precision import grad_error
    from solvingpapers_amd.ops import _ext
    assert _ext.load()
    r = grad_error(layers=2, T=8192, accum=4)
    print(r)
    # one bf16 rounding of the exact sum costs r["bf16_floor"] (~2e-3); four sequential
    # roundings of growing partial sums cost at most ~sqrt(4 + 3 + 2 + 1) of that
    assert r["rel_err"] < 4.0 * r["bf16_floor"], r
    assert r["cosine"] > 0.9999, r
    for w in r["worst"]:
        assert w["rel_err"] < 1e-2, w
