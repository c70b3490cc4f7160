"""MLA latent decode kernel (csrc/kernels/mla_decode.hip) at DeepSeek widths (C 512, R 64):
time per call vs split count, B = 1 / 8, one query token, 16 or 128 heads.

usage: python tools/bench_mla_decode.py
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from solvingpapers_amd.ops import _ext  # noqa: E402


def timed(fn, iters=50):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    assert _ext.load()
    ops = _ext.ops()
    for B, H, S in ((1, 16, 1056), (1, 16, 4096), (8, 16, 4096), (1, 128, 4096), (4, 128, 4096)):
        q = torch.randn(B, 1, H, 512, device="cuda").bfloat16()
        qr = torch.randn(B, 1, H, 64, device="cuda").bfloat16()
        cc = torch.randn(B, S, 512, device="cuda").bfloat16()
        cr = torch.randn(B, S, 64, device="cuda").bfloat16()
        row = {"B": B, "H": H, "S": S, "MB": round(B * S * 576 * 2 / 1e6, 2)}
        for ns in (0, 1, 4, 16, 64):
            us = timed(lambda: ops.mla_decode(q, qr, cc, cr, 0.07, S, None, ns))
            row[f"us_ns{ns}"] = round(us, 1)
        row["GBps_default"] = round(row["MB"] * 1e3 / row["us_ns0"], 0)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
