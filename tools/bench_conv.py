"""Implicit-GEMM conv kernels vs torch/MIOpen conv2d (bf16) at AlexNet (batch 128) and ViT-B/16
patch-embed (batch 256) shapes: fwd, data grad, weight grad in TFLOP/s (useful FLOPs,
2*N*OH*OW*OC*C*KH*KW per GEMM).

usage: python tools/bench_conv.py [--iters N]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from solvingpapers_amd.ops import _ext, conv as C  # noqa: E402

SHAPES = {  # name: (N, C, H, W, OC, K, stride, pad)
    "alexnet_conv1": (128, 3, 224, 224, 96, 11, 4, 1),
    "alexnet_conv2": (128, 96, 26, 26, 256, 5, 1, 2),
    "alexnet_conv3": (128, 256, 12, 12, 384, 3, 1, 1),
    "alexnet_conv4": (128, 384, 12, 12, 384, 3, 1, 1),
    "alexnet_conv5": (128, 384, 12, 12, 256, 3, 1, 1),
    "vit_b16_patch": (256, 3, 224, 224, 768, 16, 16, 0),
}


def timed(fn, iters):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    assert _ext.load()
    ops = _ext.ops()
    for name, (N, Cc, H, W, OC, K, s, p) in SHAPES.items():
        x = torch.randn(N, Cc, H, W, device="cuda").bfloat16()
        w = (torch.randn(OC, Cc, K, K, device="cuda") * 0.02).bfloat16()
        b = torch.zeros(OC, device="cuda", dtype=torch.bfloat16)
        nhwc = not C.nchw_direct_ok(Cc, H, W, K, K, s, s, p, p)
        geo = C.geometry(x.shape, w.shape, (s, s), (p, p), nhwc)
        OH, OW, Cp = geo[13], geo[14], geo[5]
        xg = C._gathered(x.contiguous(memory_format=torch.channels_last) if nhwc else x, geo)
        wp = ops.conv_pack_weight(w, Cp) if nhwc else w.reshape(OC, -1).contiguous()
        kt = C._cached("fwd", geo, x.device, C.fwd_table)
        fl = 2.0 * N * OH * OW * OC * Cc * K * K
        row = {"shape": name, "GFLOP": round(fl / 1e9, 1)}
        row["fwd_TF"] = round(fl / timed(lambda: ops.conv_fwd(xg, wp, kt, b, geo), a.iters) / 1e9, 1)
        dy = torch.randn(N, OH, OW, OC, device="cuda").bfloat16()
        row["wgrad_TF"] = round(fl / timed(lambda: ops.conv_wgrad(dy, xg, kt, geo, True, torch.bfloat16), a.iters)
                                / 1e9, 1)
        gn = C.geometry(x.shape, w.shape, (s, s), (p, p), True)
        kd, bt = C._cached("dgrad", gn, x.device, C.dgrad_tables)
        wpn = ops.conv_pack_weight(w, gn[5])
        if Cc >= 8:
            row["dgrad_TF"] = round(fl / timed(lambda: ops.conv_dgrad(dy, wpn, kd, bt, gn), a.iters) / 1e9, 1)
        xc = x.contiguous(memory_format=torch.channels_last)
        row["torch_fwd_TF"] = round(fl / timed(lambda: F.conv2d(xc, w, b, s, p), a.iters) / 1e9, 1)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
