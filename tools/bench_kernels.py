"""Per-kernel timing of the hand-written memory-bound / small-op kernels at the north-star shapes,
as achieved HBM bandwidth (ideal bytes / time). Run under ``rocprofv3 --pmc`` for counters.

usage: python tools/bench_kernels.py [--iters N] [--only name,name]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from solvingpapers_amd.ops import _ext  # noqa: E402
from solvingpapers_amd import ops as O  # noqa: E402
from solvingpapers_amd.ops import misc, optim_kernels  # noqa: E402

DEV = "cuda"
BF = torch.bfloat16


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


def cases():
    g = torch.Generator(device=DEV).manual_seed(0)

    def rn(*shape, dtype=BF, req=False):
        return torch.randn(*shape, device=DEV, dtype=dtype, generator=g).requires_grad_(req)

    N, D = 8192, 4096                                       # LLaMA3-8B rows x width
    x, w = rn(N, D), torch.ones(D, device=DEV, dtype=BF)
    out = {}
    out["rmsnorm_fwd_8192x4096"] = (lambda: O.rms_norm(x, w, 1e-5), 2 * N * D * 2)
    xr, wr = rn(N, D, req=True), torch.ones(D, device=DEV, dtype=BF, requires_grad=True)
    yr = O.rms_norm(xr, wr, 1e-5)
    dy = rn(N, D)
    out["rmsnorm_bwd_8192x4096"] = (lambda: torch.autograd.grad(yr, (xr, wr), dy, retain_graph=True),
                                    3 * N * D * 2)
    _, hn, rstd, _ = _ext.ops().norm_fwd(x, None, w, None, 1e-5)
    out["rmsnorm_bwd_kernel_8192x4096"] = (lambda: _ext.ops().norm_bwd(dy, x, w, rstd, None, None, None, None),
                                           3 * N * D * 2)
    Nv, Dv = 256 * 197, 768                                 # ViT-B/16 batch 256
    xl, wl, bl = rn(Nv, Dv), torch.ones(Dv, device=DEV, dtype=BF), torch.zeros(Dv, device=DEV, dtype=BF)
    out["layernorm_fwd_50432x768"] = (lambda: O.layer_norm(xl, wl, bl), 2 * Nv * Dv * 2)
    F = 14336
    gu = rn(N, 2 * F)
    out["swiglu_fwd_8192x14336"] = (lambda: O.swiglu(gu), 3 * N * F * 2)
    gug = rn(4096, 2 * 24576)
    out["geglu_fwd_4096x24576"] = (lambda: O.geglu(gug), 3 * 4096 * 24576 * 2)
    qkv = rn(1, N, 48, 128)                                 # 32 q + 8 k + 8 v heads
    out["rope_qk_inplace_8192x40x128"] = (lambda: O.rope_packed_(qkv, 40, 500000.0), 2 * N * 40 * 128 * 2)
    V = 128256
    logits = rn(N, V)
    tgt = torch.randint(0, V, (N,), device=DEV, generator=g)
    out["xent_fwd_8192x128256"] = (lambda: O.cross_entropy(logits, tgt), N * V * 2)
    emb = rn(V, D)
    ids = torch.randint(0, V, (1, N), device=DEV, generator=g)
    out["embedding_fwd_8192x4096"] = (lambda: O.embedding(emb, ids), 2 * N * D * 2)
    n = 1 << 28                                             # 268M-param AdamW slice (bf16 p, fp32 master/m/v, bf16 g)
    p = torch.zeros(n, device=DEV, dtype=BF)
    mst, m, v = (torch.zeros(n, device=DEV) for _ in range(3))
    gr = torch.full((n,), 1e-3, device=DEV, dtype=BF)
    out["adamw_268M"] = (lambda: optim_kernels.adamw_(p, mst, gr, m, v, 3e-4, 0.9, 0.95, 1e-8, 0.1, 1),
                         n * (2 + 2 + 3 * 4 * 2 + 2))
    mb, vb = (torch.zeros(n, device=DEV, dtype=BF) for _ in range(2))   # bf16 moments (DeepSeek benches)
    out["adamw_268M_bf16mom"] = (lambda: optim_kernels.adamw_(p, mst, gr, mb, vb, 3e-4, 0.9, 0.95, 1e-8, 0.1, 1),
                                 n * (2 + 2 + 4 * 2 + 2 * 2 * 2))
    out["sqsum_268M_bf16"] = (lambda: optim_kernels.sqsum(gr),
                              n * 2)
    s, t = rn(16384, 1000, dtype=torch.float32), rn(16384, 1000, dtype=torch.float32)
    y = torch.randint(0, 1000, (16384,), device=DEV, generator=g)
    out["kd_loss_16384x1000"] = (lambda: misc.distillation_loss(s, t, y, 7.0, 0.3), 2 * 16384 * 1000 * 4)
    sb, tb = rn(65536, 10), rn(65536, 10)                   # reference shape: CIFAR-10 logits, big batch
    yb = torch.randint(0, 10, (65536,), device=DEV, generator=g)
    out["kd_loss_grad_65536x10_bf16"] = (lambda: _ext.ops().kd_loss_fwd(sb, tb, yb, 7.0, 0.3, True), 3 * 65536 * 10 * 2)
    out["kd_loss_grad_16384x1000"] = (lambda: _ext.ops().kd_loss_fwd(s, t, y, 7.0, 0.3, True), 3 * 16384 * 1000 * 4)
    xd = rn(N, D)
    out["dropout_8192x4096"] = (lambda: misc.dropout(xd, 0.1, True), 2 * N * D * 2)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    assert _ext.load(), "HIP extension missing"
    only = set(filter(None, a.only.split(",")))
    for name, (fn, nbytes) in cases().items():
        if only and name not in only:
            continue
        ms = timed(fn, a.iters)
        print(json.dumps({"kernel": name, "ms": round(ms, 4), "GB": round(nbytes / 1e9, 3),
                          "TB_per_s": round(nbytes / ms / 1e9, 2)}), flush=True)


if __name__ == "__main__":
    main()
