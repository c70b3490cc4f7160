"""Per-tile segment cycles of the 8-phase GEMM (gemm8.hip) from its s_memtime stamp build:
    tools/build_variant.sh g8st -DSPA_G8_STAMP=1
    SPA_EXT_SO=ab/_C_g8st.so python tools/g8_stamps.py
For each case (the dsv3_style expert GEMMs and a dense K = 768 control) one launch is stamped and
the blocks' mean cycles are printed per segment: tile mapping (kernel entry to the first DMA
issue), prologue (first DMA issued to the first two K-tiles landed), K-loop, epilogue (through
the stores' completion), with the K-loop's cycles per K-tile for comparison."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from solvingpapers_amd.ops import _ext  # noqa: E402
from solvingpapers_amd.ops import moe as M  # noqa: E402

ops = _ext.ops()
assert ops.g8_stamps().numel() > 0, "load the stamp build: SPA_EXT_SO=ab/_C_g8st.so"
dev = "cuda"
torch.manual_seed(0)
T, E, k, D, F = 8192, 64, 6, 2048, 1408
idx, _ = M.route(torch.randn(T, E, device=dev), k)
plan = M.permute(idx, E)
A = T * k
x = torch.randn(A, D, device=dev, dtype=torch.bfloat16)
W13 = torch.randn(E, 2 * F, D, device=dev, dtype=torch.bfloat16) * 0.02
dy13 = torch.randn(A, 2 * F, device=dev, dtype=torch.bfloat16)
MN, K = 8192, 768
xa = torch.randn(MN, K, device=dev, dtype=torch.bfloat16)
wa = torch.randn(1, MN, K, device=dev, dtype=torch.bfloat16)
ta = torch.randn(K, MN, device=dev, dtype=torch.bfloat16)
off1 = torch.tensor([0, MN], dtype=torch.int32, device=dev)
offk = torch.tensor([0, K], dtype=torch.int32, device=dev)
cases = {
    "fwd W13 (K 2048)": lambda: ops.grouped_gemm8(x, W13, plan.offsets, 0, None, False),
    "dX W13 (K 2816)": lambda: ops.grouped_gemm8(dy13, W13, plan.offsets, 1, None, False),
    "dW W13 (K ~768)": lambda: ops.grouped_gemm8(dy13, x, plan.offsets, 2, None, False),
    "dW W13 accumulate": lambda: ops.grouped_gemm8(dy13, x, plan.offsets, 2, out_acc, True),
    "dense fwd K 768": lambda: ops.grouped_gemm8(xa, wa, off1, 0, None, False),
    "dense dW K 768": lambda: ops.grouped_gemm8(ta, ta, offk, 2, None, False),
}
# ViT-B/16 weight gradients (wgrad8: token slices of one dense dW, fp32 partials), T = 256 x 197
Tv = 256 * 197
vit = {}
for nm, (n_, k_) in {"qkv": (2304, 768), "proj": (768, 768), "fc1": (3072, 768), "fc2": (768, 3072)}.items():
    dyv = torch.randn(Tv, n_, device=dev, dtype=torch.bfloat16)
    xv = torch.randn(Tv, k_, device=dev, dtype=torch.bfloat16)
    vit[nm] = (dyv, xv)
for nm, (dyv, xv) in vit.items():
    cases[f"ViT wgrad8 {nm}"] = (lambda d=dyv, xx=xv: ops.wgrad8(d, xx, None, False, 0))
out_acc = ops.grouped_gemm8(dy13, x, plan.offsets, 2, None, False)
for name, fn in cases.items():
    for _ in range(3):
        fn()
    ops.g8_stamps()                     # read-and-clear: only the next launch's blocks stay live
    fn()
    st = ops.g8_stamps().double()
    live = st[:, 4] > 0
    st = st[live]
    kt = st[:, 4]
    seg = st[:, :4].mean(0).tolist()
    per_k = (st[:, 2] / kt).mean().item()
    tot = sum(seg)
    print(f"{name:20s} blocks {int(live.sum()):5d}  mean K-tiles {kt.mean().item():5.1f} | mapping {seg[0]:7.0f}  "
          f"prologue {seg[1]:7.0f}  K-loop {seg[2]:8.0f} ({per_k:5.0f}/K-tile)  epilogue {seg[3]:7.0f} cycles | "
          f"outside the K-loop {100 * (tot - seg[2]) / tot:4.1f} %", flush=True)
