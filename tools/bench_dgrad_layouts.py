"""dgrad formulations at LLaMA3-8B shapes (T = 8192): dX = dY W as hipBLASLt's NN form (W [N, K]
read K-strided) vs the NT form on a transposed weight copy (W^T [K, N], K-contiguous like the
forward's operands), ABBA-timed with the shipped GEMM table loaded."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from solvingpapers_amd.utils.tuning import load_gemm_tuning  # noqa: E402

T = 8192
shapes = {"wqkv": (6144, 4096), "wo": (4096, 4096), "w13": (28672, 4096), "w2": (4096, 14336),
          "head": (128256, 4096)}


def tm(fn, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(it):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / it


print("table loaded:", load_gemm_tuning(None))
for name, (N, K) in shapes.items():
    dy = torch.randn(T, N, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02
    wt = w.t().contiguous()
    fl = 2 * T * N * K
    nn = lambda: torch.mm(dy, w)          # noqa: E731
    nt = lambda: torch.mm(dy, wt.t())     # noqa: E731
    a1, b1, b2, a2 = tm(nn), tm(nt), tm(nt), tm(nn)
    tnn, tnt = (a1 + a2) / 2, (b1 + b2) / 2
    ttr = tm(lambda: w.t().contiguous())
    print(f"{name}: NN {fl / tnn / 1e12:.0f} TF ({tnn * 1e3:.3f} ms) | NT on W^T {fl / tnt / 1e12:.0f} TF "
          f"({tnt * 1e3:.3f} ms) | transpose W {ttr * 1e3:.3f} ms", flush=True)
