"""Weight-gradient operand layouts at LLaMA3-8B shapes (T = 8192), one GEMM per form:

  both   dW = dYt @ Xt^T    both operands transposed to token-contiguous rows (current path)
  dy     dW = dYt @ X       only dY transposed (the dgrad-like NN form)
  x      dW = dY^T @ Xt^T   only X transposed
  direct dW = dY^T @ X      no transpose (hipBLASLt's slow form on gfx950)
  wgrad8 dW = dY^T @ X      csrc/kernels/gemm8.hip token-major path, split over tokens, fp32 partials

Prints GEMM time, transpose time (csrc/kernels/layout.hip) and the sum per form.
    python tools/bench_wgrad_layouts.py [--tune OUT.csv] [--vit]
--tune lets TunableOp search hipBLASLt + rocBLAS for every form's shape first (results to OUT.csv).
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from solvingpapers_amd.ops import _ext  # noqa: E402
from solvingpapers_amd.ops.layout import transpose2d  # noqa: E402
from solvingpapers_amd.utils.tuning import load_gemm_tuning  # noqa: E402

T = 8192
shapes = {"wqkv": (6144, 4096), "wo": (4096, 4096), "w13": (28672, 4096), "w2": (4096, 14336)}
if "--vit" in sys.argv:   # ViT-B/16 at batch 256: 256 x 197 tokens
    T = 256 * 197
    shapes = {"qkv": (2304, 768), "proj": (768, 768), "fc1": (3072, 768), "fc2": (768, 3072)}


def tm(fn, it=20):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(it):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / it * 1e3


def main():
    tune = sys.argv[sys.argv.index("--tune") + 1] if "--tune" in sys.argv else None
    print("table loaded:", load_gemm_tuning(), flush=True)
    if tune:
        import torch.cuda.tunable as tunable
        os.environ.setdefault("PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS", "15")
        tunable.tuning_enable(True)
        tunable.set_filename(tune, False)
    for name, (N, K) in shapes.items():
        x = torch.randn(T, K, device="cuda", dtype=torch.bfloat16)
        dy = torch.randn(T, N, device="cuda", dtype=torch.bfloat16)
        out = torch.empty(N, K, device="cuda", dtype=torch.bfloat16)
        dyT, xT = transpose2d(dy), transpose2d(x)
        fl = 2 * T * N * K
        forms = {
            "both": (lambda: torch.mm(dyT, xT.t(), out=out), lambda: (transpose2d(dy), transpose2d(x))),
            "dy": (lambda: torch.mm(dyT, x, out=out), lambda: transpose2d(dy)),
            "x": (lambda: torch.mm(dy.t(), xT.t(), out=out), lambda: transpose2d(x)),
            "direct": (lambda: torch.mm(dy.t(), x, out=out), None),
            "wgrad8": (lambda: _ext.ops().wgrad8(dy, x, out, False, 0), None),
            # accumulating into the gradient (micro-batches 2.. of a step): out += ...
            "both+a": (lambda: out.addmm_(dyT, xT.t()), lambda: (transpose2d(dy), transpose2d(x))),
            "dy+a": (lambda: out.addmm_(dyT, x), lambda: transpose2d(dy)),
            "x+a": (lambda: out.addmm_(dy.t(), xT.t()), lambda: transpose2d(x)),
            "direct+a": (lambda: out.addmm_(dy.t(), x), None),
        }

        ref = torch.mm(dy.t(), x)
        for f, (g, tr) in forms.items():
            if tune:
                print(f"  tuning {name}/{f} ...", flush=True)
            if f.endswith("+a"):
                out.zero_()
            g()
            assert torch.allclose(out.float(), ref.float(), atol=1e-1, rtol=2e-2), (name, f)
            tg = tm(g)
            tt = tm(tr) if tr is not None else 0.0
            print(f"{name:5s} {f:6s} gemm {tg:.3f} ms ({fl / tg / 1e9:.0f} TF)  transposes {tt:.3f} ms"
                  f"  total {tg + tt:.3f} ms", flush=True)
    if tune:
        tunable.write_file()


if __name__ == "__main__":
    main()
