"""wgrad formulations at LLaMA3-8B shapes (T=8192): hipBLASLt TN (dy^T x) vs transposing both
operands to K-contiguous first and running the NT (fwd-style) kernel."""
import time
import torch

T = 8192
shapes = {"wqkv": (6144, 4096), "wo": (4096, 4096), "w13": (28672, 4096), "w2": (4096, 14336)}


def tm(fn, it=10):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(it):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / it


for name, (N, K) in shapes.items():
    x = torch.randn(T, K, device="cuda", dtype=torch.bfloat16)
    dy = torch.randn(T, N, device="cuda", dtype=torch.bfloat16)
    out = torch.empty(N, K, device="cuda", dtype=torch.bfloat16)
    dyT = dy.t().contiguous()
    xT = x.t().contiguous()
    fl = 2 * T * N * K
    t_tn = tm(lambda: torch.mm(dy.t(), x, out=out))
    t_nt = tm(lambda: torch.mm(dyT, xT.t(), out=out))
    t_tr = tm(lambda: (dy.t().contiguous(), x.t().contiguous()))
    print(f"{name}: TN {fl / t_tn / 1e12:.0f} TF ({t_tn*1e3:.3f} ms) | NT-only {fl / t_nt / 1e12:.0f} TF ({t_nt*1e3:.3f} ms)"
          f" | torch transposes {t_tr*1e3:.3f} ms", flush=True)
