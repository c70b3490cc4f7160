#!/bin/bash
# kernel-trace profile of graph decode (LLaMA3-8B, B=1) and a GEMV-shape probe
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_decode -o run --output-format csv -- python bench/decode.py --prompt 1024 --new 64 --graph > gpurun_out/prof_decode.log 2>&1 || exit 1
grep metric gpurun_out/prof_decode.log
timeout -k 10 120 python - > gpurun_out/gemv_probe.log 2>&1 <<'EOF' || exit 2
import torch, time
torch.manual_seed(0)
def t(fn, n=50):
    for _ in range(5): fn()
    torch.cuda.synchronize(); s = time.perf_counter()
    for _ in range(n): fn()
    torch.cuda.synchronize(); return (time.perf_counter() - s) / n
for (N, K) in [(6144, 4096), (4096, 4096), (28672, 4096), (4096, 14336), (128256, 4096)]:
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)
    for M in (1, 16):
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        dt = t(lambda: torch.mm(x, w.t()))
        print(f"M={M:3d} N={N:6d} K={K:5d}: {dt*1e6:8.1f} us  {N*K*2/dt/1e9:7.0f} GB/s weights", flush=True)
EOF
cat gpurun_out/gemv_probe.log
