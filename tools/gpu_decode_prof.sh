#!/bin/bash
# kernel-trace profile of graph decode (LLaMA3-8B, B=1) and a GEMV-vs-hipBLASLt probe on
# weights rotated through > 1 GB (so the 256 MB Infinity Cache cannot serve them)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_decode -o run --output-format csv -- python bench/decode.py --prompt 1024 --new 64 --graph > gpurun_out/prof_decode.log 2>&1 || exit 1
grep metric gpurun_out/prof_decode.log
timeout -k 10 150 python - > gpurun_out/gemv_probe.log 2>&1 <<'EOF' || exit 2
import torch
from solvingpapers_amd.ops import _ext
torch.manual_seed(0)
def t(fn, ws, n=40):
    for i in range(4): fn(ws[i % len(ws)])
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(); e0.record()
    for i in range(n): fn(ws[i % len(ws)])
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e-3
for (N, K) in [(6144, 4096), (4096, 4096), (28672, 4096), (4096, 14336), (128256, 4096)]:
    nb = max(2, (1 << 30) // (N * K * 2) + 1)
    ws = [torch.randn(N, K, device="cuda", dtype=torch.bfloat16) for _ in range(nb)]
    for M in (1, 4):
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        dm = t(lambda w: torch.mm(x, w.t()), ws)
        dg = t(lambda w: _ext.ops().gemv(x, w), ws)
        print(f"M={M} N={N:6d} K={K:5d}: hipBLASLt {dm*1e6:7.1f} us {N*K*2/dm/1e12:5.2f} TB/s | "
              f"gemv {dg*1e6:7.1f} us {N*K*2/dg/1e12:5.2f} TB/s", flush=True)
    del ws
EOF
cat gpurun_out/gemv_probe.log
