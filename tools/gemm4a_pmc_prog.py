"""A short program for rocprofv3 --pmc: dense 8192^3 bf16 on gemm4a (register-staged), gemm8 and
hipBLASLt, a few dispatches each (random operands), so the counter passes compare the three kernels
on identical work. tools/gpu_tasks.sh g4pmc."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from solvingpapers_amd.ops import _ext

ops = _ext.ops()
S = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
x = torch.rand(S, S, device="cuda").sub_(0.5).bfloat16()
w = torch.rand(1, S, S, device="cuda").sub_(0.5).bfloat16()
off = torch.tensor([0, S], dtype=torch.int32, device="cuda")
for _ in range(3):
    ops.gemm4a(x, w, off, 0, None)
    ops.grouped_gemm8(x, w, off, 0, None, False)
    torch.mm(x, w[0].t())
torch.cuda.synchronize()
print("done")
