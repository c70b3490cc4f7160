"""Probe: hipBLASLt fp8 GEMMs through torch._scaled_mm on this ROCm build (tensorwise and
rowwise scales), timed against bf16 torch.mm at DeepSeek-V3 projection shapes."""
import json
import torch


def tm(fn, it=10):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it


for M, N, K in ((4096, 24576, 1536), (4096, 7168, 16384), (4096, 32768, 512), (8192, 8192, 8192)):
    a = torch.randn(M, K, device="cuda").bfloat16()
    b = torch.randn(N, K, device="cuda").bfloat16()
    row = {"M": M, "N": N, "K": K}
    fl = 2.0 * M * N * K
    row["bf16_TF"] = round(fl / tm(lambda: torch.mm(a, b.t())) / 1e9)
    a8 = a.to(torch.float8_e4m3fn)
    b8 = b.to(torch.float8_e4m3fn)
    one = torch.ones((), device="cuda")
    try:
        row["fp8_tensorwise_TF"] = round(fl / tm(lambda: torch._scaled_mm(a8, b8.t(), one, one, out_dtype=torch.bfloat16)) / 1e9)
    except Exception as ex:  # noqa: BLE001
        row["fp8_tensorwise"] = str(ex)[:120]
    sa = torch.ones(M, 1, device="cuda")
    sb = torch.ones(1, N, device="cuda")
    try:
        row["fp8_rowwise_TF"] = round(fl / tm(lambda: torch._scaled_mm(a8, b8.t(), sa, sb, out_dtype=torch.bfloat16)) / 1e9)
    except Exception as ex:  # noqa: BLE001
        row["fp8_rowwise"] = str(ex)[:120]
    print(json.dumps(row), flush=True)
