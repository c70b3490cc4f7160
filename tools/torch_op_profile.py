"""Which framework ops launch the non-GEMM "glue" kernels (fills, copies, casts, cats) of a
DeepSeek-V3-style training step: torch.profiler over one fwd+bwd+AdamW step, ops sorted by
device time with their input shapes.
    python tools/torch_op_profile.py [--fp8] [--rows 40] [--preset dsv3_style --mb 2] [--stack]
--stack: only aten ops, grouped by the framework frames that launched them."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from solvingpapers_amd.models import deepseekv3 as ds  # noqa: E402
from solvingpapers_amd.train.optim import FlatAdamW  # noqa: E402
from solvingpapers_amd.utils.flat import FlatParams  # noqa: E402


def main():
    fp8 = "--fp8" in sys.argv
    rows = int(sys.argv[sys.argv.index("--rows") + 1]) if "--rows" in sys.argv else 40
    preset = sys.argv[sys.argv.index("--preset") + 1] if "--preset" in sys.argv else "dsv3_v3"
    mb = int(sys.argv[sys.argv.index("--mb") + 1]) if "--mb" in sys.argv else 1
    kw = dict(n_layers=4, n_experts=32, n_dense_layers=1) if preset == "dsv3_v3" else {}
    c = ds.config(preset, block_size=4096, moe_fp8=fp8, fp8_linears=fp8, **kw)
    m = ds.DeepSeekV3(c, device="cuda", dtype=torch.bfloat16, seed=1)
    flat = FlatParams(m, groups=m.param_groups(), grad_dtype=torch.bfloat16)
    opt = FlatAdamW(flat, lr=3e-4, betas=(0.9, 0.95), weight_decay=0.1, max_grad_norm=1.0)
    for l in m.moe_layers():
        l.balance_group = None
    t = torch.randint(0, c.vocab_size, (mb, 4097), device="cuda")

    def step():
        opt.zero_grad()
        loss = m(t[:, :-1], t[:, 1:])
        loss.backward()
        opt.step()
    for _ in range(2):
        step()
    torch.cuda.synchronize()
    acts = [torch.profiler.ProfilerActivity.CPU, torch.profiler.ProfilerActivity.CUDA]
    stack = "--stack" in sys.argv
    with torch.profiler.profile(activities=acts, record_shapes=True, with_stack=stack) as prof:
        step()
        torch.cuda.synchronize()
    if stack:
        # the aten (non-HIP-extension) ops by device time, each with the framework frames that issued it
        ev = [e for e in prof.key_averages(group_by_stack_n=8) if e.key.startswith("aten::") and e.self_device_time_total > 0]
        ev.sort(key=lambda e: -e.self_device_time_total)
        for e in ev[:rows]:
            frames = [f for f in e.stack if "solvingpapers_amd" in f or "bench" in f][:4]
            print(f"{e.self_device_time_total / 1e3:8.3f} ms  {e.count:5d}x  {e.key}")
            for f in frames:
                print(f"            {f}")
        return
    print(prof.key_averages(group_by_input_shape=True).table(sort_by="self_cuda_time_total", row_limit=rows,
                                                             max_name_column_width=60, max_shapes_column_width=70))


if __name__ == "__main__":
    main()
