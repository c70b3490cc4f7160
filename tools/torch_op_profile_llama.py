"""Which framework ops launch the non-GEMM glue kernels (fills, copies, casts, adds) of the
headline step: torch.profiler over one accumulated LLaMA3-8B-width step (bench.py's loop, fewer
layers), aten ops only, sorted by device time, with input shapes.
    python tools/torch_op_profile_llama.py [--layers 4] [--rows 40]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from solvingpapers_amd.models import llama3  # noqa: E402
from solvingpapers_amd.train.optim import FlatAdamW  # noqa: E402
from solvingpapers_amd.utils.flat import FlatParams  # noqa: E402
from solvingpapers_amd.utils.tuning import load_gemm_tuning  # noqa: E402


def main():
    layers = int(sys.argv[sys.argv.index("--layers") + 1]) if "--layers" in sys.argv else 4
    rows = int(sys.argv[sys.argv.index("--rows") + 1]) if "--rows" in sys.argv else 40
    load_gemm_tuning(None)
    c = llama3.config("llama3_8b", max_seq_len=8192, n_layers=layers)
    m = llama3.Llama3(c, device="cuda", dtype=torch.bfloat16, seed=1)
    flat = FlatParams(m, groups=m.param_groups(), grad_dtype=torch.bfloat16)
    opt = FlatAdamW(flat, lr=3e-4, betas=(0.9, 0.95), eps=1e-8, weight_decay=0.1, max_grad_norm=1.0)
    m.param_wait_cb = flat.wait_bucket
    t = torch.randint(0, c.vocab_size, (1, 8193), device="cuda")

    def step():
        opt.zero_grad()
        for _ in range(4):
            loss = m(t[:, :-1], t[:, 1:]) / 4
            loss.backward()
        opt.step(overlap=True)

    for _ in range(2):
        step()
    torch.cuda.synchronize()
    acts = [torch.profiler.ProfilerActivity.CPU, torch.profiler.ProfilerActivity.CUDA]
    with torch.profiler.profile(activities=acts, record_shapes=True) as prof:
        step()
        torch.cuda.synchronize()
    avg = [e for e in prof.key_averages(group_by_input_shape=True) if e.key.startswith("aten::")]
    avg.sort(key=lambda e: -e.self_device_time_total)
    print(f"{'op':32s} {'calls':>6s} {'self device ms':>15s}  input shapes")
    for e in avg[:rows]:
        print(f"{e.key[:32]:32s} {e.count:6d} {e.self_device_time_total / 1e3:15.3f}  {str(e.input_shapes)[:150]}")


if __name__ == "__main__":
    main()
