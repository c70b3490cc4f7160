"""Which framework ops launch the non-GEMM kernels of a ViT-B/16 training step (batch 256):
torch.profiler over one fwd+bwd+AdamW step, ops by device time with input shapes, then the
forward-op stack of every elementwise add (to find where standalone adds come from).
    python tools/torch_op_profile_vit.py [--rows 40] [--mb 256]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from solvingpapers_amd.models import vit  # noqa: E402
from solvingpapers_amd.ops.xent import cross_entropy  # noqa: E402
from solvingpapers_amd.train.optim import FlatAdamW  # noqa: E402
from solvingpapers_amd.utils.flat import FlatParams  # noqa: E402


def main():
    rows = int(sys.argv[sys.argv.index("--rows") + 1]) if "--rows" in sys.argv else 40
    mb = int(sys.argv[sys.argv.index("--mb") + 1]) if "--mb" in sys.argv else 256
    c = vit.config("vit_b16")
    m = vit.ViT(c, device="cuda", dtype=torch.bfloat16)
    flat = FlatParams(m, groups=m.param_groups(), grad_dtype=torch.bfloat16)
    opt = FlatAdamW(flat, lr=1e-3, weight_decay=0.05, max_grad_norm=1.0)
    x = torch.randn(mb, 3, 224, 224, device="cuda", dtype=torch.bfloat16)
    y = torch.randint(0, 1000, (mb,), device="cuda")

    def step():
        opt.zero_grad()
        cross_entropy(m(x), y).backward()
        opt.step()
    for _ in range(2):
        step()
    torch.cuda.synchronize()
    acts = [torch.profiler.ProfilerActivity.CPU, torch.profiler.ProfilerActivity.CUDA]
    with torch.profiler.profile(activities=acts, record_shapes=True, with_stack=True) as prof:
        step()
        torch.cuda.synchronize()
    print(prof.key_averages(group_by_input_shape=True).table(sort_by="self_cuda_time_total", row_limit=rows,
                                                             max_name_column_width=60, max_shapes_column_width=70))
    print(prof.key_averages(group_by_stack_n=8).table(sort_by="self_cuda_time_total", row_limit=12,
                                                      max_name_column_width=60))
    # where each elementwise add sits: its chain of enclosing CPU ops (autograd node names
    # for the ones the engine runs while accumulating gradients)
    seen = {}
    for e in prof.events():
        if e.name in ("aten::add", "aten::add_") and e.device_type == torch.autograd.DeviceType.CPU:
            chain, p = [], e.cpu_parent
            while p is not None and len(chain) < 4:
                chain.append(p.name)
                p = p.cpu_parent
            k = (e.name, str(e.input_shapes), " <- ".join(chain), " <- ".join((e.stack or [])[:3]))
            seen[k] = seen.get(k, 0) + 1
    for k, n in sorted(seen.items(), key=lambda kv: -kv[1]):
        print(n, "x", *k)


if __name__ == "__main__":
    main()
