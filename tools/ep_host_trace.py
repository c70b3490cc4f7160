"""Host-side cost of one expert-parallel MoE layer: 2 EP ranks sharing
cuda:0 over gloo (the 1-GPU rehearsal), DeepSeek-V2-Lite expert widths (D 2048, 64 experts,
top-6, F 1408), 4096 tokens per rank. torch.profiler records the CPU side of every op in
``ep_moe_ffn`` (rank 0 writes a chrome trace + a per-op table): the dispatch builds its
(source, expert) regroup on the device (csrc/kernels/ep.hip) and the only host sync is one
D2H copy of the 2*E split counts per layer.

usage: python tools/ep_host_trace.py [out_dir]
"""
import json
import os
import socket
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), SPA_DIST_BACKEND="gloo")
    from solvingpapers_amd.parallel import dist as sdist
    sdist.init_distributed()
    import torch.distributed as dist
    from solvingpapers_amd.models import deepseekv3 as ds
    c = ds.config("dsv3_style", n_experts=64, top_k=6, n_shared=2, expert_hidden=1408, aux_free=False)
    grp = dist.new_group([0, 1])
    m = ds.MoE(c, ep_group=grp, device="cuda:0", dtype=torch.bfloat16)
    m.reset_parameters(0.02, torch.Generator(device="cuda:0").manual_seed(3))
    g = torch.Generator(device="cuda:0").manual_seed(rank)
    x = torch.randn(1, 4096, c.dim, device="cuda:0", dtype=torch.bfloat16, generator=g).requires_grad_(True)

    def step():
        y = m(x)
        y.float().sum().backward()

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    dist.barrier(grp)
    t0 = time.perf_counter()
    n = 5
    for _ in range(n):
        step()
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / n * 1e3
    acts = [torch.profiler.ProfilerActivity.CPU]
    with torch.profiler.profile(activities=acts, record_shapes=False) as prof:
        for _ in range(2):
            with torch.profiler.record_function("moe_layer_fwd_bwd"):
                step()
        torch.cuda.synchronize()
    if rank == 0:
        os.makedirs(out_dir, exist_ok=True)
        prof.export_chrome_trace(os.path.join(out_dir, "ep_moe_layer_host_trace.json"))
        tab = prof.key_averages().table(sort_by="self_cpu_time_total", row_limit=25)
        with open(os.path.join(out_dir, "ep_moe_layer_host_ops.txt"), "w") as f:
            f.write(tab)
        ev = [e for e in prof.key_averages() if e.key == "moe_layer_fwd_bwd"]
        host_ms = ev[0].cpu_time_total / ev[0].count / 1e3 if ev else None
        print(json.dumps({"ep": world, "backend": "gloo (1-GPU rehearsal)", "tokens_per_rank": 4096,
                          "experts": 64, "top_k": 6, "wall_ms_per_layer_fwd_bwd": round(wall, 2),
                          "host_cpu_ms_per_layer_fwd_bwd": round(host_ms, 2) if host_ms else None}), flush=True)
    sdist.cleanup()


if __name__ == "__main__":
    out = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/ep_trace"
    mp.spawn(worker, args=(2, _port(), out), nprocs=2, join=True)
