"""Multi-GPU pre-flight on one GPU: the real benches, at reduced depth,
under a 1-rank ``torch.distributed.run`` with SPA_FORCE_COLLECTIVES=1, so their DP buckets
(LLaMA widths, both DP reductions, ZeRO-1) and the EP fp8 dispatch at dsv3 widths go through
librccl exactly as an N-rank launch does. Full-depth numbers: profiles/r6_rccl_preflight.txt.
Plus the device shard sum of the a2a DP reduction against an fp32 oracle."""
import json
import os
import socket
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _launch(script, args, extra_env=None, timeout=240):
    env = dict(os.environ, SPA_FORCE_COLLECTIVES="1", PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""))
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.update(extra_env or {})
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr=127.0.0.1", f"--master-port={_port()}", os.path.join(ROOT, script), *args]
    r = subprocess.run(cmd, env=env, cwd=ROOT, timeout=timeout, capture_output=True, text=True)
    print(r.stdout[-3000:])
    print(r.stderr[-3000:], file=sys.stderr)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = []
    for l in r.stdout.splitlines():
        if l.startswith("{"):
            try:
                lines.append(json.loads(l))
            except ValueError:            # a diagnostic dict print, not the result line
                pass
    assert lines, r.stdout[-2000:]
    return lines[-1]


@pytest.mark.parametrize("extra,env", [([], {}), ([], {"SPA_DP_REDUCE": "ring"}), (["--zero1"], {})])
def test_bench_llama8b_widths_through_rccl_world1(extra, env):
    out = _launch("bench.py", ["--layers", "2", "--seq", "2048", "--steps", "2", "--warmup", "1", *extra], env)
    assert out["backend"] == "nccl" and out["world_size"] == 1
    assert "forced-collectives" in out["config"]["parallelism"]
    assert out["value"] > 0 and out["loss"] == out["loss"]          # finite


def test_dsv3_v3_fp8_ep_dispatch_through_rccl_world1():
    out = _launch("bench/dsv3_train.py", ["--preset", "dsv3_v3", "--layers", "2", "--experts", "8",
                                          "--dense-layers", "1", "--seq", "1024", "--mb", "1", "--fp8",
                                          "--steps", "2", "--warmup", "1", "--gemm-table", "none"])
    assert "forced-collectives" in out["config"]["parallelism"]
    assert out["value"] > 0 and out["loss"] == out["loss"]


def test_ep_rccl_live_memory_flat_across_microbatches():
    """Regression (profiles/r6_ep_memory.txt): through a real RCCL group the EP exchanges' Work objects
    used to stay referenced after wait() and pinned ~3 GB per MoE layer and micro-batch."""
    out = _launch("tools/ep_mem_probe.py", ["--check", "--seq", "2048"])
    for a in out["arms"]:
        assert a["arm"] == "ep-forced"
        assert abs(a["growth_gb"]) < 0.05, out
        assert a["live_boxes"] == 0, out


@pytest.mark.parametrize("N,n", [(1, 4096), (8, 1 << 20), (8, 1000 + 3), (4, 8 * 7919)])
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
def test_shard_sum_matches_fp32(N, n, dt):
    from solvingpapers_amd.ops._ext import ops
    g = torch.Generator(device="cuda").manual_seed(N * n)
    x = torch.randn(N * n, device="cuda", generator=g).to(dt)
    out = torch.empty(n, device="cuda", dtype=dt)
    ops().shard_sum_(out, x, N, 1.0 / N)
    want = x.view(N, n).double().sum(0) / N
    err = (out.double() - want).abs().max().item()
    tol = 0 if dt == torch.float32 and N == 1 else (1e-5 if dt == torch.float32 else 1e-2)
    assert err <= tol * max(1.0, want.abs().max().item()), err
    if dt == torch.bfloat16:   # one rounding of the fp32 sum: within half a bf16 ulp of the exact mean
        assert ((out.double() - want).abs() <= want.abs() * 2.0 ** -8 + 1e-30).all()
