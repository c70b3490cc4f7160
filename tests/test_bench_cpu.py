"""bench.py launch contract (VERDICT r1 'what's weak' #1): ``python bench.py --gpus N`` with no
WORLD_SIZE in the environment must start N ranks itself (torch.distributed.run as a child
process, never an exec) and report ``n_gpus`` from the live process group. Rehearsed on
CPU with the gloo backend and a tiny LLaMA shape."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run_bench(*extra, env_extra=None):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(SPA_DIST_BACKEND="gloo", CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS="2")
    env.update(env_extra or {})
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--model", "llama3_tiny", "--seq", "32", "--steps", "1",
           "--warmup", "0", "--accum", "1", *extra]
    r = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=600)
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    return r, lines


def test_bench_self_launches_two_ranks():
    r, lines = _run_bench("--gpus", "2")
    assert r.returncode == 0, r.stderr[-3000:]
    assert len(lines) == 1, r.stdout                     # rank 0 prints exactly one line
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["world_size"] == 2 and out["backend"] == "gloo"
    assert out["launcher"] == "bench.py self-launch"
    assert out["config"]["parallelism"] == "dp2" and out["config"]["global_batch"] == 2
    assert out["value"] > 0 and out["steps"] == 1
    for k in ("metric", "unit", "ms_per_step", "higher_is_better", "scaling", "vs_baseline", "dtype", "data"):
        assert k in out


def test_bench_single_rank_default():
    r, lines = _run_bench()
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 1 and out["world_size"] == 1 and out["launcher"] == "direct"


def test_bench_failing_rank_propagates_exit_code():
    # an unknown preset makes every rank raise: the parent must exit non-zero
    r, lines = _run_bench("--gpus", "2", "--model", "no_such_model")
    assert r.returncode != 0 and not lines
