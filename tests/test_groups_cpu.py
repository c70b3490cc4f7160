"""DP x TP and DP x EP through the real training entry point.

``python -m solvingpapers_amd.train gemma --tp 2`` and ``... dsv3 --ep 2`` on a 4-rank gloo
world (torch.distributed.run on CPU): the ProcessGroups layout (parallel/groups.py), data
sharded by the data coordinate, replicas that must stay identical do, checkpoints carry the
layout, and a run resumed from a mid-run checkpoint ends bit-identical to a straight run.
"""
import json
import os
import socket
import subprocess
import sys

import pytest
import torch

from solvingpapers_amd.parallel.groups import layout_ranks

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_layout_ranks_partitions():
    lay = layout_ranks(8, tp=2, ep=2)
    assert lay["tp"] == [[0, 1], [2, 3], [4, 5], [6, 7]]
    assert lay["dp"] == [[0, 2, 4, 6], [1, 3, 5, 7]]
    assert lay["ep"] == [[0, 2], [4, 6], [1, 3], [5, 7]]
    assert lay["expert_dp"] == [[0, 4], [2, 6], [1, 5], [3, 7]]
    for kind, groups in lay.items():                     # every kind partitions the world
        assert sorted(r for g in groups for r in g) == list(range(8)), kind
    lay = layout_ranks(8, tp=1, ep=8)
    assert lay["ep"] == [list(range(8))] and lay["expert_dp"] == [[r] for r in range(8)]
    with pytest.raises(ValueError):
        layout_ranks(8, tp=3)
    with pytest.raises(ValueError):
        layout_ranks(8, tp=2, ep=3)


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _torchrun(nproc, args):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(SPA_DIST_BACKEND="gloo", CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr=127.0.0.1", f"--master-port={_port()}", "-m", "solvingpapers_amd.train", *args]
    r = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    return [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]


def _final(d, nproc):
    with open(os.path.join(d, "latest")) as f:
        step_dir = os.path.join(d, f.read().strip())
    return [torch.load(os.path.join(step_dir, f"rank{r:05d}.pt"), weights_only=True) for r in range(nproc)]


CASES = {
    "gemma_dp2_tp2": ["gemma", "--preset", "gemma_tiny", "--tp", "2", "--no-sp", "--set", "vocab_size=256", "--set", "dim=64",
                      "--set", "n_heads=4", "--set", "head_dim=16", "--set", "ffn_hidden=128"],
    "gemma_dp2_tp2_sp": ["gemma", "--preset", "gemma_tiny", "--tp", "2", "--sp", "--set", "vocab_size=256", "--set",
                         "dim=64", "--set", "n_heads=4", "--set", "head_dim=16", "--set", "ffn_hidden=128"],
    # even --accum under SP: the Trainer runs the micro-batches as Gemma.forward_pair
    "gemma_dp2_tp2_sp_pairs": ["gemma", "--preset", "gemma_tiny", "--tp", "2", "--sp", "--accum", "2", "--set",
                               "vocab_size=256", "--set", "dim=64", "--set", "n_heads=4", "--set", "head_dim=16",
                               "--set", "ffn_hidden=128"],
    "dsv3_dp4_ep2": ["dsv3", "--preset", "dsv3_tiny", "--ep", "2", "--set", "vocab_size=256", "--set", "dim=64",
                     "--set", "n_heads=2", "--set", "expert_hidden=32", "--set", "dense_hidden=128",
                     "--set", "kv_lora_rank=32", "--set", "qk_nope_dim=16", "--set", "qk_rope_dim=16",
                     "--set", "v_head_dim=16", "--set", "mtp_heads=0"],
}


@pytest.mark.parametrize("case", list(CASES))
def test_cli_parallel_layouts_train_and_resume(case, tmp_path):
    base = CASES[case] + ["--device", "cpu", "--seq", "16", "--batch", "2", "--lr", "1e-3", "--ckpt-every", "2"]
    straight = _torchrun(4, base + ["--steps", "4", "--ckpt-dir", str(tmp_path / "a")])
    assert [r["step"] for r in straight if "loss" in r] == [0, 1, 2, 3]
    _torchrun(4, base + ["--steps", "2", "--ckpt-dir", str(tmp_path / "b")])
    resumed = _torchrun(4, base + ["--steps", "4", "--ckpt-dir", str(tmp_path / "b")])
    assert [r["step"] for r in resumed if "loss" in r] == [2, 3]
    a, b = _final(str(tmp_path / "a"), 4), _final(str(tmp_path / "b"), 4)
    for r in range(4):
        assert torch.equal(a[r]["param"], b[r]["param"]), r          # resume is bit-exact per rank
        assert a[r]["extra"]["layout"] == {"world": 4, "tp": 2 if "tp" in case else 1,
                                           "ep": 2 if "ep" in case else 1, "dp": 2 if "tp" in case else 4}
    if "tp" in case:
        # ranks 0/2 and 1/3 hold the same TP shard in different DP replicas
        assert torch.equal(a[0]["param"], a[2]["param"]) and torch.equal(a[1]["param"], a[3]["param"])
        assert not torch.equal(a[0]["param"], a[1]["param"])
    else:
        # EP groups {0,1} {2,3}: ranks 0/2 hold the same experts (expert-DP replicas)
        assert torch.equal(a[0]["param"], a[2]["param"]) and torch.equal(a[1]["param"], a[3]["param"])
        assert not torch.equal(a[0]["param"], a[1]["param"])
