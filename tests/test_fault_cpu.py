"""Failure detection / elastic restart: a 2-rank gloo job under
``torchrun --max-restarts 1`` loses rank 1 abruptly in the middle of training
(``SPA_FAULT_STEP``: ``os._exit`` with no cleanup), the elastic agent tears the job down
and restarts it, the trainer auto-resumes from the last atomic checkpoint, and the
final parameters are bit-identical to an uninterrupted run (batches are a pure function
of (seed, rank, step), RNG and optimizer state are checkpointed)."""
import glob
import os
import socket
import subprocess
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(tmp, name, fault):
    ck = os.path.join(tmp, name)
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="1")
    for k in ("SPA_FAULT_STEP", "SPA_FAULT_RANK", "SPA_FAULT_MARKER"):
        env.pop(k, None)
    if fault:
        env.update(SPA_FAULT_STEP="6", SPA_FAULT_RANK="1", SPA_FAULT_MARKER=os.path.join(tmp, name + ".fault"))
    # dynamic c10d rendezvous: each restart round re-rendezvouses under a fresh round id
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "2",
           "--max-restarts", "1", "--rdzv-backend", "c10d", "--rdzv-endpoint", f"127.0.0.1:{_port()}",
           "--rdzv-id", f"spa-{name}-{os.getpid()}",
           "-m", "solvingpapers_amd.train", "llama3", "--preset", "llama3_ref", "--device", "cpu",
           "--set", "vocab_size=128", "--set", "dim=64", "--set", "ffn_hidden=128", "--set", "init='std'",
           "--batch", "2", "--seq", "16", "--steps", "10", "--ckpt-dir", ck, "--ckpt-every", "4", "--lr", "1e-2"]
    r = subprocess.run(cmd, env=env, cwd=tmp, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return ck, r


def _final_params(ck):
    with open(os.path.join(ck, "latest")) as f:
        d = f.read().strip()
    out = []
    for p in sorted(glob.glob(os.path.join(ck, d, "rank*.pt"))):
        out.append(torch.load(p, weights_only=True))
    return d, out


def test_rank_crash_restart_resume_is_bit_exact(tmp_path):
    tmp = str(tmp_path)
    ck_ref, _ = _run(tmp, "ref", fault=False)
    ck_f, r = _run(tmp, "fault", fault=True)
    assert os.path.exists(os.path.join(tmp, "fault.fault")), "the fault never fired"
    log = r.stdout + r.stderr
    assert "exitcode" in log or "restart" in log.lower() or "Restarting" in log
    d_ref, ref = _final_params(ck_ref)
    d_f, got = _final_params(ck_f)
    assert d_ref == d_f
    assert len(ref) == len(got) == 2
    for a, b in zip(ref, got):
        assert a["step"] == b["step"] == 9
        assert torch.equal(a["param"], b["param"])
