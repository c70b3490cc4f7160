"""First contact with RCCL on the 1-GPU box: a real ``nccl`` process group of
size 1 bound to cuda:0 (``device_id``), with SPA_FORCE_COLLECTIVES=1 so the DP bucket all-reduce
(AVG, bf16), ZeRO-1 reduce-scatter / all-gather, the launch-stream all-to-all, the EP dispatch with
its pinned split-size D2H (bf16 and fp8 payloads) and the async routing-bias all-reduce all run
through librccl instead of short-circuiting at world 1. The checks run in a fresh child process
(tests/rccl_world1_child.py) so the process group never leaks into the other GPU tests."""
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_rccl_world1_drives_every_collective_path():
    child = os.path.join(os.path.dirname(os.path.abspath(__file__)), "rccl_world1_child.py")
    root = os.path.dirname(os.path.dirname(child))
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(_port()), SPA_FORCE_COLLECTIVES="1",
               PYTHONPATH=root + os.pathsep + os.environ.get("PYTHONPATH", ""))
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    r = subprocess.run([sys.executable, "-u", child], env=env, cwd=root, timeout=200,
                       capture_output=True, text=True)
    print(r.stdout[-4000:])
    print(r.stderr[-4000:], file=sys.stderr)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "RCCL_WORLD1_OK" in r.stdout
