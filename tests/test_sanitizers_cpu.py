"""Race detection / sanitizers for the host runtime: the native token loader
(csrc/runtime/token_loader.cpp: producer threads, ring, seek, mmap source) is compiled
into a stress harness (tools/sanitize/loader_stress.cpp) with AddressSanitizer +
UndefinedBehaviorSanitizer (leak checking on) and, separately, with ThreadSanitizer, and
must run clean. GPU sanitizers are unavailable on this pool; device kernels are covered
by the oracle tests and the range-checked buffer loads."""
import hashlib
import os
import shutil
import subprocess

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tools", "sanitize", "loader_stress.cpp")
DEP = os.path.join(ROOT, "csrc", "runtime", "token_loader.cpp")


def _build(kind, flags):
    tdir = os.path.dirname(torch.__file__)
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    h = hashlib.sha1((open(SRC).read() + open(DEP).read() + " ".join(flags)).encode()).hexdigest()[:12]
    out_dir = os.path.join(ROOT, "build", "sanitize")
    os.makedirs(out_dir, exist_ok=True)
    exe = os.path.join(out_dir, f"loader_{kind}_{h}")
    if not os.path.exists(exe):
        cmd = ["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", *flags, f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
               f"-I{tdir}/include", f"-I{tdir}/include/torch/csrc/api/include", SRC, f"-L{tdir}/lib",
               f"-Wl,-rpath,{tdir}/lib", "-ltorch", "-ltorch_cpu", "-lc10", "-pthread", "-o", exe + ".tmp"]
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
        assert r.returncode == 0, r.stderr[-3000:]
        os.replace(exe + ".tmp", exe)
    return exe


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
@pytest.mark.parametrize("kind,flags,env", [
    ("asan", ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined"],
     {"ASAN_OPTIONS": "detect_leaks=1:abort_on_error=1", "UBSAN_OPTIONS": "print_stacktrace=1"}),
    ("tsan", ["-fsanitize=thread"], {"TSAN_OPTIONS": "halt_on_error=1:second_deadlock_stack=1"}),
])
def test_token_loader_under_sanitizers(kind, flags, env):
    exe = _build(kind, flags)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=600, env=dict(os.environ, **env))
    assert r.returncode == 0 and "loader stress ok" in r.stdout, (r.stdout[-2000:] + r.stderr[-4000:])
    assert "ERROR: AddressSanitizer" not in r.stderr and "WARNING: ThreadSanitizer" not in r.stderr
