"""In-tree native build for the gfx950 extension (``solvingpapers_amd/_C.so``).

No hipify, no setuptools CUDAExtension: we emit a ``build.ninja`` that drives
``hipcc --offload-arch=gfx950`` over every ``csrc/kernels/*.hip`` (device code +
torch op registration) and ``csrc/runtime/*.cpp`` (host-only runtime: data
loader, bucket planner), then links one shared object that
``torch.ops.load_library`` loads.  The .so lands inside the package so it
travels with the repo snapshot to the GPU box.

Usage: ``python -m solvingpapers_amd._build [-j N] [--debug]``.
"""
from __future__ import annotations

import argparse
import os
import shutil
import subprocess
import sys
import sysconfig
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
PKG = ROOT / "solvingpapers_amd"
CSRC = ROOT / "csrc"
BUILD = ROOT / "build"
OUT = PKG / "_C.so"
ARCH = os.environ.get("SPA_OFFLOAD_ARCH", "gfx950")
# variant builds for kernel A/B and profiling (tools/build_variant.sh): SPA_BUILD_VARIANT=name puts
# objects under build/name and the library at ab/_C_name.so (loaded through SPA_EXT_SO),
# SPA_BUILD_DEFINES adds device-compile flags (e.g. -DSPA_DKDV3_STAMP=1); the in-tree _C.so is untouched
VARIANT = os.environ.get("SPA_BUILD_VARIANT", "")
if VARIANT:
    BUILD = ROOT / "build" / VARIANT
    OUT = ROOT / "ab" / f"_C_{VARIANT}.so"
# per-file device flags: attention_short.hip without SLP vectorisation (hipcc packed its P * dP
# products into v_pk_mul_f32 behind register shuffles: 24-34 more VALU per call on a VALU-bound
# kernel; the other attention kernels keep it: the hd-256 forward needs 46 more VALU without it)
EXTRA_FLAGS = {"attention_short.hip": "-fno-slp-vectorize"}


def _torch_paths():
    import torch
    tdir = Path(torch.__file__).resolve().parent
    inc = [tdir / "include", tdir / "include" / "torch" / "csrc" / "api" / "include"]
    lib = tdir / "lib"
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return inc, lib, abi


def sources():
    devs = sorted((CSRC / "kernels").glob("*.hip"))
    hosts = sorted((CSRC / "runtime").glob("*.cpp"))
    return devs, hosts


def write_ninja(debug: bool = False) -> Path:
    inc, lib, abi = _torch_paths()
    py_inc = sysconfig.get_paths()["include"]
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    incs = " ".join(f"-I{p}" for p in [CSRC / "include", *inc, py_inc, "/opt/rocm/include"])
    common = (
        f"-std=c++17 -fPIC -D_GLIBCXX_USE_CXX11_ABI={abi} -DTORCH_EXTENSION_NAME=_C "
        "-DTORCH_API_INCLUDE_EXTENSION_H -D__HIP_PLATFORM_AMD__=1 -DUSE_ROCM=1 "
        "-DHIP_ENABLE_WARP_SYNC_BUILTINS=1 -Wno-unused-result -Wno-unused-command-line-argument "
        "-Wno-deprecated-declarations"
    )
    opt = "-O0 -g" if debug else "-O3"
    dev_flags = f"{common} {opt} --offload-arch={ARCH} -munsafe-fp-atomics"
    if VARIANT:
        dev_flags += " " + os.environ.get("SPA_BUILD_DEFINES", "")
    host_flags = f"{common} {opt} -pthread"
    ldflags = (
        f"-shared -fPIC --offload-arch={ARCH} -L{lib} -Wl,-rpath,{lib} "
        "-lc10 -lc10_hip -ltorch -ltorch_cpu -ltorch_hip -ltorch_python -lamdhip64 -pthread"
    )
    BUILD.mkdir(exist_ok=True)
    devs, hosts = sources()
    lines = [
        "ninja_required_version = 1.3",
        f"hipcc = {hipcc}",
        f"incs = {incs}",
        f"devflags = {dev_flags}",
        f"hostflags = {host_flags}",
        f"ldflags = {ldflags}",
        "rule hip",
        "  command = $hipcc $devflags $incs -MD -MF $out.d -c $in -o $out",
        "  depfile = $out.d",
        "  deps = gcc",
        "  description = HIPCC $in",
        "rule cxx",
        "  command = $hipcc -x c++ $hostflags $incs -MD -MF $out.d -c $in -o $out",
        "  depfile = $out.d",
        "  deps = gcc",
        "  description = CXX $in",
        "rule link",
        "  command = $hipcc $in $ldflags -o $out",
        "  description = LINK $out",
    ]
    objs = []
    for s in devs:
        o = BUILD / "obj" / (s.stem + ".hip.o")
        objs.append(o)
        lines.append(f"build {o}: hip {s}")
        if s.name in EXTRA_FLAGS:
            lines.append(f"  devflags = {dev_flags} {EXTRA_FLAGS[s.name]}")
    for s in hosts:
        o = BUILD / "obj" / (s.stem + ".cpp.o")
        objs.append(o)
        lines.append(f"build {o}: cxx {s}")
    lines.append(f"build {OUT}: link {' '.join(str(o) for o in objs)}")
    lines.append(f"default {OUT}")
    nf = BUILD / "build.ninja"
    text = "\n".join(lines) + "\n"
    if not nf.exists() or nf.read_text() != text:
        nf.write_text(text)
    return nf


def build(jobs: int | None = None, debug: bool = False, verbose: bool = False) -> Path:
    OUT.parent.mkdir(parents=True, exist_ok=True)
    (BUILD / "obj").mkdir(parents=True, exist_ok=True)
    nf = write_ninja(debug)
    jobs = jobs or min(8, os.cpu_count() or 4, int(os.environ.get("MAX_JOBS", "16")))
    cmd = [shutil.which("ninja") or "ninja", "-f", str(nf), "-j", str(jobs)]
    if verbose:
        cmd.append("-v")
    r = subprocess.run(cmd, cwd=str(ROOT))
    if r.returncode != 0:
        raise RuntimeError(f"native build failed (exit {r.returncode})")
    return OUT


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("-j", type=int, default=None)
    ap.add_argument("--debug", action="store_true")
    ap.add_argument("-v", action="store_true")
    a = ap.parse_args(argv)
    p = build(a.j, a.debug, a.v)
    print(p)


if __name__ == "__main__":
    sys.exit(main())
