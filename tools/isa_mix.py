"""Instruction mix of a kernel's loop blocks from the gfx950 assembly of one .hip file (CPU only:
hipcc --offload-device-only -S). Prints, per basic block that holds MFMAs, the count of MFMA /
VALU / transcendental / LDS / SALU instructions and the top VALU opcodes, plus VGPR / scratch
figures -- the quick check of what a source change did to a hot loop before spending a GPU run.

  python tools/isa_mix.py csrc/kernels/attention.hip attn_bwd_short_kernel [--flags "-fno-slp-vectorize"]
"""
import argparse
import collections
import re
import subprocess
import sys
import sysconfig
from pathlib import Path


def assemble(src, flags=""):
    import torch
    t = Path(torch.__file__).parent
    out = Path("/tmp") / (Path(src).stem + ".isa_mix.s")
    cmd = (f"hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -D__HIP_PLATFORM_AMD__=1 -DUSE_ROCM=1 "
           f"-DHIP_ENABLE_WARP_SYNC_BUILTINS=1 -I{Path(__file__).resolve().parents[1] / 'csrc/include'} "
           f"-I{t}/include -I{t}/include/torch/csrc/api/include -I{sysconfig.get_paths()['include']} "
           f"-D_GLIBCXX_USE_CXX11_ABI=1 -Wno-unused-result -Wno-deprecated-declarations -munsafe-fp-atomics "
           f"--offload-device-only -S {flags} {src} -o {out}")
    subprocess.run(cmd, shell=True, check=True)
    return out.read_text()


def mix(asm, pattern):
    names = [n for n in re.findall(r"^(_Z\S+):", asm, re.M) if re.search(pattern, n)]
    for name in names:
        i = asm.index(name + ":")
        j = asm.index(".Lfunc_end", i)
        body, tail = asm[i:j], asm[j:j + 6000]
        vg = re.search(r"; NumVgprs: (\d+)", tail)
        sc = re.search(r"; ScratchSize: (\d+)", tail)
        print(f"== {name}  vgpr {vg and vg.group(1)}  scratch {sc and sc.group(1)}")
        cur = "entry"
        for part in re.split(r"\n(\.LBB\d+_\d+):", body):
            if part.startswith(".LBB"):
                cur = part
                continue
            c = collections.Counter()
            for line in part.split("\n"):
                line = line.strip()
                if not line or line[0] in ";." or ":" in line.split()[0]:
                    continue
                op = line.split()[0]
                if op.startswith("v_mfma"):
                    c["MFMA"] += 1
                elif op.startswith("v_accvgpr"):
                    c["accmov"] += 1
                elif op.startswith("v_"):
                    c["VALU"] += 1
                    if op.startswith(("v_exp", "v_log", "v_rcp", "v_rsq", "v_sqrt")):
                        c["trans"] += 1
                    c[op] += 1
                elif op.startswith("ds_"):
                    c["LDS"] += 1
                elif op.startswith("s_"):
                    c["SALU"] += 1
                elif op.startswith(("global_", "buffer_")):
                    c["VMEM"] += 1
            if c["MFMA"]:
                head = {k: c[k] for k in ("MFMA", "VALU", "trans", "LDS", "SALU", "VMEM", "accmov") if c[k]}
                ops = {k: v for k, v in c.most_common() if k.startswith("v_")}
                top = ", ".join(f"{k} {v}" for k, v in list(ops.items())[:8])
                # vector issue cycles (MI355X_MICROARCH constants: transcendental 8, other VALU 4,
                # MFMA 8 of its 32) against the MFMA pipe's 32 per 32x32x16
                issue = 8 * c["trans"] + 4 * (c["VALU"] - c["trans"]) + 8 * c["MFMA"]
                print(f"  {cur:12s} {head}  issue~{issue} cyc vs mfma {32 * c['MFMA']}  | {top}")


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("src")
    ap.add_argument("pattern")
    ap.add_argument("--flags", default="")
    a = ap.parse_args()
    mix(assemble(a.src, a.flags), a.pattern)
    sys.exit(0)
