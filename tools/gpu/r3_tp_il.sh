#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/overlap_proxy.py --layers 2 --which tp --rounds 3 > gpurun_out/r3il.log 2>&1; echo "tp rc=$?"
grep -v amdgpu.ids gpurun_out/r3il.log | cut -c1-900
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r3il_prof -o run -- python tools/overlap_proxy.py --which tp --variants interleave --arms interleave:overlap --iters 2 --rounds 1 > gpurun_out/r3il_prof.log 2>&1; echo "prof rc=$?"
