#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/overlap_proxy.py --layers 2 --which tp --rounds 4 > gpurun_out/r3tl.log 2>&1; echo "tp rc=$?"
grep -v amdgpu.ids gpurun_out/r3tl.log | cut -c1-700
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r3tl_prof -o run -- python tools/overlap_proxy.py --which tp --arms pipelined --iters 2 --rounds 1 > gpurun_out/r3tl_prof.log 2>&1; echo "prof rc=$?"
