#!/bin/bash
# Overlap proxy after the TP sync-point fix, plus kernel traces of the EP compute vs pipe_comp arms
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/overlap_proxy.py --layers 2 > gpurun_out/r3o_overlap.log 2>&1; echo "overlap rc=$?"
grep -v amdgpu.ids gpurun_out/r3o_overlap.log | cut -c1-700
for arm in compute pipe_comp; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3o_prof_$arm -o run -- python3 -u tools/overlap_proxy.py --which ep --arms $arm --rounds 1 --iters 3 > gpurun_out/r3o_prof_$arm.log 2>&1 || { echo "prof $arm failed"; exit 1; }
done
echo prof done
