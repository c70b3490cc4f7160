#!/bin/bash
# Overlap proxy: default HW queues vs GPU_MAX_HW_QUEUES=8 (two compute streams + two comm streams)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/overlap_proxy.py --layers 2 > gpurun_out/r3o2_q4.log 2>&1; echo "q4 rc=$?"
grep -v amdgpu.ids gpurun_out/r3o2_q4.log | cut -c1-900
GPU_MAX_HW_QUEUES=8 timeout -k 10 400 python -u tools/overlap_proxy.py --layers 2 > gpurun_out/r3o2_q8.log 2>&1; echo "q8 rc=$?"
grep -v amdgpu.ids gpurun_out/r3o2_q8.log | cut -c1-900
