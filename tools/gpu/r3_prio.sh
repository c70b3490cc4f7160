#!/bin/bash
# stream priorities for the two-chunk pipelines: proxy with high-priority side + comm streams vs none
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/overlap_proxy.py --layers 2 > gpurun_out/r3pr_hi.log 2>&1; echo "hi rc=$?"
grep -v amdgpu.ids gpurun_out/r3pr_hi.log | cut -c1-700
SPA_SIDE_PRIO=0 SPA_COMM_PRIO=0 timeout -k 10 400 python -u tools/overlap_proxy.py --layers 2 > gpurun_out/r3pr_lo.log 2>&1; echo "lo rc=$?"
grep -v amdgpu.ids gpurun_out/r3pr_lo.log | cut -c1-700
SPA_SIDE_PRIO=0 timeout -k 10 400 python -u tools/overlap_proxy.py --layers 2 --which tp > gpurun_out/r3pr_commhi.log 2>&1; echo "commhi rc=$?"
grep -v amdgpu.ids gpurun_out/r3pr_commhi.log | cut -c1-700
