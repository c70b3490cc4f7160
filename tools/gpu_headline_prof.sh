#!/bin/bash
# kernel-trace profile of the headline step (2 timed steps + 1 warmup), summarised on the box
mkdir -p gpurun_out/prof_head
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_head -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 > gpurun_out/prof_head/bench.log 2>&1
rc=$?; grep metric gpurun_out/prof_head/bench.log | cut -c1-200
f=$(find gpurun_out/prof_head -name "*kernel_stats.csv" | head -1)
cp "$f" gpurun_out/headline_kernel_stats.csv && python tools/prof_summary.py "$f" 3 > gpurun_out/headline_summary.txt
rm -rf gpurun_out/prof_head/*/
cat gpurun_out/headline_summary.txt
exit $rc
