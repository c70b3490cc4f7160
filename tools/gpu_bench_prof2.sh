#!/bin/bash
# headline bench + kernel-trace profile of the LLaMA3-8B training step
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python bench.py --steps 6 --warmup 2 > gpurun_out/bench.log 2>&1 || exit 1
grep metric gpurun_out/bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_full -o run --output-format csv -- python bench.py --steps 2 --warmup 1 > gpurun_out/prof_full.log 2>&1 || exit 2
echo done
