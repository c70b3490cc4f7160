#!/bin/bash
# session restart check: attention micro-bench at the LLaMA shape and the headline bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/bench_attn.py > gpurun_out/r3b_attn.log 2>&1; echo "attn rc=$?"
grep -i attn gpurun_out/r3b_attn.log | cut -c1-300
timeout -k 10 400 python -u bench.py --steps 8 --warmup 2 > gpurun_out/r3b_bench.log 2>&1; echo "bench rc=$?"
grep '^{' gpurun_out/r3b_bench.log | cut -c1-400
