#!/bin/bash
# headline bench A/B: tuned GEMM table vs library defaults (same box)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python bench.py --steps 6 --warmup 2 > gpurun_out/bench_tuned.log 2>&1 || exit 1
grep metric gpurun_out/bench_tuned.log
SPA_GEMM_TUNING=0 timeout -k 10 300 python bench.py --steps 6 --warmup 2 > gpurun_out/bench_default.log 2>&1 || exit 2
grep metric gpurun_out/bench_default.log
timeout -k 10 300 python bench.py --steps 6 --warmup 2 > gpurun_out/bench_tuned2.log 2>&1 || exit 3
grep metric gpurun_out/bench_tuned2.log
