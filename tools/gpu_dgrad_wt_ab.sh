#!/bin/bash
# cached-W^T dgrad: GPU tests, then the headline bench ABBA (default on / SPA_DGRAD_WT=0)
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_llama_gpu.py tests/test_xent_gpu.py tests/test_moe_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_dgrad.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_dgrad.log; [ $rc -eq 0 ] || exit 1
for arm in on off off on; do
  e=""; [ $arm = off ] && e="SPA_DGRAD_WT=0"
  env $e timeout -k 10 600 python bench.py --steps 6 --warmup 2 > gpurun_out/bench_dgrad_$arm.log 2>&1 || exit 2
  echo "$arm $(grep metric gpurun_out/bench_dgrad_$arm.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["mem_gb"])')"
done | tee gpurun_out/dgrad_wt_ab.txt
