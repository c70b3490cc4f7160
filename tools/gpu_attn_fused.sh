#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_kernels_gpu.py tests/test_llama_gpu.py -q -x -p no:cacheprovider -k "attn or attention or llama or flash" > gpurun_out/pytest_attn.log 2>&1
rc=$?; echo pytest rc=$rc; tail -4 gpurun_out/pytest_attn.log; [ $rc -eq 0 ] || exit $rc
for cfg in "--T 8192" "--T 2048 --B 4" "--T 4096 --hd 64 --H 16 --Hkv 16" "--T 197 --B 64 --H 12 --Hkv 12 --hd 64 --noncausal"; do
  timeout -k 10 120 python tools/bench_attn.py $cfg || exit 1
  SPA_ATTN_BWD_SPLIT=1 timeout -k 10 120 python tools/bench_attn.py $cfg || exit 1
done
timeout -k 10 600 python bench.py --steps 6 --warmup 2 > gpurun_out/bench.log 2>&1; rc=$?; grep metric gpurun_out/bench.log; exit $rc
