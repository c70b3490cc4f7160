#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_kernels_gpu.py tests/test_llama_gpu.py -q -x -p no:cacheprovider -k "transpose or wgrad or llama or linear or xent" > gpurun_out/pytest_wgrad.log 2>&1
rc=$?; echo pytest rc=$rc; tail -3 gpurun_out/pytest_wgrad.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --steps 6 --warmup 2 > gpurun_out/bench.log 2>&1; rc=$?; grep metric gpurun_out/bench.log; [ $rc -eq 0 ] || exit $rc
SPA_WGRAD_NT=0 timeout -k 10 600 python bench.py --steps 6 --warmup 2 > gpurun_out/bench_tn.log 2>&1; rc=$?; grep metric gpurun_out/bench_tn.log; exit $rc
