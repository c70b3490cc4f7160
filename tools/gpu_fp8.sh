#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_moe_gpu.py tests/test_kernels_gpu.py -q -x -p no:cacheprovider -k "fp8 or transpose" > gpurun_out/pytest_fp8.log 2>&1
rc=$?; echo pytest rc=$rc; tail -15 gpurun_out/pytest_fp8.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/bench_moe.py > gpurun_out/bench_moe.log 2>&1; rc=$?; cat gpurun_out/bench_moe.log | grep -v amdgpu; exit $rc
