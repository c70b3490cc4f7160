#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_xent_gpu.py tests/test_llama_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "xent or llama or cross" > gpurun_out/pytest_xent.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_xent.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 600 python bench.py --steps 6 --warmup 2 > gpurun_out/bench_xent.log 2>&1; rc=$?; grep metric gpurun_out/bench_xent.log | cut -c1-250; exit $rc
