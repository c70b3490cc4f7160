#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_llama_gpu.py -q -x -p no:cacheprovider > gpurun_out/pytest_llama.log 2>&1
rc=$?; echo pytest rc=$rc; tail -2 gpurun_out/pytest_llama.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --steps 6 --warmup 2 > gpurun_out/bench.log 2>&1; rc=$?; grep metric gpurun_out/bench.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --steps 6 --warmup 2 --no-opt-overlap > gpurun_out/bench_noov.log 2>&1; rc=$?; grep metric gpurun_out/bench_noov.log; exit $rc
