#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_moe_gpu.py -q -x -p no:cacheprovider -k grouped > gpurun_out/pytest_gg.log 2>&1
rc=$?; echo pytest rc=$rc; tail -3 gpurun_out/pytest_gg.log; [ $rc -eq 0 ] || exit $rc


timeout -k 10 300 python tools/bench_moe.py > gpurun_out/bench_moe.log 2>&1; rc=$?; cat gpurun_out/bench_moe.log; exit $rc
