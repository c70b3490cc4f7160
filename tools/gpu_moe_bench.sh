#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 300 python tools/bench_moe.py > gpurun_out/bench_moe.log 2>&1; rc=$?; cat gpurun_out/bench_moe.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench/vit_train.py --steps 5 --warmup 2 > gpurun_out/vit_bench.log 2>&1; rc=$?; tail -3 gpurun_out/vit_bench.log; exit $rc
