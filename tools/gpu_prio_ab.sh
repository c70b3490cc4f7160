#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "flash" > gpurun_out/pytest_prio.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_prio.log; [ $rc -eq 0 ] || exit 1
for i in 1 2; do timeout -k 10 150 python tools/bench_attn.py --iters 20 --ab SPA_ATTN_PRIO=1 || exit 2; done > gpurun_out/prio_ab.txt 2>&1
timeout -k 10 150 python tools/bench_attn.py --iters 20 --T 197 --B 256 --H 12 --Hkv 12 --hd 64 --noncausal --ab SPA_ATTN_PRIO=1 >> gpurun_out/prio_ab.txt 2>&1 || exit 2
cat gpurun_out/prio_ab.txt
