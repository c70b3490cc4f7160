#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "flash or splitv or pipe" > gpurun_out/pytest_splitv.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_splitv.log; [ $rc -eq 0 ] || exit 1
for i in 1 2; do timeout -k 10 120 python tools/bench_attn.py --T 8192 --H 16 --Hkv 1 --hd 256 --ab SPA_ATTN_SPLITV=0 || exit 2; done > gpurun_out/splitv_ab.txt 2>&1
cat gpurun_out/splitv_ab.txt
timeout -k 10 300 python bench/gemma_tp.py --layers 6 --steps 3 --warmup 1 > gpurun_out/gemma6.log 2>&1; rc=$?; grep metric gpurun_out/gemma6.log | cut -c1-300; exit $rc
