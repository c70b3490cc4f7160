#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_attention_dropout_gpu.py -x -q --timeout 120 --timeout-method thread -k "flash or attn or short or dropout or mla" > gpurun_out/pytest_xcd.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_xcd.log; [ $rc -eq 0 ] || exit 1
for i in 1 2; do timeout -k 10 150 python tools/bench_attn.py --iters 20 --ab SPA_ATTN_XCD=0 || exit 2; done > gpurun_out/xcd_ab.txt 2>&1
timeout -k 10 150 python tools/bench_attn.py --iters 20 --T 4096 --B 2 --ab SPA_ATTN_XCD=0 >> gpurun_out/xcd_ab.txt 2>&1 || exit 2
cat gpurun_out/xcd_ab.txt
