#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "flash or fwd_pipe" > gpurun_out/pytest_pipe.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_pipe.log; [ $rc -eq 0 ] || exit 1
for i in 1 2; do timeout -k 10 120 python tools/bench_attn.py --ab SPA_ATTN_FWD_PIPE=0 || exit 2; done > gpurun_out/fwd_pipe_ab.txt 2>&1
timeout -k 10 120 python tools/bench_attn.py --T 4096 --B 2 --H 16 --Hkv 16 --ab SPA_ATTN_FWD_PIPE=0 >> gpurun_out/fwd_pipe_ab.txt 2>&1
cat gpurun_out/fwd_pipe_ab.txt
