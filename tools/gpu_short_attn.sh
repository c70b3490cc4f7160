#!/bin/bash
# short-sequence fused attention backward: tests, A/B micro-bench at the ViT-B/16 shape, ViT bench
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "flash or short or variants or packed" > gpurun_out/pytest_attn.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_attn.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 120 python tools/bench_attn.py --T 197 --B 256 --H 12 --Hkv 12 --hd 64 --noncausal --ab SPA_ATTN_SHORT=0 > gpurun_out/attn_short.log 2>&1 || exit 2
timeout -k 10 120 python tools/bench_attn.py --T 256 --B 128 --H 8 --Hkv 8 --hd 64 --ab SPA_ATTN_SHORT=0 >> gpurun_out/attn_short.log 2>&1 || exit 2
cat gpurun_out/attn_short.log
timeout -k 10 300 python bench/vit_train.py --steps 8 --warmup 2 > gpurun_out/vit.log 2>&1; rc=$?; grep metric gpurun_out/vit.log; exit $rc
