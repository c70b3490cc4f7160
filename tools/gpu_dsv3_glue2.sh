#!/bin/bash
# DeepSeek split residual stream: tests, dsv3_style bench (bf16 moments default, and fp32 moments A/B)
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_moe_gpu.py tests/test_decode_gpu.py tests/test_mla_decode_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_dsv3.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_dsv3.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench/dsv3_train.py --preset dsv3_style --steps 4 --warmup 2 > gpurun_out/dsv3s.log 2>&1; rc=$?; grep metric gpurun_out/dsv3s.log | cut -c1-400; [ $rc -eq 0 ] || exit 2
timeout -k 10 300 python bench/dsv3_train.py --preset dsv3_style --steps 4 --warmup 2 --fp32-moments > gpurun_out/dsv3s_fp32m.log 2>&1; rc=$?; grep metric gpurun_out/dsv3s_fp32m.log | cut -c1-400; [ $rc -eq 0 ] || exit 3
timeout -k 10 300 python bench/dsv3_train.py --preset dsv3_v3 --layers 4 --dense-layers 1 --experts 32 --mb 1 --steps 4 --warmup 2 --fp8 > gpurun_out/dsv3v3_fp8.log 2>&1; rc=$?; grep metric gpurun_out/dsv3v3_fp8.log | cut -c1-400; exit $rc
