#!/bin/bash
# DeepSeek glue fusions: tests, dsv3_style bench, torch op profile
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_moe_gpu.py -x -q --timeout 120 --timeout-method thread -k "mla or router or deepseek or route" > gpurun_out/pytest_dsv3.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_dsv3.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench/dsv3_train.py --preset dsv3_style --steps 4 --warmup 2 > gpurun_out/dsv3s.log 2>&1; rc=$?; grep metric gpurun_out/dsv3s.log | cut -c1-330; [ $rc -eq 0 ] || exit 2
timeout -k 10 300 python tools/torch_op_profile.py --preset dsv3_style --mb 2 --rows 45 > gpurun_out/dsv3s_ops.txt 2>&1; rc=$?; head -60 gpurun_out/dsv3s_ops.txt | cut -c1-250; exit $rc
