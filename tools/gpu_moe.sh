#!/bin/bash
# MoE kernels + DeepSeek-V3 GPU tests
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_moe_gpu.py -q -x -p no:cacheprovider > gpurun_out/pytest_moe.log 2>&1
rc=$?
echo rc=$rc
tail -40 gpurun_out/pytest_moe.log
exit $rc
