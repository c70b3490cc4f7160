#!/bin/bash
# DeepSeek GPU tests + small-depth DSV3-style bench + kernel profile
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 600 python -m pytest tests/test_moe_gpu.py -q -x -p no:cacheprovider > gpurun_out/pytest_moe.log 2>&1
rc=$?; echo pytest rc=$rc; tail -5 gpurun_out/pytest_moe.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench/dsv3_train.py --steps 4 --warmup 2 --layers 4 > gpurun_out/dsv3_bench.log 2>&1
rc=$?; echo bench rc=$rc; tail -5 gpurun_out/dsv3_bench.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_dsv3 -o run -- python3 bench/dsv3_train.py --steps 2 --warmup 1 --layers 4 > gpurun_out/dsv3_prof.log 2>&1
rc=$?; echo prof rc=$rc; tail -3 gpurun_out/dsv3_prof.log
exit $rc
