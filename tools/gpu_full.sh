#!/bin/bash
# full GPU suite + parity profile
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 900 python -m pytest tests/ -m gpu -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo pytest rc=$rc; tail -5 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench/parity.py --which B1,B5,B9 > gpurun_out/parity_eager.log 2>&1; rc=$?; grep run gpurun_out/parity_eager.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_b9 -o run --output-format csv -- python3 bench/parity.py --which B9 --steps 20 --warmup 3 > gpurun_out/prof_b9.log 2>&1
rc=$?; echo prof rc=$rc; exit $rc
