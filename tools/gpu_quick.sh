#!/bin/bash
# norm kernel tests + parity throughput + short headline bench
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -q -x -p no:cacheprovider -k "norm or xent" > gpurun_out/pytest_norm.log 2>&1
rc=$?; echo pytest rc=$rc; tail -2 gpurun_out/pytest_norm.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench/parity.py --which B1,B5,B9 > gpurun_out/parity_eager.log 2>&1; rc=$?; grep run gpurun_out/parity_eager.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --steps 6 --warmup 2 > gpurun_out/bench.log 2>&1; rc=$?; grep metric gpurun_out/bench.log; exit $rc
