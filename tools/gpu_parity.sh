#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_graphs_gpu.py tests/test_misc_gpu.py tests/test_kernels_gpu.py -q -x -p no:cacheprovider -k "graph or dropout or adamw" > gpurun_out/pytest_graph.log 2>&1
rc=$?; echo pytest rc=$rc; tail -15 gpurun_out/pytest_graph.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench/parity.py --which B1,B5,B9 > gpurun_out/parity_eager.log 2>&1; rc=$?; cat gpurun_out/parity_eager.log | grep run; [ $rc -eq 0 ] || { tail -20 gpurun_out/parity_eager.log; exit $rc; }
timeout -k 10 600 python bench/parity.py --which B1,B5,B9 --graph > gpurun_out/parity_graph.log 2>&1; rc=$?; cat gpurun_out/parity_graph.log | grep run; [ $rc -eq 0 ] || { tail -20 gpurun_out/parity_graph.log; exit $rc; }
timeout -k 10 900 python bench/parity.py --which B14,B15,B16,B17 > gpurun_out/parity_quality.log 2>&1; rc=$?; cat gpurun_out/parity_quality.log | grep run; exit $rc
