#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "flash or rowsum or spike or rescale" > gpurun_out/pytest_lmfma.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_lmfma.log; [ $rc -eq 0 ] || exit 1
for i in 1 2; do
  timeout -k 10 120 python tools/bench_attn.py --T 197 --B 256 --H 12 --Hkv 12 --hd 64 --noncausal --ab SPA_ATTN_FWD_LMFMA=1 || exit 2
  timeout -k 10 120 python tools/bench_attn.py --ab SPA_ATTN_FWD_LMFMA=1 || exit 2
done > gpurun_out/lmfma_ab.txt 2>&1
cat gpurun_out/lmfma_ab.txt
