#!/bin/bash
# record + tune the direct (transpose-free) weight-gradient GEMMs, then A/B the bench
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
cp tuning/tunableop_llama8b.csv gpurun_out/tunableop_llama8b.csv
SPA_WGRAD_NT=0 PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=0 PYTORCH_TUNABLEOP_RECORD_UNTUNED=1 \
PYTORCH_TUNABLEOP_UNTUNED_FILENAME=gpurun_out/untuned_tn.csv PYTORCH_TUNABLEOP_FILENAME=gpurun_out/unused.csv \
  timeout -k 10 300 python bench.py --layers 2 --steps 1 --warmup 1 --gemm-table /nonexistent > gpurun_out/record.log 2>&1 || exit 1
timeout -k 10 900 python tools/tune_gemms.py gpurun_out/untuned_tn0.csv gpurun_out/tunableop_llama8b.csv || exit 2
timeout -k 10 300 python bench.py --steps 6 --warmup 2 --gemm-table gpurun_out/tunableop_llama8b.csv > gpurun_out/bench_nt.log 2>&1 || exit 3
grep -o '"value": [0-9.]*' gpurun_out/bench_nt.log
SPA_WGRAD_NT=0 timeout -k 10 300 python bench.py --steps 6 --warmup 2 --gemm-table gpurun_out/tunableop_llama8b.csv > gpurun_out/bench_tn.log 2>&1 || exit 4
grep -o '"value": [0-9.]*' gpurun_out/bench_tn.log
