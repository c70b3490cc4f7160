#!/bin/bash
# Tune the LLaMA3-8B training GEMMs with PyTorch TunableOp (hipBLASLt + rocBLAS solution search).
# Every layer has the same GEMM shapes, so a 2-layer model at T=8192 covers them all (plus the
# LM head). 1) record the untuned GEMMs (no tuning, fast); 2) tune them one by one with progress
# (resuming from tuning/tunableop_llama8b.csv); 3) time the full bench with and without.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
cp tuning/tunableop_llama8b.csv gpurun_out/tunableop_llama8b.csv
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=0 PYTORCH_TUNABLEOP_RECORD_UNTUNED=1 \
PYTORCH_TUNABLEOP_UNTUNED_FILENAME=gpurun_out/untuned.csv PYTORCH_TUNABLEOP_FILENAME=gpurun_out/unused.csv \
  timeout -k 10 300 python bench.py --layers 2 --steps 1 --warmup 1 > gpurun_out/record.log 2>&1 || exit 1
ls gpurun_out/
timeout -k 10 900 python tools/tune_gemms.py gpurun_out/untuned0.csv gpurun_out/tunableop_llama8b.csv 2>&1 | tee gpurun_out/tune.log || exit 2
