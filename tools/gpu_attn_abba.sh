#!/bin/bash
# ABBA same-process A/B of the round-2 forward options (pipelined sub-tiles, MFMA row sums, split-V)
mkdir -p gpurun_out
{
for i in 1 2; do
  timeout -k 10 150 python tools/bench_attn.py --iters 20 --ab SPA_ATTN_FWD_PIPE=0,SPA_ATTN_FWD_LMFMA=1 || exit 2
  timeout -k 10 150 python tools/bench_attn.py --iters 20 --T 197 --B 256 --H 12 --Hkv 12 --hd 64 --noncausal --ab SPA_ATTN_FWD_LMFMA=1 || exit 2
done
timeout -k 10 150 python tools/bench_attn.py --iters 20 --T 8192 --H 16 --Hkv 1 --hd 256 --ab SPA_ATTN_SPLITV=0 || exit 2
} > gpurun_out/attn_abba.txt 2>&1
cat gpurun_out/attn_abba.txt
