#!/bin/bash
# A/B of two builds of the extension on the attention micro-bench: the in-tree .so (N) vs a saved
# baseline build (B, path in $BASE_SO, default ab/_C_base.so; loaded through SPA_EXT_SO), separate
# processes in the order B N N B, at the LLaMA3-8B, ViT-B/16, Gemma-7B and DeepSeek MLA shapes
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/aab
for shape in "--H 32 --Hkv 8 --hd 128" "--B 256 --T 197 --H 12 --Hkv 12 --hd 64 --noncausal" "--H 16 --Hkv 1 --hd 256" "--T 4096 --H 128 --Hkv 128 --hd 192 --hdv 128"; do
  for arm in B N N B; do
    if [ $arm = B ]; then export SPA_EXT_SO=${BASE_SO:-ab/_C_base.so}; else unset SPA_EXT_SO; fi
    timeout -k 10 120 python -u tools/bench_attn.py $shape --iters 20 > gpurun_out/aab/one.log 2>&1 || { tail -5 gpurun_out/aab/one.log; exit 1; }
    echo "$arm $(grep -h 'attn B' gpurun_out/aab/one.log | cut -c1-200)"
  done
done
