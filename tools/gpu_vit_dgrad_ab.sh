#!/bin/bash
# ViT-B/16: dgrad on cached W^T for its (< 4M-element) weights too (SPA_DGRAD_WT_MIN=0) vs default, ABBA
mkdir -p gpurun_out
for arm in def all all def; do
  e=""; [ $arm = all ] && e="SPA_DGRAD_WT_MIN=0"
  env $e timeout -k 10 300 python bench/vit_train.py --steps 8 --warmup 2 > gpurun_out/vit_dgrad_$arm.log 2>&1 || exit 1
  echo "$arm $(grep metric gpurun_out/vit_dgrad_$arm.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done | tee gpurun_out/vit_dgrad_abba.txt
