#!/bin/bash
# dsv3_v3 widths (4 layers, 32 experts), bf16 vs fp8 (block-scaled experts + fp8 projections), ABBA on one box
mkdir -p gpurun_out
for arm in bf16 fp8 fp8 bf16; do
  e=""; [ $arm = fp8 ] && e="--fp8"
  timeout -k 10 400 python bench/dsv3_train.py --preset dsv3_v3 --layers 4 --dense-layers 1 --experts 32 --mb 1 --steps 4 --warmup 2 $e > gpurun_out/dsv3v3_$arm.log 2>&1 || exit 1
  echo "$arm $(grep metric gpurun_out/dsv3v3_$arm.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done | tee gpurun_out/dsv3v3_fp8_abba.txt
