#!/bin/bash
# stream-K grid knobs vs a co-running collective stand-in (tools/overlap_interference.py)
mkdir -p gpurun_out
: > gpurun_out/sk_env.jsonl
for e in "NONE=1" "TENSILE_STREAMK_MAX_CUS=240" "TENSILE_STREAMK_MAX_CUS=224" "TENSILE_STREAMK_DYNAMIC_GRID=1" "TENSILE_STREAMK_DATA_PARALLEL=1"; do
  echo "{\"env\": \"$e\"}" >> gpurun_out/sk_env.jsonl
  env $e timeout -k 10 200 python tools/overlap_interference.py --layers 4 --nwg 16 --iters 3 >> gpurun_out/sk_env.jsonl 2>> gpurun_out/sk_env.err || exit 1
done
cat gpurun_out/sk_env.jsonl
