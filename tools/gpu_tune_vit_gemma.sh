#!/bin/bash
# TunableOp tables for the ViT-B/16 and Gemma-7B benches: record their GEMMs (no tuning), tune them
# one shape at a time (resuming from tuning/tunableop_<name>.csv), then A/B each bench with and
# without its table on this box. Usage: bash tools/gpu_tune_vit_gemma.sh vit|gemma
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
n=$1
if [ "$n" = vit ]; then cmd="python bench/vit_train.py --steps 1 --warmup 1"; bench="python bench/vit_train.py --steps 8 --warmup 2";
else cmd="python bench/gemma_tp.py --layers 2 --steps 1 --warmup 1"; bench="python bench/gemma_tp.py --layers 6 --steps 3 --warmup 1"; fi
[ -f tuning/tunableop_$n.csv ] && cp tuning/tunableop_$n.csv gpurun_out/tunableop_$n.csv
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=0 PYTORCH_TUNABLEOP_RECORD_UNTUNED=1 \
PYTORCH_TUNABLEOP_UNTUNED_FILENAME=gpurun_out/untuned_$n.csv PYTORCH_TUNABLEOP_FILENAME=gpurun_out/unused_$n.csv \
  timeout -k 10 300 $cmd > gpurun_out/record_$n.log 2>&1 || exit 1
wc -l gpurun_out/untuned_${n}0.csv
timeout -k 10 800 python -u tools/tune_gemms.py gpurun_out/untuned_${n}0.csv gpurun_out/tunableop_$n.csv > gpurun_out/tune_$n.log 2>&1; rc=$?
tail -3 gpurun_out/tune_$n.log; [ $rc -eq 0 ] || exit 2
for arm in base tuned base tuned; do
  extra=""; [ $arm = tuned ] && extra="--gemm-table gpurun_out/tunableop_$n.csv"
  timeout -k 10 300 $bench $extra > gpurun_out/ab_$n.log 2>&1 || exit 3
  echo "$arm $(grep metric gpurun_out/ab_$n.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["value"])')"
done | tee gpurun_out/tune_ab_$n.txt
