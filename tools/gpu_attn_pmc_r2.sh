#!/bin/bash
# rocprofv3 counter pass over the round-2 attention kernels (LLaMA3-8B, ViT-B/16, Gemma MQA hd 256)
mkdir -p gpurun_out/apmc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
run() {  # name, bench_attn args
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS \
    -d gpurun_out/apmc/$1 -o run --output-format csv -- python3 tools/bench_attn.py --iters 2 ${@:2} > gpurun_out/apmc/$1.log 2>&1 || return 1
  f=$(find gpurun_out/apmc/$1 -name "*counter_collection.csv" | head -1)
  echo "== $1: ${@:2}" >> gpurun_out/attn_pmc_r2.txt
  grep "attn " gpurun_out/apmc/$1.log >> gpurun_out/attn_pmc_r2.txt
  python tools/pmc_summary.py "$f" attn_ >> gpurun_out/attn_pmc_r2.txt
  rm -rf gpurun_out/apmc/$1
}
: > gpurun_out/attn_pmc_r2.txt
run llama && run vit --T 197 --B 256 --H 12 --Hkv 12 --hd 64 --noncausal && run gemma --T 8192 --H 16 --Hkv 1 --hd 256
rc=$?; cat gpurun_out/attn_pmc_r2.txt; exit $rc
