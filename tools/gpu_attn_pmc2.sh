#!/bin/bash
# attention micro-bench + two PMC passes (stall breakdown, MFMA/VALU/LDS) at the LLaMA3-8B shape
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 120 python tools/bench_attn.py > gpurun_out/attn_bench.log 2>&1 || exit 1
cat gpurun_out/attn_bench.log
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS -d gpurun_out/pmc1 -o run --output-format csv -- python tools/bench_attn.py --iters 2 > gpurun_out/pmc1.log 2>&1 || exit 2
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_WAVES -d gpurun_out/pmc2 -o run --output-format csv -- python tools/bench_attn.py --iters 2 > gpurun_out/pmc2.log 2>&1 || exit 3
echo done
