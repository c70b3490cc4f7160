#!/bin/bash
# attention correctness (GPU tests) + micro-bench + one PMC pass at the LLaMA3-8B shape
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "flash or packed or variants" > gpurun_out/pytest_attn.log 2>&1; rc=$?; tail -5 gpurun_out/pytest_attn.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 120 python tools/bench_attn.py --ab SPA_ATTN_DKDV=1 > gpurun_out/attn_bench.log 2>&1 || exit 2
timeout -k 10 120 python tools/bench_attn.py --T 2048 --B 4 >> gpurun_out/attn_bench.log 2>&1 || exit 2
timeout -k 10 120 python tools/bench_attn.py --T 4096 --H 16 --Hkv 1 --hd 256 >> gpurun_out/attn_bench.log 2>&1 || exit 2
timeout -k 10 120 python tools/bench_attn.py --T 197 --B 64 --H 12 --Hkv 12 --hd 64 --noncausal --ab SPA_ATTN_DKDV=1 >> gpurun_out/attn_bench.log 2>&1 || exit 2
cat gpurun_out/attn_bench.log
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_BUSY_CYCLES -d gpurun_out/pmc3 -o run --output-format csv -- python tools/bench_attn.py --iters 2 > gpurun_out/pmc3.log 2>&1 || exit 3
echo done
