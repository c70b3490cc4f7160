set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU -d gpurun_out/pmc34a -o run --output-format csv -- python3 tools/bench_attn.py --iters 2 > gpurun_out/g34a.log 2>&1; echo a=$?
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MFMA SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM -d gpurun_out/pmc34b -o run --output-format csv -- python3 tools/bench_attn.py --iters 2 > gpurun_out/g34b.log 2>&1; echo b=$?
ls gpurun_out/pmc34a gpurun_out/pmc34b
