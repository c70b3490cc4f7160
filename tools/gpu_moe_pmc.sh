# MFMA / LDS counters of the MoE grouped GEMM (bf16 + fp8) at the DeepSeek-style shape
mkdir -p gpurun_out/moepmc
export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT -d gpurun_out/moepmc/a -o run --output-format csv -- python3 tools/bench_moe.py > gpurun_out/moepmc/a.log 2>&1
