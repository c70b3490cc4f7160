# per-kernel bandwidth of the memory-bound HIP kernels + two rocprofv3 counter passes
mkdir -p gpurun_out/kpmc
export TMPDIR=/tmp
timeout -k 10 180 python -u tools/bench_kernels.py --iters 20 > gpurun_out/kpmc/bw.jsonl 2> gpurun_out/kpmc/bw.err &&
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT FETCH_SIZE -d gpurun_out/kpmc/a -o run --output-format csv -- python3 tools/bench_kernels.py --iters 2 > gpurun_out/kpmc/a.log 2>&1 &&
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc WRITE_SIZE GRBM_GPU_ACTIVE -d gpurun_out/kpmc/b -o run --output-format csv -- python3 tools/bench_kernels.py --iters 2 > gpurun_out/kpmc/b.log 2>&1
