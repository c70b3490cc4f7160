set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "attention or attn" > gpurun_out/g35_t.log 2>&1; rc=$?; echo trc=$rc; tail -2 gpurun_out/g35_t.log
[ $rc -eq 0 ] || exit $rc
mkdir -p gpurun_out/p35
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/p35 -o run --output-format csv -- python3 -u tools/bench_attn.py --iters 20 > gpurun_out/g35.log 2>&1; echo rc=$?
grep -i "attn" gpurun_out/p35/run_kernel_stats.csv | cut -c1-150
grep "attn B" gpurun_out/g35.log
