set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py tests/test_xent_gpu.py -x -q --timeout 100 --timeout-method thread -p no:cacheprovider -k "bias_grad or wgrad or linear or xent" > gpurun_out/g23_t.log 2>&1; rc=$?; echo trc=$rc; tail -3 gpurun_out/g23_t.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench/vit_train.py --steps 6 --warmup 2 > gpurun_out/g23.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/p23 -o vit --output-format csv -- python3 bench/vit_train.py --steps 3 --warmup 1 > gpurun_out/g23p.log 2>&1; echo rc=$?
grep -v amdgpu.ids gpurun_out/g23.log | cut -c1-300
