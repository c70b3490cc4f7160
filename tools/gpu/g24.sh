set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py tests/test_xent_gpu.py -x -q --timeout 100 --timeout-method thread -p no:cacheprovider -k "wgrad or bias_grad or linear or xent" > gpurun_out/g24_t.log 2>&1; rc=$?; echo trc=$rc; tail -3 gpurun_out/g24_t.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/bench_wgrad_layouts.py --vit > gpurun_out/g24.log 2>&1 && \
timeout -k 10 300 python -u tools/bench_wgrad_layouts.py >> gpurun_out/g24.log 2>&1 && \
timeout -k 10 300 python -u bench/vit_train.py --steps 6 --warmup 2 >> gpurun_out/g24.log 2>&1; echo rc=$?
grep -v amdgpu.ids gpurun_out/g24.log | cut -c1-300
