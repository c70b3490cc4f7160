set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py tests/test_xent_gpu.py tests/test_conv_gpu.py -x -q --timeout 100 --timeout-method thread -p no:cacheprovider -k "transpose or wgrad or linear or xent or vit" > gpurun_out/g22_t.log 2>&1; rc=$?; echo trc=$rc; tail -3 gpurun_out/g22_t.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench/vit_train.py --steps 6 --warmup 2 > gpurun_out/g22.log 2>&1 && \
SPA_WGRAD_NT=0 timeout -k 10 300 python -u bench/vit_train.py --steps 6 --warmup 2 >> gpurun_out/g22.log 2>&1 && \
timeout -k 10 400 python -u bench.py --steps 6 --warmup 2 >> gpurun_out/g22.log 2>&1; echo rc=$?
grep -v amdgpu.ids gpurun_out/g22.log | cut -c1-400
