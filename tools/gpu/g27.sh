set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_misc_gpu.py tests/test_conv_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/g27_t.log 2>&1; rc=$?; echo trc=$rc; tail -3 gpurun_out/g27_t.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench/vit_train.py --steps 8 --warmup 2 > gpurun_out/g27.log 2>&1; echo rc=$?
grep -v amdgpu.ids gpurun_out/g27.log | cut -c1-250
