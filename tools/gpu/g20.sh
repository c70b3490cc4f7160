set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "attention or attn" > gpurun_out/g20_t.log 2>&1; rc=$?; echo trc=$rc; tail -3 gpurun_out/g20_t.log
[ $rc -lt 124 ] || exit $rc
timeout -k 10 400 python -u bench.py --steps 6 --warmup 2 > gpurun_out/g20_b.log 2>&1; echo brc=$?
grep -v amdgpu.ids gpurun_out/g20_b.log | tail -3
