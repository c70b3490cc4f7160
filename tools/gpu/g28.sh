set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 100 --timeout-method thread -p no:cacheprovider -k "adamw" > gpurun_out/g28_t.log 2>&1; rc=$?; echo trc=$rc; tail -3 gpurun_out/g28_t.log
[ $rc -eq 0 ] || exit $rc
A="--preset dsv3_v3 --layers 4 --experts 32 --dense-layers 1 --seq 4096 --mb 1 --steps 4 --warmup 2"
timeout -k 10 400 python -u bench/dsv3_train.py $A > gpurun_out/g28.log 2>&1 && \
timeout -k 10 400 python -u bench/dsv3_train.py $A --bf16-moments >> gpurun_out/g28.log 2>&1 && \
timeout -k 10 400 python -u bench/dsv3_train.py $A --fp8 >> gpurun_out/g28.log 2>&1 && \
timeout -k 10 400 python -u bench/dsv3_train.py $A --fp8 --bf16-moments >> gpurun_out/g28.log 2>&1; echo rc=$?
grep -v amdgpu.ids gpurun_out/g28.log | cut -c1-220
