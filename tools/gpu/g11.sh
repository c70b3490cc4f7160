set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > gpurun_out/g11_$name.log 2>&1; local rc=$?;
         echo "$name rc=$rc"; if [ $rc -ge 124 ]; then tail -30 gpurun_out/g11_$name.log; exit $rc; fi; }
step tests 600 python -u -m pytest tests/test_moe_gpu.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider
tail -4 gpurun_out/g11_tests.log
grep -E "FAIL|Error|assert" gpurun_out/g11_tests.log | head -20
true
true
step dsv3bf 400 python -u bench/dsv3_train.py --preset dsv3_v3 --layers 4 --experts 32 --dense-layers 1 --seq 4096 --mb 1 --steps 4 --warmup 2
grep '^{' gpurun_out/g11_dsv3bf.log
step dsv3f8 400 python -u bench/dsv3_train.py --preset dsv3_v3 --layers 4 --experts 32 --dense-layers 1 --seq 4096 --mb 1 --steps 4 --warmup 2 --fp8 && step dsv3f8e 400 python -u bench/dsv3_train.py --preset dsv3_v3 --layers 4 --experts 32 --dense-layers 1 --seq 4096 --mb 1 --steps 4 --warmup 2 --fp8 --fp8-experts-only
grep -h "^{" gpurun_out/g11_dsv3f8.log gpurun_out/g11_dsv3f8e.log
step dsv3bfa 400 python -u bench/dsv3_train.py --preset dsv3_v3 --layers 4 --experts 32 --dense-layers 1 --seq 4096 --mb 1 --accum 4 --steps 3 --warmup 1
step dsv3f8a 400 python -u bench/dsv3_train.py --preset dsv3_v3 --layers 4 --experts 32 --dense-layers 1 --seq 4096 --mb 1 --accum 4 --steps 3 --warmup 1 --fp8
grep -h "^{" gpurun_out/g11_dsv3bfa.log gpurun_out/g11_dsv3f8a.log
