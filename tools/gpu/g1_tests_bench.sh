set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/g1_pytest.log 2>&1; echo "pytest rc=$?" >> gpurun_out/g1_pytest.log
tail -5 gpurun_out/g1_pytest.log
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 > gpurun_out/g1_bench.log 2>&1; echo "bench rc=$?"
tail -3 gpurun_out/g1_bench.log
