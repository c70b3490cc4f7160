set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_parallel_tp_ep_gpu.py tests/test_xent_gpu.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/g2_pytest.log 2>&1; echo "pytest rc=$?" >> gpurun_out/g2_pytest.log
tail -15 gpurun_out/g2_pytest.log
timeout -k 10 300 python -u tools/bench_xent.py > gpurun_out/g2_xent.jsonl 2>&1; echo "xent rc=$?"
cat gpurun_out/g2_xent.jsonl
