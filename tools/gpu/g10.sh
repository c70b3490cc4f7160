set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_moe_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "grouped or deepseek or ffn" && timeout -k 10 300 env SPA_BENCH_ABLATE=1 python -u tools/bench_moe.py > gpurun_out/g10_moe.log 2>&1; echo rc=$?
cat gpurun_out/g10_moe.log
