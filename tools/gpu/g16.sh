set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_moe_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "grouped or deepseek or ffn or fp8" > gpurun_out/g16_t.log 2>&1; echo trc=$?; tail -2 gpurun_out/g16_t.log
timeout -k 10 300 python -u tools/bench_moe.py > gpurun_out/g16_moe.log 2>&1; echo rc=$?
grep -v "amdgpu.ids" gpurun_out/g16_moe.log
