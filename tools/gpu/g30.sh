set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/g30_t.log 2>&1; rc=$?; echo trc=$rc
grep -E "passed|failed|error" gpurun_out/g30_t.log | tail -5
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/g30_s.log 2>&1; echo src=$?; tail -2 gpurun_out/g30_s.log
