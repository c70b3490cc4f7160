set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
cp tuning/tunableop_llama8b.csv gpurun_out/tunableop_llama8b.csv
SPA_TUNE_MAX_DIM=200000 timeout -k 10 600 python -u tools/tune_gemms.py tools/gpu/lmhead_untuned2.csv gpurun_out/tunableop_llama8b.csv > gpurun_out/g33_tune.log 2>&1; rc=$?; echo tune=$rc
tail -3 gpurun_out/g33_tune.log
[ $rc -eq 0 ] || exit $rc
cp gpurun_out/tunableop_llama8b.csv tuning/tunableop_llama8b.csv
timeout -k 10 400 python -u bench.py --steps 6 --warmup 2 > gpurun_out/g33.log 2>&1; echo brc=$?
grep -v amdgpu.ids gpurun_out/g33.log | cut -c1-200
