set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py --steps 6 --warmup 2 > gpurun_out/g32.log 2>&1; echo brc=$?
grep -v amdgpu.ids gpurun_out/g32.log | cut -c1-300
cp tuning/tunableop_llama8b.csv gpurun_out/tunableop_llama8b.csv
timeout -k 10 600 python -u tools/tune_gemms.py tools/gpu/lmhead_untuned.csv gpurun_out/tunableop_llama8b.csv > gpurun_out/g32_tune.log 2>&1; rc=$?; echo tune=$rc
tail -5 gpurun_out/g32_tune.log
