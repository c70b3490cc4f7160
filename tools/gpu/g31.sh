# Tune the GEMM layouts the per-shape dW rule introduced (x / dy forms) into the LLaMA table.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
cp tuning/tunableop_llama8b.csv gpurun_out/tunableop_llama8b.csv
SPA_GEMM_TUNING=0 PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=0 PYTORCH_TUNABLEOP_RECORD_UNTUNED=1 \
PYTORCH_TUNABLEOP_UNTUNED_FILENAME=gpurun_out/untuned.csv PYTORCH_TUNABLEOP_FILENAME=gpurun_out/unused.csv \
  timeout -k 10 300 python bench.py --layers 2 --steps 1 --warmup 1 > gpurun_out/g31_record.log 2>&1; rc=$?; echo rec=$rc
[ $rc -eq 0 ] || exit $rc
ls gpurun_out/ | grep -i tun
SPA_TUNE_MAX_DIM=60000 timeout -k 10 780 python -u tools/tune_gemms.py gpurun_out/untuned0.csv gpurun_out/tunableop_llama8b.csv > gpurun_out/g31_tune.log 2>&1; rc=$?; echo tune=$rc
tail -12 gpurun_out/g31_tune.log
