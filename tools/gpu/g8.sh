set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof8
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > gpurun_out/g8_$name.log 2>&1; local rc=$?;
         echo "$name rc=$rc"; if [ $rc -ge 124 ]; then tail -30 gpurun_out/g8_$name.log; exit $rc; fi; }
step moe 300 python -u tools/bench_moe.py
cat gpurun_out/g8_moe.log
step pmc1 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d gpurun_out/prof8/p1 -o p1 --output-format csv -- python tools/bench_moe.py
step pmc2 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES -d gpurun_out/prof8/p2 -o p2 --output-format csv -- python tools/bench_moe.py
ls gpurun_out/prof8/*/
