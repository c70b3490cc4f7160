#!/bin/bash
# counter pass over a 4-layer LLaMA3-8B-shape training step: MFMA-busy share and HBM bytes per kernel
mkdir -p gpurun_out/hpmc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE \
  -d gpurun_out/hpmc/a -o run --output-format csv -- python3 bench.py --layers 4 --steps 1 --warmup 1 > gpurun_out/hpmc/a.log 2>&1 || exit 1
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc FETCH_SIZE \
  -d gpurun_out/hpmc/b -o run --output-format csv -- python3 bench.py --layers 4 --steps 1 --warmup 1 > gpurun_out/hpmc/b.log 2>&1 || exit 2
fa=$(find gpurun_out/hpmc/a -name "*counter_collection.csv" | head -1)
fb=$(find gpurun_out/hpmc/b -name "*counter_collection.csv" | head -1)
python tools/pmc_step_summary.py "$fa" "$fb" > gpurun_out/headline_pmc.txt
rm -rf gpurun_out/hpmc/a gpurun_out/hpmc/b
cat gpurun_out/headline_pmc.txt
