#!/bin/bash
# rocprofv3 kernel stats of the secondary configs: Gemma-7B MQA (6 layers, T 8192) and dsv3_style (full depth)
mkdir -p gpurun_out/prof_gemma gpurun_out/prof_dsv3s
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_gemma -o run --output-format csv -- python3 bench/gemma_tp.py --layers 6 --steps 3 --warmup 1 > gpurun_out/prof_gemma/bench.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_dsv3s -o run --output-format csv -- python3 bench/dsv3_train.py --preset dsv3_style --steps 3 --warmup 1 > gpurun_out/prof_dsv3s/bench.log 2>&1
rc=$?; echo rc=$rc; grep -h metric gpurun_out/prof_gemma/bench.log gpurun_out/prof_dsv3s/bench.log | cut -c1-300
for d in prof_gemma prof_dsv3s; do
  f=$(find gpurun_out/$d -name "*kernel_stats.csv" | head -1)
  cp "$f" gpurun_out/${d}_kernel_stats.csv && python tools/prof_summary.py "$f" 3 > gpurun_out/${d}_summary.txt
  rm -rf gpurun_out/$d/*/   # traces: too large to bring back
done
cat gpurun_out/prof_gemma_summary.txt gpurun_out/prof_dsv3s_summary.txt
exit $rc
