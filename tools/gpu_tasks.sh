#!/bin/bash
# GPU-box task runner: one named task per gpurun call, e.g.
#   gpurun --timeout 1200 -- 'bash tools/gpu_tasks.sh validate'
# Profiler databases go to /tmp on the box (gpurun copies back at most 64 MiB); only summaries
# land in gpurun_out. Every GPU step runs under its own time limit and the steps are chained: the first failing step
# ends the call (no retries). Logs and summaries go to gpurun_out/<task>_*; copy the ones worth
# keeping into profiles/.
#
# tasks:
#   start          attention micro-bench at the LLaMA shape + a short headline bench
#   validate       every GPU test, smoke(), headline bench, ViT / dsv3_style / Gemma-7B benches, B8
#   headline-prof  rocprofv3 kernel trace of 3 headline optimizer steps + per-kernel summary
#   headline-pmc   two counter passes over a 4-layer headline step (MFMA busy, HBM bytes)
#   kernels-pmc    memory-bound kernel bandwidths + LDS / VALU counter passes
#   attn-ab ENV    bench_attn.py A/B of an SPA_* switch (LLaMA, ViT and Gemma shapes), ABBA
#   parity         fp32 reference-loop parity rows B1/B3/B5/B7 and B8 end to end
#   overlap        TP / EP collective-overlap proxy (tools/overlap_proxy.py)
#   dsv3-prof      dsv3_style at accum 1 and 4, kernel trace at accum 4
#   vit-gemma-prof kernel traces of one ViT-B/16 and one Gemma-7B (28 layers) optimizer step
#   gemm-ab V..    gemm8 default vs SPA_GG8_ABLATE=V (dense 8192^3 + dsv3_style grouped), ABBA
#   gemm-validate  GEMM/MoE GPU tests, schedule A/B vs the round-2 one, dsv3_style + ViT benches
#   defer-ab       MoE GPU tests; dsv3_style accum 4 with / without deferred expert Wgrad, ABBA
#   g8-e2e         dsv3_style (accum 4) and ViT-B/16 with the shipped gemm8 vs the round-2 one, ABBA
#   gemm-pmc       gemm8 vs hipBLASLt on a dense 8192^3 + one counter pass
#   attn-ds        dS-materialising backward: GPU tests, attention ABBA vs the dq kernel, headline bench
#   attn-quick     attention GPU tests, packed-layout ABBA vs the dq kernel, per-kernel times
#   ep-pair        micro-batch-pair EP overlap: MoE GPU tests, EP=8 proxy, dsv3_style pairs vs one-by-one ABBA
#   headline-ab ENV  bench.py default vs ENV=VAL, separate processes in ABBA order
#   headline-args A  bench.py default vs extra bench.py arguments A, ABBA
#   ext-ab K C     in-tree build vs $BASE_SO: GPU tests -k K, bench_kernels case C, headline, B N N B
#   attn-pmc       attention counters + clocks in the headline step (4 layers) and in isolation; GEMM-interleaved timing
#   secondary      ViT-B/16, dsv3_style, dsv3_v3 (bf16 + fp8), Gemma-7B benches
#   dkdv5          dS-path GPU tests (incl. the v5 dK/dV kernel), LLaMA-shape ABBA SPA_ATTN_DKDV5=1, kernel times
#   dkdv5-var      dkdv5 variants vs dkdv3 (ABBA, one process) + stamp profiles of dkdv3 / dkdv5 variants
#   epcap [CF]     capacity-mode EP dispatch: MoE GPU tests + EP=8 proxy one-by-one exact vs capacity
#   dbgbounds      debug-bounds build (device guards) over the ragged-shape GPU cases
#   gradprec [N]   bf16-vs-fp32 gradient accumulation: 8B-width error test + N-step loss-curve A/B
#   v3mem          dsv3_v3 fp8 (4 layers, accum 4) unforced vs through a 1-rank RCCL group: peak memory after the Work fix
#   env-ab ENV CMD B N N B of one env switch on any bench command (separate processes)
#   opt-overlap    kernel traces of the headline at side-stream priority 0 / -1 (optimizer overlap)
#   rccl           world-1 RCCL test (every collective path) + headline ABBA with TENSILE_STREAMK_DATA_PARALLEL=1
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
task=${1:?task}; shift
O=gpurun_out/$task

run() {  # run <seconds> <log> <cmd...>: one GPU step under its own limit; stop the call on failure
  local t=$1 log=$2; shift 2
  timeout -k 10 "$t" "$@" > "$log" 2>&1
  local rc=$?
  echo "[$rc] $*"
  if [ $rc -ne 0 ]; then tail -20 "$log"; exit $rc; fi
}
jsonl() { grep -h '^{' "$@" | cut -c1-600; }

case $task in
dkdv5)
  run 300 ${O}_pytest.log python -u -m pytest tests/test_kernels_gpu.py -k "ds_path" -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
  tail -2 ${O}_pytest.log
  run 200 ${O}_ab.log python -u tools/bench_attn.py --iters 20 --packed --ab SPA_ATTN_DKDV5=1
  grep -h 'attn B\|with SPA' ${O}_ab.log | cut -c1-300
  run 200 ${O}_ab2.log python -u tools/bench_attn.py --iters 20 --packed --ab SPA_ATTN_DKDV5=1
  grep -h 'with SPA' ${O}_ab2.log | cut -c1-300
  export SPA_ATTN_DKDV5=1
  run 200 ${O}_prof.log rocprofv3 --kernel-trace --stats -d /tmp/$task -o run -- python3 tools/bench_attn.py --iters 10 --packed
  unset SPA_ATTN_DKDV5
  python tools/rocpd_summary.py /tmp/$task/run_results.db --top 8 > ${O}_summary.txt 2>&1
  head -14 ${O}_summary.txt | cut -c1-150 ;;
dkdv5-var)
  # dkdv5-var "1,5,9" "1 9": SPA_ATTN_DKDV5 variants vs dkdv3 (ABBA, one process), then stamp profiles
  vs=${1:-1,3,5,7}; sv=${2:-0 1}
  run 300 ${O}_ab.log python -u tools/bench_attn.py --iters 20 --packed --ab $(echo $vs | sed 's/\([0-9]*\)/SPA_ATTN_DKDV5=\1/g')
  grep -h 'attn B\|with SPA' ${O}_ab.log | cut -c1-300
  for v in $sv; do
    run 200 ${O}_st$v.log env SPA_EXT_SO=ab/_C_stamp5.so SPA_ATTN_STAMP=1 SPA_ATTN_DKDV5=$v python -u tools/bench_attn.py --iters 5 --packed
    echo "== SPA_ATTN_DKDV5=$v (stamp build)"; grep -h 'attn B\|role' ${O}_st$v.log | cut -c1-300
  done ;;
preflight)
  # multi-GPU pre-flight on one GPU: GPU tests of the forced-collective benches,
  # the N=8 DP-reduction numerics, full-size benches unforced vs forced through a 1-rank nccl group
  run 600 ${O}_pytest.log python -u -m pytest tests/test_preflight_gpu.py tests/test_rccl_gpu.py -x -v -p no:cacheprovider --timeout 300 --timeout-method thread
  grep -h 'PASS\|FAIL\|passed\|failed' ${O}_pytest.log | cut -c1-200
  run 400 ${O}_ring.log python -u tools/grad_precision.py --mode ring --layers 2
  jsonl ${O}_ring.log
  TR="python -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr=127.0.0.1 --master-port=29533"
  run 400 ${O}_b0.log python -u bench.py --steps 6 --warmup 2
  run 400 ${O}_b1.log env SPA_FORCE_COLLECTIVES=1 $TR bench.py --steps 6 --warmup 2
  run 400 ${O}_b2.log env SPA_FORCE_COLLECTIVES=1 SPA_DP_REDUCE=ring $TR bench.py --steps 6 --warmup 2
  run 400 ${O}_b3.log env SPA_FORCE_COLLECTIVES=1 $TR bench.py --steps 6 --warmup 2 --zero1
  run 400 ${O}_b4.log python -u bench.py --steps 6 --warmup 2
  jsonl ${O}_b?.log
  V3="--preset dsv3_v3 --layers 4 --dense-layers 1 --experts 32 --mb 1 --accum 4 --steps 3 --warmup 1 --fp8"
  run 400 ${O}_v0.log python -u bench/dsv3_train.py $V3
  run 400 ${O}_v1.log env SPA_FORCE_COLLECTIVES=1 $TR bench/dsv3_train.py $V3
  jsonl ${O}_v?.log ;;
v3mem)
  TR="python -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr=127.0.0.1 --master-port=29533"
  V3="--preset dsv3_v3 --layers 4 --dense-layers 1 --experts 32 --mb 1 --accum 4 --steps 3 --warmup 1 --fp8"
  run 400 ${O}_v0.log python -u bench/dsv3_train.py $V3
  run 400 ${O}_v1.log env SPA_FORCE_COLLECTIVES=1 $TR bench/dsv3_train.py $V3
  run 400 ${O}_v2.log python -u bench/dsv3_train.py $V3
  run 400 ${O}_v3.log env SPA_FORCE_COLLECTIVES=1 $TR bench/dsv3_train.py $V3
  jsonl ${O}_v?.log ;;
rccl)
  run 300 ${O}_pytest.log python -u -m pytest tests/test_rccl_gpu.py -x -v -s -p no:cacheprovider --timeout 240 --timeout-method thread
  grep -h 'rccl-world1\|passed\|failed' ${O}_pytest.log | cut -c1-200
  for arm in base var var base; do
    if [ $arm = var ]; then run 400 ${O}_$arm.log env TENSILE_STREAMK_DATA_PARALLEL=1 python -u bench.py --steps 6 --warmup 2
    else run 400 ${O}_$arm.log python -u bench.py --steps 6 --warmup 2; fi
    echo "$arm streamk_dp $(grep -ho '"value": [0-9.]*' ${O}_$arm.log)"
  done ;;
epcap)
  # host-sync-free (capacity) EP dispatch: MoE GPU tests, then the EP=8 proxy at accum-1 form
  run 400 ${O}_pytest.log python -u -m pytest tests/test_moe_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
  tail -2 ${O}_pytest.log
  run 600 ${O}_proxy.log python -u tools/overlap_proxy.py --which ep --layers 2 --capacity ${1:-1.25}
  run 600 ${O}_proxyb.log python -u tools/overlap_proxy.py --which ep --layers 2 --capacity ${1:-1.25} --balanced
  grep -hv amdgpu.ids ${O}_proxy.log ${O}_proxyb.log | cut -c1-1200 ;;
dbgbounds)
  # debug-bounds build (ab/_C_dbg.so) over the ragged-shape GPU cases; guards must stay silent
  run 900 ${O}_pytest.log python -u -m pytest tests/test_debug_bounds_gpu.py -x -v -s -p no:cacheprovider --timeout 900 --timeout-method thread
  grep -h "passed\|failed\|SPA_DEBUG_BOUNDS\|Error" ${O}_pytest.log | cut -c1-300 | tail -20 ;;
gradprec)
  # bf16 vs fp32 gradient accumulation: the 8B-width GPU test, then the loss-curve A/B
  run 300 ${O}_pytest.log python -u -m pytest tests/test_grad_precision_gpu.py -x -v -s -p no:cacheprovider --timeout 240 --timeout-method thread
  grep -h "rel_err\|passed\|failed" ${O}_pytest.log | cut -c1-900
  run 900 ${O}_curve.log python -u tools/grad_precision.py --mode curve --steps ${1:-500}
  grep -h summary ${O}_curve.log ;;
start)
  run 300 ${O}_attn.log python -u tools/bench_attn.py
  grep -i 'attn B' ${O}_attn.log | cut -c1-300
  run 400 ${O}_bench.log python -u bench.py --steps 8 --warmup 2
  jsonl ${O}_bench.log ;;
validate)
  run 900 ${O}_pytest.log python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
  tail -2 ${O}_pytest.log
  run 180 ${O}_smoke.log python -c "import __graft_entry__ as g; g.smoke()"
  tail -1 ${O}_smoke.log
  # the driver's headline window (20 timed steps), secondary benches over >= 10 steps
  run 600 ${O}_bench.log python -u bench.py --steps 20 --warmup 3
  run 300 ${O}_vit.log python -u bench/vit_train.py --steps 20 --warmup 5
  run 300 ${O}_dsv3s.log python -u bench/dsv3_train.py --preset dsv3_style --steps 10 --warmup 2
  V3="--preset dsv3_v3 --layers 4 --dense-layers 1 --experts 32 --mb 1 --accum 4 --steps 10 --warmup 1"
  run 300 ${O}_v3.log python -u bench/dsv3_train.py $V3
  run 300 ${O}_v3fp8.log python -u bench/dsv3_train.py $V3 --fp8
  run 400 ${O}_gemma.log python -u bench/gemma_tp.py --layers 28 --steps 10 --warmup 1
  jsonl ${O}_bench.log ${O}_vit.log ${O}_dsv3s.log ${O}_v3.log ${O}_v3fp8.log ${O}_gemma.log ;;
headline-prof)
  run 400 ${O}.log rocprofv3 --kernel-trace --stats -d /tmp/$task -o run -- python3 bench.py --steps 2 --warmup 1
  jsonl ${O}.log
  python tools/rocpd_summary.py /tmp/$task/run_results.db --last-step adamw --top 40 > ${O}_summary.txt 2>&1
  head -50 ${O}_summary.txt | cut -c1-160 ;;
env-ab)
  # env-ab SPA_X=v "bench/dsv3_train.py --preset dsv3_style --steps 10 --warmup 2": B N N B, separate processes
  ab=${1:?SPA_X=v}; cmd=${2:?bench command}
  for arm in base var var base; do
    if [ $arm = var ]; then run 400 ${O}_$arm.log env $ab python -u $cmd
    else run 400 ${O}_$arm.log python -u $cmd; fi
    echo "$arm $ab $(grep -ho '"value": [0-9.]*' ${O}_$arm.log)"
  done ;;
opt-overlap)
  # does the side-stream AdamW co-run with the next step's forward? kernel traces at the default and
  # at high side-stream priority (SPA_OPT_PRIO=-1): busy-union vs summed kernel time per arm
  for pr in 0 -1; do
    run 400 ${O}_$pr.log env SPA_OPT_PRIO=$pr rocprofv3 --kernel-trace -d /tmp/${task}_$pr -o run -- python3 bench.py --steps 3 --warmup 1
    jsonl ${O}_$pr.log
    python tools/rocpd_summary.py /tmp/${task}_$pr/run_results.db --top 4 > ${O}_${pr}_summary.txt 2>&1
    echo "== SPA_OPT_PRIO=$pr"; head -8 ${O}_${pr}_summary.txt | cut -c1-160
  done ;;
headline-pmc)
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE \
    -d ${O}_a -o run --output-format csv -- python3 bench.py --layers 4 --steps 1 --warmup 1 > ${O}_a.log 2>&1 || exit 1
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc FETCH_SIZE \
    -d ${O}_b -o run --output-format csv -- python3 bench.py --layers 4 --steps 1 --warmup 1 > ${O}_b.log 2>&1 || exit 2
  python tools/pmc_step_summary.py "$(find ${O}_a -name '*counter_collection.csv' | head -1)" \
    "$(find ${O}_b -name '*counter_collection.csv' | head -1)" > ${O}.txt
  rm -rf ${O}_a ${O}_b
  cat ${O}.txt ;;
kernels-pmc)
  run 180 ${O}_bw.jsonl python -u tools/bench_kernels.py --iters 20
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT FETCH_SIZE \
    -d ${O}_a -o run --output-format csv -- python3 tools/bench_kernels.py --iters 2 > ${O}_a.log 2>&1 || exit 1
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc WRITE_SIZE GRBM_GPU_ACTIVE \
    -d ${O}_b -o run --output-format csv -- python3 tools/bench_kernels.py --iters 2 > ${O}_b.log 2>&1 || exit 2
  for d in ${O}_a ${O}_b; do python tools/pmc_summary.py "$(find $d -name '*counter_collection.csv' | head -1)"; done > ${O}.txt 2>&1
  cat ${O}.txt ;;
attn-ab)
  ab=${1:?SPA_X=v[,SPA_Y=w]}
  for i in 1 2; do
    run 150 ${O}_llama_$i.log python -u tools/bench_attn.py --iters 20 --ab "$ab"
    run 150 ${O}_vit_$i.log python -u tools/bench_attn.py --iters 20 --T 197 --B 256 --H 12 --Hkv 12 --hd 64 --noncausal --ab "$ab"
    run 150 ${O}_gemma_$i.log python -u tools/bench_attn.py --iters 10 --T 8192 --H 16 --Hkv 1 --hd 256 --ab "$ab"
  done
  grep -h 'attn B' ${O}_*.log | cut -c1-300 ;;
parity)
  run 900 ${O}_fp32.log python -u bench/parity.py --which B1,B3,B5,B7 --dtype fp32 --ref-loop --graph
  run 600 ${O}_b8.log python -u bench/parity.py --which B8 --ref-loop --graph
  jsonl ${O}_fp32.log ${O}_b8.log ;;
overlap)
  run 400 ${O}.log python -u tools/overlap_proxy.py --layers 2
  grep -v amdgpu.ids ${O}.log | cut -c1-900 ;;
attn-ds)
  run 300 ${O}_pytest.log python -u -m pytest tests/test_kernels_gpu.py -k "ds_path or flash" -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
  tail -2 ${O}_pytest.log
  run 200 ${O}_ab.log python -u tools/bench_attn.py --iters 20 --interleave --ab SPA_ATTN_DQ_DS=0
  grep -h 'attn B\|after a GEMM\|with SPA' ${O}_ab.log | cut -c1-300
  run 400 ${O}_bench.log python -u bench.py --steps 6 --warmup 2
  jsonl ${O}_bench.log ;;
attn-quick)
  # attention GPU tests + packed-layout ABBA vs the dq kernel + per-kernel times
  run 300 ${O}_pytest.log python -u -m pytest tests/test_kernels_gpu.py -k "ds_path or flash" -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
  tail -2 ${O}_pytest.log
  run 200 ${O}_ab.log python -u tools/bench_attn.py --iters 20 --packed --ab SPA_ATTN_DQ_DS=0
  grep -h 'attn B\|with SPA' ${O}_ab.log | cut -c1-300
  run 200 ${O}_prof.log rocprofv3 --kernel-trace --stats -d /tmp/$task -o run -- python3 tools/bench_attn.py --iters 10 --packed
  python tools/rocpd_summary.py /tmp/$task/run_results.db --top 8 > ${O}_summary.txt 2>&1
  head -14 ${O}_summary.txt | cut -c1-150 ;;
ep-pair)
  # micro-batch-pair EP overlap: GPU tests, the 1-GPU EP=8 proxy, dsv3_style accum 4 pairs vs one by one (ABBA)
  run 400 ${O}_pytest.log python -u -m pytest tests/test_moe_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
  tail -2 ${O}_pytest.log
  run 500 ${O}_proxy.log python -u tools/overlap_proxy.py --which ep --layers 2
  grep -v amdgpu.ids ${O}_proxy.log | cut -c1-900
  for arm in pair one one pair; do
    flag=""; [ $arm = one ] && flag="--no-pair"
    run 300 ${O}_$arm.log python -u bench/dsv3_train.py --preset dsv3_style --steps 3 --warmup 1 --accum 4 $flag
    echo "$arm $(grep -ho '"value": [0-9.]*' ${O}_$arm.log)"
  done ;;
headline-ab)
  # headline bench.py A/B of one env switch, separate processes in ABBA order: headline-ab SPA_X=v
  ab=${1:?SPA_X=v}
  for arm in base var var base; do
    if [ $arm = var ]; then run 400 ${O}_$arm.log env $ab python -u bench.py --steps 6 --warmup 2
    else run 400 ${O}_$arm.log python -u bench.py --steps 6 --warmup 2; fi
    echo "$arm $ab $(grep -ho '"value": [0-9.]*' ${O}_$arm.log)"
  done ;;
headline-args)
  # headline bench.py default vs extra bench.py arguments, ABBA: headline-args "--mb 2 --accum 2"
  extra=${1:?bench args}
  for arm in base var var base; do
    if [ $arm = var ]; then run 400 ${O}_$arm.log python -u bench.py --steps 6 --warmup 2 $extra
    else run 400 ${O}_$arm.log python -u bench.py --steps 6 --warmup 2; fi
    echo "$arm $extra $(grep -ho '"value": [0-9.]*\|"mem_gb": [0-9.]*' ${O}_$arm.log | tr '\n' ' ')"
  done ;;
ext-ab)
  # in-tree extension (N) vs another build (B, SPA_EXT_SO=$BASE_SO): pytest -k EXPR, the
  # bench_kernels.py case KCASE and the headline bench, each in separate processes B N N B
  expr=${1:?pytest -k expr}; kcase=${2:?bench_kernels case}; base=${BASE_SO:-ab/_C_base.so}
  run 300 ${O}_pytest.log python -u -m pytest tests -m gpu -k "$expr" -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
  tail -1 ${O}_pytest.log
  for arm in B N N B; do
    if [ $arm = B ]; then export SPA_EXT_SO=$base; else unset SPA_EXT_SO; fi
    run 120 ${O}_k.log python -u tools/bench_kernels.py --only $kcase --iters 20
    echo "$arm $(grep -h '^{' ${O}_k.log)"
  done
  for arm in B N N B; do
    if [ $arm = B ]; then export SPA_EXT_SO=$base; else unset SPA_EXT_SO; fi
    run 400 ${O}_h.log python -u bench.py --steps 6 --warmup 2
    echo "$arm headline $(grep -ho '"value": [0-9.]*' ${O}_h.log)"
  done
  unset SPA_EXT_SO ;;
attn-pmc)
  run 200 ${O}_il.log python -u tools/bench_attn.py --iters 20 --interleave
  grep -h 'attn B\|after a GEMM' ${O}_il.log
  C="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY GRBM_GUI_ACTIVE"
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $C -d ${O}_a -o run --output-format csv -- python3 bench.py --layers 4 --steps 1 --warmup 1 > ${O}_a.log 2>&1 || { tail -5 ${O}_a.log; exit 1; }
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $C -d ${O}_b -o run --output-format csv -- python3 tools/bench_attn.py --iters 3 > ${O}_b.log 2>&1 || { tail -5 ${O}_b.log; exit 2; }
  { echo "== in situ (bench.py --layers 4)"; python tools/pmc_summary.py "$(find ${O}_a -name '*counter_collection.csv' | head -1)" attn Cijk;
    echo "== isolated (tools/bench_attn.py)"; python tools/pmc_summary.py "$(find ${O}_b -name '*counter_collection.csv' | head -1)" attn; } > ${O}.txt 2>&1
  rm -rf ${O}_a ${O}_b
  cut -c1-250 ${O}.txt ;;
secondary)
  run 300 ${O}_vit.log python -u bench/vit_train.py --steps 20 --warmup 5
  run 300 ${O}_dsv3s.log python -u bench/dsv3_train.py --preset dsv3_style --steps 4 --warmup 2
  # dsv3_v3 widths at one EP=8 rank's share (4 layers, 1 dense, 32 of the 256 experts): the full
  # 61-layer model does not fit one GPU
  V3="--preset dsv3_v3 --layers 4 --dense-layers 1 --experts 32 --mb 1 --accum 4 --steps 3 --warmup 1"
  run 300 ${O}_v3.log python -u bench/dsv3_train.py $V3
  run 300 ${O}_v3fp8.log python -u bench/dsv3_train.py $V3 --fp8
  run 300 ${O}_v3fp8b.log python -u bench/dsv3_train.py $V3 --fp8
  run 300 ${O}_v3b.log python -u bench/dsv3_train.py $V3
  run 400 ${O}_gemma.log python -u bench/gemma_tp.py --layers 28 --steps 3 --warmup 1
  jsonl ${O}_*.log ;;
dsv3-prof)
  run 300 ${O}_a1.log python -u bench/dsv3_train.py --preset dsv3_style --steps 4 --warmup 2
  run 300 ${O}_a4.log python -u bench/dsv3_train.py --preset dsv3_style --steps 3 --warmup 1 --accum 4
  jsonl ${O}_a1.log ${O}_a4.log
  run 400 ${O}_prof.log rocprofv3 --kernel-trace --stats -d /tmp/$task -o run -- python3 bench/dsv3_train.py --preset dsv3_style --steps 2 --warmup 1 --accum 4
  python tools/rocpd_summary.py /tmp/$task/run_results.db --last-step adamw --top 45 > ${O}_summary.txt 2>&1
  head -60 ${O}_summary.txt | cut -c1-170 ;;
vit-gemma-prof)
  run 300 ${O}_vit.log rocprofv3 --kernel-trace --stats -d /tmp/${task}_v -o run -- python3 bench/vit_train.py --steps 3 --warmup 2
  python tools/rocpd_summary.py /tmp/${task}_v/run_results.db --last-step adamw --top 30 > ${O}_vit_summary.txt 2>&1
  head -40 ${O}_vit_summary.txt | cut -c1-170
  run 400 ${O}_gemma.log rocprofv3 --kernel-trace --stats -d /tmp/${task}_g -o run -- python3 bench/gemma_tp.py --layers 28 --steps 2 --warmup 1
  python tools/rocpd_summary.py /tmp/${task}_g/run_results.db --last-step adamw --top 30 > ${O}_gemma_summary.txt 2>&1
  head -40 ${O}_gemma_summary.txt | cut -c1-170 ;;
gemm-ab)
  for v in "${@:?schedule}"; do
    run 300 ${O}_$v.log python -u tools/bench_gemm8_dense.py 8192 --iters 10 --ab $v
    grep -v amdgpu.ids ${O}_$v.log
  done ;;
gemm-validate)
  run 400 ${O}_pytest.log python -u -m pytest tests/test_moe_gpu.py tests/test_kernels_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
  tail -2 ${O}_pytest.log
  run 300 ${O}_ab.log python -u tools/bench_gemm8_dense.py 8192 --iters 10 --ab 8
  grep -v amdgpu.ids ${O}_ab.log
  run 300 ${O}_dsv3a1.log python -u bench/dsv3_train.py --preset dsv3_style --steps 4 --warmup 2
  run 300 ${O}_dsv3a4.log python -u bench/dsv3_train.py --preset dsv3_style --steps 3 --warmup 1 --accum 4
  run 300 ${O}_vit.log python -u bench/vit_train.py --steps 20 --warmup 5
  jsonl ${O}_dsv3a1.log ${O}_dsv3a4.log ${O}_vit.log ;;
g8-e2e)
  for arm in new old old new; do
    if [ $arm = old ]; then export SPA_GG8_ABLATE=8; else unset SPA_GG8_ABLATE; fi
    run 300 ${O}_d_$arm.log python -u bench/dsv3_train.py --preset dsv3_style --steps 3 --warmup 1 --accum 4
    run 300 ${O}_v_$arm.log python -u bench/vit_train.py --steps 20 --warmup 5
    echo "$arm $(grep -ho '"value": [0-9.]*' ${O}_d_$arm.log ${O}_v_$arm.log | tr '\n' ' ')"
  done
  unset SPA_GG8_ABLATE ;;
lpt)
  run 300 ${O}_pytest.log python -u -m pytest tests/test_moe_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
  tail -2 ${O}_pytest.log
  run 300 ${O}_ab.log python -u tools/bench_gemm8_dense.py 8192 --iters 10 --ab 8
  grep -v amdgpu.ids ${O}_ab.log
  run 300 ${O}_a4.log python -u bench/dsv3_train.py --preset dsv3_style --steps 3 --warmup 1 --accum 4
  run 300 ${O}_a1.log python -u bench/dsv3_train.py --preset dsv3_style --steps 4 --warmup 2
  jsonl ${O}_a4.log ${O}_a1.log ;;
defer-ab)
  run 300 ${O}_pytest.log python -u -m pytest tests/test_moe_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
  tail -2 ${O}_pytest.log
  for arm in on off off on; do
    flag="--defer-wgrad"; [ $arm = off ] && flag="--no-defer-wgrad"
    run 300 ${O}_$arm.log python -u bench/dsv3_train.py --preset dsv3_style --steps 3 --warmup 1 --accum 4 $flag
    echo "$arm $(grep -h '^{' ${O}_$arm.log | cut -c1-200)"
  done ;;
defer-prof)
  for arm in on off; do
    flag="--defer-wgrad"; [ $arm = off ] && flag="--no-defer-wgrad"
    run 400 ${O}_$arm.log rocprofv3 --kernel-trace --stats -d /tmp/${task}_$arm -o run -- python3 bench/dsv3_train.py --preset dsv3_style --steps 2 --warmup 1 --accum 4 $flag
    python tools/rocpd_summary.py /tmp/${task}_$arm/run_results.db --last-step adamw --top 30 > ${O}_$arm.txt 2>&1
    head -24 ${O}_$arm.txt | cut -c1-150
  done ;;
g4wire)
  # gemm4a / gemm4r wiring: GPU tests, then ViT-B/16 (wgrad8 partials: gemm4r vs gemm8) and dsv3_style
  # (expert dW: gemm4r vs gemm8), each default (N) vs the gemm8 path (B), B N N B
  run 600 ${O}_pytest.log python -u -m pytest tests/test_gemm4a_gpu.py tests/test_moe_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
  tail -2 ${O}_pytest.log
  for arm in B N N B; do
    if [ $arm = B ]; then export SPA_WGRAD_G4=0 SPA_GG_DW=g8; else unset SPA_WGRAD_G4 SPA_GG_DW; fi
    run 300 ${O}_vit.log python -u bench/vit_train.py --steps 20 --warmup 5
    echo "$arm vit $(grep -ho '"value": [0-9.]*' ${O}_vit.log)"
    run 400 ${O}_s.log python -u bench/dsv3_train.py --preset dsv3_style --steps 10 --warmup 3
    echo "$arm dsv3_style $(grep -ho '"value": [0-9.]*' ${O}_s.log)"
  done
  unset SPA_WGRAD_G4 SPA_GG_DW ;;
mapab)
  # grouped-GEMM tile mapping (real tiles on the lowest block ids) vs the previous build
  # (B = SPA_EXT_SO=ab/_C_premap.so), dsv3_style accum 1 and dsv3_v3 fp8 accum 4, B N N B
  base=${BASE_SO:-ab/_C_premap.so}
  V3="--preset dsv3_v3 --layers 4 --dense-layers 1 --experts 32 --mb 1 --accum 4 --steps 6 --warmup 2 --fp8"
  for arm in B N N B; do
    if [ $arm = B ]; then export SPA_EXT_SO=$base; else unset SPA_EXT_SO; fi
    run 400 ${O}_s.log python -u bench/dsv3_train.py --preset dsv3_style --steps 10 --warmup 3
    echo "$arm dsv3_style $(grep -ho '"value": [0-9.]*' ${O}_s.log)"
    run 400 ${O}_v.log python -u bench/dsv3_train.py $V3
    echo "$arm dsv3_v3_fp8 $(grep -ho '"value": [0-9.]*' ${O}_v.log)"
  done
  unset SPA_EXT_SO ;;
g4pmc)
  # gemm4a (register-staged) vs gemm8 vs hipBLASLt, dense 8192^3: two counter passes
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS GRBM_GUI_ACTIVE \
    -d ${O}_a -o run --output-format csv -- python3 tools/gemm4a_pmc_prog.py > ${O}_a.log 2>&1 || { tail -5 ${O}_a.log; exit 1; }
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_INSTS_LDS TCC_HIT_sum TCC_MISS_sum \
    -d ${O}_b -o run --output-format csv -- python3 tools/gemm4a_pmc_prog.py > ${O}_b.log 2>&1 || { tail -5 ${O}_b.log; exit 1; }
  for d in ${O}_a ${O}_b; do python tools/pmc_summary.py "$(find $d -name '*counter_collection.csv' | head -1)"; done > ${O}.txt 2>&1
  rm -rf ${O}_a ${O}_b
  cat ${O}.txt | cut -c1-600 ;;
gemm-pmc)
  run 120 ${O}_bench.log python -u tools/bench_gemm8_dense.py 8192 --iters 20
  cat ${O}_bench.log | grep -v amdgpu.ids
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE \
    -d ${O}_a -o run --output-format csv -- python3 tools/bench_gemm8_dense.py 8192 --iters 3 > ${O}_a.log 2>&1 || { tail -5 ${O}_a.log; exit 1; }
  python tools/pmc_summary.py "$(find ${O}_a -name '*counter_collection.csv' | head -1)" > ${O}.txt 2>&1
  cat ${O}.txt | cut -c1-400 ;;
*)
  echo "unknown task $task"; exit 2 ;;
esac
