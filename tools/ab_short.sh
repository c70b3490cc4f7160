# A/B of the in-tree extension (N) against ab/_C_base.so (B) on the ViT-B/16 attention shape and
# the ViT-B/16 training bench, B N N B in separate processes (round-5 short-backward rework)
set -o pipefail
O=gpurun_out/abshort
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "flash_attention or short" > ${O}_t.log 2>&1 || { tail -30 ${O}_t.log; exit 1; }
tail -2 ${O}_t.log
for arm in B N N B; do
  if [ $arm = B ]; then export SPA_EXT_SO=ab/_C_base.so; else unset SPA_EXT_SO; fi
  timeout -k 10 150 python -u tools/bench_attn.py --iters 30 --T 197 --B 256 --H 12 --Hkv 12 --hd 64 --noncausal > ${O}_a.log 2>&1 || exit 1
  echo "$arm $(grep -h 'attn B' ${O}_a.log | cut -c1-200)"
done
for arm in B N N B; do
  if [ $arm = B ]; then export SPA_EXT_SO=ab/_C_base.so; else unset SPA_EXT_SO; fi
  timeout -k 10 300 python -u bench/vit_train.py --steps 12 --warmup 3 > ${O}_v.log 2>&1 || exit 1
  echo "$arm vit $(grep -ho '"value": [0-9.]*' ${O}_v.log)"
done
