# gemm8 epilogue / tile-mapping rework: GPU tests, stamp profile, B N N B against ab/_C_base.so
set -o pipefail
O=gpurun_out/g8ab
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_moe_gpu.py tests/test_kernels_gpu.py -k "grouped_gemm or wgrad8 or moe_ffn or deepseek" > ${O}_t.log 2>&1 || { tail -30 ${O}_t.log; exit 1; }
tail -2 ${O}_t.log
SPA_EXT_SO=ab/_C_g8st.so timeout -k 10 150 python -u tools/g8_stamps.py > ${O}_st.log 2>&1 || exit 1
grep -v amdgpu.ids ${O}_st.log
for arm in B N N B; do
  if [ $arm = B ]; then export SPA_EXT_SO=ab/_C_base.so; else unset SPA_EXT_SO; fi
  timeout -k 10 150 python -u tools/g8_cases.py > ${O}_c.log 2>&1 || exit 1
  echo "$arm $(grep -v amdgpu.ids ${O}_c.log)"
done
