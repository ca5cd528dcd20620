# round 5: C3 (f32 MAT52-ARD N = 8192) -- f32 update kernel variants: 8 waves (WN 4), DMA after the first half
set -o pipefail
O=gpurun_out/r5t; mkdir -p $O; : > $O/c3.txt
GPK_LIB=variants/libgpk_wnf32_4.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_parity.py -k "c3 or fp32 or float32" -m gpu > $O/tests_wn4.log 2>&1; tail -1 $O/tests_wn4.log
for v in "" wnf32_4 gmidf32 "" wnf32_4 gmidf32; do
  L=gaussianprocessfundamentals_amd/libgpk.so; [ -n "$v" ] && L=variants/libgpk_$v.so
  GPK_LIB=$L timeout -k 10 200 python bench.py --config C3 --steps 60 --warmup 10 --no-cpu-baseline --no-check > $O/c3.log 2>&1 || { tail -3 $O/c3.log; exit 1; }
  echo "${v:-base} $(grep '^{' $O/c3.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["value"], r["achieved"], r["frac"])')" | tee -a $O/c3.txt
done
