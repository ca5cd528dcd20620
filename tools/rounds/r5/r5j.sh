# round 5: MFMA pair K build (compile-time D, interleaved blocks) -- tests and K build A/B over register budgets
set -o pipefail
O=gpurun_out/r5j; mkdir -p $O
timeout -k 10 600 python -u -m pytest -q --timeout 150 --timeout-method thread tests/test_gpu_kbuild.py \
  tests/test_gpu_parity.py tests/test_gpu_properties.py -m gpu > $O/tests.log 2>&1
rc=$?; grep -E "passed|failed|FAILED" $O/tests.log | tail -15
[ $rc -eq 124 ] || [ $rc -eq 134 ] || [ $rc -eq 137 ] || [ $rc -eq 139 ] && exit $rc
for v in "" asm3minb2 asm3minb3 nopairmfma "" asm3minb2 asm3minb3 nopairmfma; do
  L=gaussianprocessfundamentals_amd/libgpk.so; [ -n "$v" ] && L=variants/libgpk_$v.so
  echo "${v:-base} $(GPK_LIB=$L timeout -k 10 200 python tools/bench_kbuild.py C5 2>&1 | grep '^{' | cut -c1-140)"
done
exit $rc
