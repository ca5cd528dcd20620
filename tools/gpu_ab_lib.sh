# A/B of a variant libgpk ($VARLIB) against the default build on one box: the variant's parity tests
# ($TESTS), then tools/single_sched.py ($SETS, sizes $SIZES) alternating base / var / base / var.
set -o pipefail
: "${VARLIB:?}" "${TESTS:=tests/test_gpu_fused_panel.py tests/test_gpu_diag_versions.py}" "${SIZES:=1024 4096 8192}"
GPK_LIB=$VARLIB timeout -k 10 300 python -u -m pytest $TESTS -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_tests.log 2>&1 || { tail -20 gpurun_out/ab_tests.log; exit 1; }
echo "var tests: $(tail -1 gpurun_out/ab_tests.log)"
for rep in 1 2; do
  for v in base var; do
    if [ $v = var ]; then L=$VARLIB; else L=$PWD/gaussianprocessfundamentals_amd/libgpk.so; fi
    GPK_LIB=$L timeout -k 10 200 python tools/single_sched.py $SIZES > gpurun_out/ab_${v}${rep}.log 2>&1 || { tail -5 gpurun_out/ab_${v}${rep}.log; exit 1; }
    grep '^{' gpurun_out/ab_${v}${rep}.log | sed "s/^/$v$rep /"
  done
done
