# round 5: the two-leaf SE + periodic K build on MFMA in its own instantiation -- tests and K build A/B
set -o pipefail
O=gpurun_out/r5i; mkdir -p $O
timeout -k 10 600 python -u -m pytest -q --timeout 150 --timeout-method thread tests/test_gpu_kbuild.py \
  tests/test_gpu_parity.py tests/test_gpu_properties.py tests/test_gpu_approx_grad.py -m gpu > $O/tests.log 2>&1
rc=$?; grep -E "passed|failed|FAILED" $O/tests.log | tail -15
[ $rc -eq 124 ] || [ $rc -eq 134 ] || [ $rc -eq 137 ] || [ $rc -eq 139 ] && exit $rc
for v in "" nopairmfma "" nopairmfma; do
  L=gaussianprocessfundamentals_amd/libgpk.so; [ -n "$v" ] && L=variants/libgpk_$v.so
  GPK_LIB=$L timeout -k 10 200 python tools/bench_kbuild.py C5 >> $O/kbuild_${v:-base}.jsonl 2>&1 || exit 1
done
grep -h "^{" $O/kbuild_base.jsonl $O/kbuild_nopairmfma.jsonl
exit $rc
