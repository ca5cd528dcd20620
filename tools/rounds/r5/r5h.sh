# round 5: SQ tasks (chain_uq 2) and the two-leaf SE + periodic K build on MFMA -- tests, spans, profile, K build A/B
set -o pipefail
O=gpurun_out/r5h; mkdir -p $O
timeout -k 10 600 python -u -m pytest -q --timeout 150 --timeout-method thread tests/test_gpu_chain.py tests/test_gpu_kbuild.py \
  tests/test_gpu_parity.py tests/test_gpu_properties.py tests/test_gpu_dropin.py -m gpu > $O/tests.log 2>&1
rc=$?; grep -E "passed|failed|FAILED" $O/tests.log | tail -15
[ $rc -eq 124 ] || [ $rc -eq 134 ] || [ $rc -eq 137 ] || [ $rc -eq 139 ] && exit $rc
for v in "" nopairmfma "" nopairmfma; do
  L=gaussianprocessfundamentals_amd/libgpk.so; [ -n "$v" ] && L=variants/libgpk_$v.so
  GPK_LIB=$L timeout -k 10 200 python tools/bench_kbuild.py C5 >> $O/kbuild_${v:-base}.jsonl 2>&1 || exit 1
done
grep -h "^{" $O/kbuild_base.jsonl $O/kbuild_nopairmfma.jsonl
for u in 1 2 1 2; do
  GPK_CHAIN_UQ=$u SETS='{"chain":1}' timeout -k 10 300 python tools/single_sched.py 1024 2048 4096 8192 >> $O/ab_uq$u.jsonl 2>&1 || exit 1
done
grep -h "^{" $O/ab_uq1.jsonl $O/ab_uq2.jsonl | cut -c1-100
GPK_CHAIN_UQ=2 timeout -k 10 120 python tools/chain_prof.py 4096 > $O/prof_uq2.txt 2>&1 || exit 1
tail -2 $O/prof_uq2.txt
GPK_CHAIN_UQ=2 timeout -k 10 200 python tools/bench_api_latency.py 4096 8192 > $O/api_uq2.log 2>&1 || exit 1
grep -h "^{" $O/api_uq2.log
exit $rc
