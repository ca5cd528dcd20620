# round 5: table-driven exp in the MFMA pair K build -- tests, A/B against the library exp, PMC
set -o pipefail
O=gpurun_out/r5m; mkdir -p $O
timeout -k 10 600 python -u -m pytest -q --timeout 150 --timeout-method thread tests/test_gpu_kbuild.py \
  tests/test_gpu_parity.py tests/test_gpu_properties.py -m gpu > $O/tests.log 2>&1
rc=$?; grep -E "passed|failed|FAILED" $O/tests.log | tail -15
[ $rc -eq 124 ] || [ $rc -eq 134 ] || [ $rc -eq 137 ] || [ $rc -eq 139 ] && exit $rc
for v in "" libexp "" libexp; do
  L=gaussianprocessfundamentals_amd/libgpk.so; [ -n "$v" ] && L=variants/libgpk_$v.so
  echo "${v:-base} $(GPK_LIB=$L timeout -k 10 200 python tools/bench_kbuild.py C5 2>&1 | grep '^{' | cut -c1-140)"
done
export TMPDIR=/tmp
KB=$O/pmc; mkdir -p $KB; i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  [ $i -eq 3 ] && continue
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$(pwd)/$KB/p$i" -o run -- python tools/bench_kbuild.py C5 > $KB/p$i.log 2>&1 || exit 1
done < tools/pmc_kbuild.txt
python tools/pmc_kbuild_summary.py $KB 16384 8 > $KB/summary.txt 2>&1; cat $KB/summary.txt
exit $rc
