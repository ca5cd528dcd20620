# round 5: pre-pass over 4 waves per block; pair_fast_kernel occupancy A/B (GPK_FAST_MINB 4 default vs 3 / 5)
set -o pipefail
O=gpurun_out/r5r; mkdir -p $O
timeout -k 10 600 python -u -m pytest -q --timeout 150 --timeout-method thread tests/test_gpu_kbuild_pair.py \
  tests/test_gpu_kbuild.py tests/test_gpu_parity.py -m gpu > $O/tests.log 2>&1
rc=$?; grep -E "passed|failed|FAILED" $O/tests.log | tail -25
[ $rc -eq 124 ] || [ $rc -eq 134 ] || [ $rc -eq 137 ] || [ $rc -eq 139 ] && exit $rc
for v in "" fastminb3 fastminb5 "" fastminb3 fastminb5; do
  L=gaussianprocessfundamentals_amd/libgpk.so; [ -n "$v" ] && L=variants/libgpk_$v.so
  echo "${v:-base} $(GPK_LIB=$L timeout -k 10 200 python tools/bench_kbuild.py C5 2>&1 | grep '^{' | cut -c1-140)" | tee -a $O/ab.txt
done
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$(pwd)/$O/stats" -o run -- python tools/bench_kbuild.py C5 > $O/stats.log 2>&1 || exit 1
exit $rc
