# packed potf2 (factor + inverse in the two halves of the wave) and one-Newton-step variants
# (historical A/B script of round 4: the variant libraries it names were built with tools/build_variant.sh and removed after the measurement -- see DESIGN §4 for the outcome)
set -o pipefail
O=gpurun_out/r4n; mkdir -p $O
timeout -k 5 60 ./tools/probe/permlane_probe > $O/permlane.txt 2>&1 && timeout -k 5 60 ./tools/probe/lat_probe > $O/lat.txt 2>&1 || exit 1
GPK_LIB=variants/libgpk_pack1.so timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_chain.py tests/test_gpu_parity.py tests/test_gpu_diag_versions.py -m gpu > $O/tests_pack1.log 2>&1 || { echo "tests failed" >> $O/tests_pack1.log; exit 1; }
GPK_LIB=variants/libgpk_pack1n1.so timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -m gpu > $O/tests_pack1n1.log 2>&1 || { echo "tests failed" >> $O/tests_pack1n1.log; }
for v in "" pack1 pack1n1 spref1 trail2; do
  L=gaussianprocessfundamentals_amd/libgpk.so; [ -n "$v" ] && L=variants/libgpk_$v.so
  GPK_LIB=$L SETS='{"chain":1};{"chain":0,"lookahead":2}' timeout -k 10 300 python tools/single_sched.py 1024 4096 8192 > $O/ab_${v:-base}.jsonl 2>&1 || exit 1
done
GPK_LIB=variants/libgpk_dprofpk.so timeout -k 10 120 python tools/diag_phase_prof.py 4096 > $O/dphase.txt 2>&1 || exit 1
GPK_CHAIN_DBG=13 GPK_LIB=variants/libgpk_dprofpk.so timeout -k 10 120 python tools/diag_phase_prof.py 4096 > $O/dphase_d13.txt 2>&1 || exit 1
GPK_LIB=variants/libgpk_pack1.so timeout -k 10 120 python tools/chain_prof.py 4096 > $O/prof.txt 2>&1 || exit 1
GPK_LIB=variants/libgpk_dprof.so timeout -k 10 120 python tools/diag_phase_prof.py 4096 > $O/dphase_base.txt 2>&1 || exit 1
