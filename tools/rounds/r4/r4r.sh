# L_kk stored after the diagonal task's hand-off: tests, spans vs the previous order, per-task profile
set -o pipefail
O=gpurun_out/r4r; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_chain.py tests/test_gpu_parity.py tests/test_gpu_dropin.py -m gpu > $O/tests.log 2>&1 || { echo "tests failed" >> $O/tests.log; exit 1; }
for v in "" deferl0 "" deferl0; do
  L=gaussianprocessfundamentals_amd/libgpk.so; [ -n "$v" ] && L=variants/libgpk_$v.so
  GPK_LIB=$L SETS='{"chain":1}' timeout -k 10 300 python tools/single_sched.py 1024 2048 4096 8192 >> $O/ab_${v:-base}.jsonl 2>&1 || exit 1
done
timeout -k 10 120 python tools/chain_prof.py 4096 > $O/prof.txt 2>&1 || exit 1
GPK_LIB=variants/libgpk_dprof.so timeout -k 10 120 python tools/diag_phase_prof.py 4096 > $O/dphase.txt 2>&1 || exit 1
