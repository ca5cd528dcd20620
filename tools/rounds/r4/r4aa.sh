# S's first column half on D's mid-way flag: tests, spans vs without, per-task profile
set -o pipefail
O=gpurun_out/r4ad; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_chain.py tests/test_gpu_parity.py tests/test_gpu_dropin.py -m gpu > $O/tests.log 2>&1 || { echo "tests failed" >> $O/tests.log; exit 1; }
for v in "" r96 "" r96; do
  L=gaussianprocessfundamentals_amd/libgpk.so; [ -n "$v" ] && L=variants/libgpk_$v.so
  GPK_LIB=$L SETS='{"chain":1}' timeout -k 10 300 python tools/single_sched.py 1024 2048 4096 6144 8192 >> $O/ab_${v:-base}.jsonl 2>&1 || exit 1
done
timeout -k 10 120 python tools/chain_prof.py 4096 > $O/prof.txt 2>&1 || exit 1
