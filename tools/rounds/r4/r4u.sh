# one Newton step + the non-positive pivot from the diagonal after the tile: probes, tests, spans
# (historical A/B script of round 4: the variant libraries it names were built with tools/build_variant.sh and removed after the measurement -- see DESIGN §4 for the outcome)
set -o pipefail
O=gpurun_out/r4u; mkdir -p $O
for b in lb_n1 lb_n2 oldbad_n2; do timeout -k 5 30 ./tools/probe/potf2_$b >> $O/probe.txt 2>&1 || exit 1; done
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_chain.py tests/test_gpu_parity.py tests/test_gpu_diag_versions.py tests/test_gpu_strategies.py tests/test_gpu_grad_handlings.py tests/test_gpu_dropin.py -m gpu > $O/tests.log 2>&1 || { echo "tests failed" >> $O/tests.log; exit 1; }
for v in "" n2 n2ob "" n2 n2ob; do
  L=gaussianprocessfundamentals_amd/libgpk.so; [ -n "$v" ] && L=variants/libgpk_$v.so
  GPK_LIB=$L SETS='{"chain":1};{"chain":0,"lookahead":2}' timeout -k 10 300 python tools/single_sched.py 1024 4096 8192 >> $O/ab_${v:-base}.jsonl 2>&1 || exit 1
done
