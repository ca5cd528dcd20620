# round 6: ADVICE r5 fixes (device timeout counter, planner knobs, Nystroem cutoff) + the eigen fallback beyond
# n = 16384 -- the touched GPU tests, then a short C2 bench (chain_timeouts_timed in its check)
set -o pipefail
O=${O:-gpurun_out/r6a}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_chain.py tests/test_gpu_syevd.py tests/test_gpu_nystroem_indefinite.py \
  tests/test_gpu_approx_metrics.py tests/test_gpu_strategies.py -m gpu -v --timeout 240 --timeout-method thread -rf -s \
  > $O/tests.log 2>&1
rc=$?
grep -E "passed|failed|FAILED|Error|m = 16400|n = 16400|duplicate" $O/tests.log | tail -30
[ $rc -eq 124 ] || [ $rc -eq 134 ] || [ $rc -eq 137 ] || [ $rc -eq 139 ] && exit $rc
timeout -k 10 300 python bench.py --config C2 --steps 200 --warmup 20 > $O/bench_c2.log 2>&1 || { tail -5 $O/bench_c2.log; exit 1; }
tail -1 $O/bench_c2.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['check'])"
exit $rc
