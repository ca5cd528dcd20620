# round 5: full GPU suite (no -x: every failure), smoke, short default bench
set -o pipefail
O=${O:-gpurun_out/r5a}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread -rf -s ${PYTEST_ARGS:-} > $O/tests.log 2>&1
rc=$?
grep -E "passed|failed|FAILED|Error" $O/tests.log | tail -25
[ $rc -eq 124 ] || [ $rc -eq 134 ] || [ $rc -eq 137 ] || [ $rc -eq 139 ] && exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
[ "${RUN_BENCH:-1}" = "1" ] || exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-300
exit $rc
