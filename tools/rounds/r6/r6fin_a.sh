# round 6 final tree, set A: full GPU suite + smoke(), default bench with CPU baseline, rocprofv3 stats of a short
# bench (the roofline kernel's average duration), the K-build cases
set -o pipefail
T=${T:-r06fin}; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error" $O/tests.log | head -20; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
grep smoke: $O/smoke.log
timeout -k 10 600 python bench.py > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
grep '^{' $O/bench.log > $O/bench_metric_b64_p2.json; cut -c1-200 $O/bench_metric_b64_p2.json
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$(pwd)/$O/prof" -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/prof.log 2>&1 || { tail -3 $O/prof.log; exit 1; }
grep '^{' $O/prof.log > $O/metric_b64_p2_bench_under_rocprof.json; cut -c1-200 $O/metric_b64_p2_bench_under_rocprof.json
timeout -k 10 120 python tools/bench_kbuild.py > $O/kbuild.jsonl 2>&1 || { tail -3 $O/kbuild.jsonl; exit 1; }
grep "^{" $O/kbuild.jsonl | cut -c1-200
echo done
