# round 5: C2 as 8 persistent launches side by side (bench default now) -- chain tests, bench line, rocprof stats
set -o pipefail
O=gpurun_out/r5w; mkdir -p $O
timeout -k 10 600 python -u -m pytest -q --timeout 150 --timeout-method thread tests/test_gpu_chain.py -m gpu > $O/tests.log 2>&1
rc=$?; grep -E "passed|failed|FAILED" $O/tests.log | tail -8
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --config C2 --steps 300 --warmup 30 --cpu-seconds 10 > $O/c2.log 2>&1 || { tail -3 $O/c2.log; exit 1; }
grep '^{' $O/c2.log > $O/c2.json; python -c "
import json; d=json.load(open('$O/c2.json')); print(d['value'], d['ms_per_step'], d['config']['schedule']); print(d['roofline']); print(d['check'])"
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$(pwd)/$O/prof" -o run -- python bench.py --config C2 --steps 100 --warmup 20 --no-cpu-baseline --no-check > $O/prof.log 2>&1 || exit 1
grep '^{' $O/prof.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('under rocprof', d['value'], d['roofline']['avg_launch_us'])"
