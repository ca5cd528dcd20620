# round 5: the C2 default (8 persistent launches x 64 workgroups) with roofline + CPU baseline, its rocprof stats
set -o pipefail
O=gpurun_out/r5ae; mkdir -p $O
timeout -k 10 300 python bench.py --config C2 --steps 300 --warmup 30 --cpu-seconds 10 > $O/c2.log 2>&1 || { tail -3 $O/c2.log; exit 1; }
grep '^{' $O/c2.log > $O/c2.json; python -c "
import json; d=json.load(open('$O/c2.json')); print(d['value'], d['ms_per_step'], d['config']['schedule']); print(d['roofline']); print(d['check']['rel_vs_oracle'], d['cpu_baseline']['value'])"
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$(pwd)/$O/prof" -o run -- python bench.py --config C2 --steps 100 --warmup 20 --no-cpu-baseline --no-check > $O/prof.log 2>&1 || exit 1
grep '^{' $O/prof.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('under rocprof', d['value'], d['roofline']['avg_launch_us'])"
