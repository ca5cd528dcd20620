# round 5 last tree: every BASELINE config with roofline + cpu_baseline, C2 one at a time, --mode grad, the drop-in
# API latency (the C4 slices and per-config rocprof of r5fin_b.sh are unchanged by the last trees' changes)
set -o pipefail
T=r05fin3; O=gpurun_out/$T; mkdir -p $O; : > $O/configs.jsonl; : > $O/c4_slices.jsonl
export TMPDIR=/tmp
for spec in "metric 10 3" "C2 300 30" "C3 60 10" "C4 20 3" "C5 20 4"; do
  set -- $spec
  timeout -k 10 400 python bench.py --config $1 --steps $2 --warmup $3 --cpu-seconds 10 > $O/cfg_$1.log 2>&1 || { tail -5 $O/cfg_$1.log; exit 1; }
  grep '^{' $O/cfg_$1.log >> $O/configs.jsonl
  tail -1 $O/configs.jsonl | python -c "
import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; k=d.get('kbuild_roofline') or {}
print('$1', d['value'], d['unit'], 'roofline', r['achieved'], '/', r['peak'], r['frac'], 'kbuild', k.get('achieved'), k.get('frac'), 'cpu', d['cpu_baseline']['value'])"
done
timeout -k 10 300 python bench.py --config C2 --batch 1 --pipeline 1 --steps 200 --warmup 10 --no-cpu-baseline > $O/cfg_c2_single.log 2>&1 || exit 1
grep '^{' $O/cfg_c2_single.log >> $O/configs.jsonl
timeout -k 10 300 python bench.py --mode grad --steps 6 --warmup 2 --no-cpu-baseline > $O/cfg_grad.log 2>&1 || exit 1
grep '^{' $O/cfg_grad.log >> $O/configs.jsonl
timeout -k 10 300 python tools/bench_api_latency.py 256 1024 2048 4096 6144 8192 > $O/api.log 2>&1 || exit 1
grep '^{' $O/api.log > $O/api_latency.jsonl; cat $O/api_latency.jsonl
echo done
