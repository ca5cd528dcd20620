# round 6 final tree, set B: every BASELINE config with roofline + cpu_baseline, C2 one at a time, --mode grad, the
# C4 per-rank slices, the --dist rehearsals, the drop-in API latency, posterior timing
set -o pipefail
T=${T:-r06fin}; O=gpurun_out/$T; mkdir -p $O; : > $O/configs.jsonl
export TMPDIR=/tmp
for spec in "metric 10 3" "C2 300 30" "C3 60 10" "C4 20 3" "C5 20 4"; do
  set -- $spec
  timeout -k 10 400 python bench.py --config $1 --steps $2 --warmup $3 --cpu-seconds 10 > $O/cfg_$1.log 2>&1 || { tail -5 $O/cfg_$1.log; exit 1; }
  grep '^{' $O/cfg_$1.log >> $O/configs.jsonl
  tail -1 $O/configs.jsonl | python -c "
import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; k=d.get('kbuild_roofline') or {}
print('$1', d['value'], d['unit'], 'roofline', r['achieved'], '/', r['peak'], r['frac'], 'kbuild', k.get('achieved'), k.get('frac'), 'cpu', d['cpu_baseline']['value'], 'check', d['check'].get('rel_vs_oracle'))"
done
timeout -k 10 300 python bench.py --config C2 --batch 1 --pipeline 1 --steps 200 --warmup 10 --no-cpu-baseline > $O/cfg_c2_single.log 2>&1 || exit 1
grep '^{' $O/cfg_c2_single.log >> $O/configs.jsonl
timeout -k 10 300 python bench.py --mode grad --steps 6 --warmup 2 --no-cpu-baseline > $O/cfg_grad.log 2>&1 || exit 1
grep '^{' $O/cfg_grad.log >> $O/configs.jsonl
STEPS=30 bash tools/c4_slices.sh $O/c4_slices.jsonl || exit 1
python -c "
import json
rows=[json.loads(l) for l in open('$O/c4_slices.jsonl')]
base=rows[0]['ms_per_step']
for r in rows:
    w=r.get('slice',{}).get('of_world',1); print('W', w, r['ms_per_step'], 'eff', round(base/w/r['ms_per_step'],4))"
timeout -k 10 300 python bench.py --dist --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_dist_rehearsal.log 2>&1 || exit 1
grep '^{' $O/bench_dist_rehearsal.log > $O/bench_dist_rehearsal.json; cut -c1-160 $O/bench_dist_rehearsal.json
timeout -k 10 300 python bench.py --config C2 --dist --steps 300 --warmup 30 --no-cpu-baseline > $O/bench_c2_dist.log 2>&1 || exit 1
grep '^{' $O/bench_c2_dist.log > $O/bench_c2_dist_rehearsal.json; cut -c1-160 $O/bench_c2_dist_rehearsal.json
timeout -k 10 300 python tools/bench_api_latency.py 256 1024 2048 4096 6144 8192 > $O/api.log 2>&1 || exit 1
grep '^{' $O/api.log > $O/api_latency.jsonl; cat $O/api_latency.jsonl
timeout -k 10 300 python tools/bench_posterior.py 4096 1024 > $O/posterior.log 2>&1 || exit 1
timeout -k 10 300 python tools/bench_posterior.py 8192 2048 >> $O/posterior.log 2>&1 || exit 1
grep '^{' $O/posterior.log > $O/posterior.jsonl; cat $O/posterior.jsonl
echo done
