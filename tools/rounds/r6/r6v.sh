# round 6: group look-ahead (chain_group_la 1 vs 2) and the eye plans' depth under the new defaults
set -o pipefail
O=${O:-gpurun_out/r6v}; mkdir -p $O
val() { python -c "import json;d=json.loads(open('$1').read().strip().splitlines()[-1]);print(d['value'])"; }
for rep in 1 2; do
  for v in "2 8" "1 8" "2 12" "2 16"; do
    set -- $v
    GPK_CHAIN_GROUP_LA=$1 GPK_CHAIN_GROUP_EYE=$2 timeout -k 10 300 python bench.py --config C2 --steps 200 --warmup 20 --no-cpu-baseline > $O/c2.json 2> $O/e.err || { tail -5 $O/e.err; exit 1; }
    GPK_CHAIN_GROUP_LA=$1 timeout -k 10 300 python bench.py --config C3 --steps 60 --warmup 10 --no-cpu-baseline > $O/c3.json 2> $O/e.err || { tail -5 $O/e.err; exit 1; }
    GPK_CHAIN_GROUP_LA=$1 GPK_CHAIN_GROUP_EYE=$2 timeout -k 10 200 python tools/bench_api_latency.py 4096 8192 > $O/api.jsonl 2>&1 || { tail -5 $O/api.jsonl; exit 1; }
    echo "rep $rep group_la=$1 group_eye=$2: C2 $(val $O/c2.json) C3 $(val $O/c3.json) api $(grep '^{' $O/api.jsonl | python -c "
import json,sys
print(' '.join('%d: %.3f / %.3f' % (d['n'], d['get_metric_ms'], d['get_metric_and_gradient_ms']) for d in map(json.loads, sys.stdin)))")"
  done
done
exit 0
