# round 6: deferred-update depth x near-diagonal sub-groups: C3 on the f32 persistent launch, value + gradient (eye plans)
set -o pipefail
O=${O:-gpurun_out/r6q}; mkdir -p $O
val() { python -c "import json;d=json.loads(open('$1').read().strip().splitlines()[-1]);print(d['value'])"; }
for spec in "8 2" "16 4" "16 2" "12 4" "8 4" "16 8"; do
  set -- $spec
  GPK_CHAIN_GROUP=$1 GPK_CHAIN_GROUP_NEAR=$2 GPK_BENCH_PERSIST_F32=1 timeout -k 10 300 python bench.py --config C3 --steps 40 --warmup 5 --no-cpu-baseline > $O/c3_g$1_n$2.json 2> $O/e.err || { tail -5 $O/e.err; exit 1; }
  echo "C3 f32 chain group=$1 near=$2: $(val $O/c3_g$1_n$2.json)"
done
for spec in "8 2" "8 4" "16 4" "12 4" "16 2"; do
  set -- $spec
  GPK_CHAIN_GROUP_EYE=$1 GPK_CHAIN_GROUP_NEAR=$2 timeout -k 10 200 python tools/bench_api_latency.py 4096 8192 > $O/api_e$1_n$2.jsonl 2>&1 || { tail -5 $O/api_e$1_n$2.jsonl; exit 1; }
  echo "eye group=$1 near=$2: $(grep '^{' $O/api_e$1_n$2.jsonl | python -c "
import json,sys
print(' '.join('%d: %.3f / %.3f' % (d['n'], d['get_metric_ms'], d['get_metric_and_gradient_ms']) for d in map(json.loads, sys.stdin)))")"
done
exit 0
