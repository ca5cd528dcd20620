# round 6: near sub-group look-ahead (chain_near_la 1 vs 2) and deferred depth 8 for f64 -- C2, C3 (f32 persistent), API
set -o pipefail
O=${O:-gpurun_out/r6u}; mkdir -p $O
GPK_CHAIN_NEAR_LA=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_chain_f32.py tests/test_gpu_chain.py -m gpu -x -q -k "bitwise" --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
val() { python -c "import json;d=json.loads(open('$1').read().strip().splitlines()[-1]);print(d['value'])"; }
for rep in 1 2; do
  for v in "2 0" "1 0" "1 8" "2 8"; do
    set -- $v
    GPK_CHAIN_NEAR_LA=$1 GPK_CHAIN_GROUP=$2 timeout -k 10 300 python bench.py --config C2 --steps 200 --warmup 20 --no-cpu-baseline > $O/c2.json 2> $O/e.err || { tail -5 $O/e.err; exit 1; }
    GPK_CHAIN_NEAR_LA=$1 timeout -k 10 300 python bench.py --config C3 --steps 60 --warmup 10 --no-cpu-baseline > $O/c3.json 2> $O/e.err || { tail -5 $O/e.err; exit 1; }
    GPK_CHAIN_NEAR_LA=$1 GPK_CHAIN_GROUP=$2 timeout -k 10 200 python tools/bench_api_latency.py 4096 8192 > $O/api.jsonl 2>&1 || { tail -5 $O/api.jsonl; exit 1; }
    echo "rep $rep near_la=$1 group=$2: C2 $(val $O/c2.json) C3 $(val $O/c3.json) api $(grep '^{' $O/api.jsonl | python -c "
import json,sys
print(' '.join('%d: %.3f / %.3f' % (d['n'], d['get_metric_ms'], d['get_metric_and_gradient_ms']) for d in map(json.loads, sys.stdin)))")"
  done
done
exit 0
