# round 6: chain_s128 (block-row panel solves) -- bitwise tests under it, then C2 / C3 / API against per-slice solves
set -o pipefail
O=${O:-gpurun_out/r6x}; mkdir -p $O
GPK_CHAIN_S128=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_chain_f32.py tests/test_gpu_chain.py tests/test_gpu_grad.py -m gpu -x -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
val() { python -c "import json;d=json.loads(open('$1').read().strip().splitlines()[-1]);print(d['value'])"; }
for rep in 1 2; do
  for v in 0 1 2; do
    GPK_CHAIN_S128=$v timeout -k 10 300 python bench.py --config C2 --steps 200 --warmup 20 --no-cpu-baseline > $O/c2.json 2> $O/e.err || { tail -5 $O/e.err; exit 1; }
    GPK_CHAIN_S128=$v timeout -k 10 300 python bench.py --config C3 --steps 60 --warmup 10 --no-cpu-baseline > $O/c3.json 2> $O/e.err || { tail -5 $O/e.err; exit 1; }
    GPK_CHAIN_S128=$v timeout -k 10 200 python tools/bench_api_latency.py 4096 8192 > $O/api.jsonl 2>&1 || { tail -5 $O/api.jsonl; exit 1; }
    echo "rep $rep s128=$v: C2 $(val $O/c2.json) C3 $(val $O/c3.json) api $(grep '^{' $O/api.jsonl | python -c "
import json,sys
print(' '.join('%d: %.3f / %.3f' % (d['n'], d['get_metric_ms'], d['get_metric_and_gradient_ms']) for d in map(json.loads, sys.stdin)))")"
  done
done
exit 0
