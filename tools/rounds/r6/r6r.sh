# round 6: chain_u128 (block-row tile updates of the next panel's column) -- bitwise tests under it, then C3 f32
# persistent, C2, API latency against the slice updates, alternating
set -o pipefail
O=${O:-gpurun_out/r6r}; mkdir -p $O
GPK_CHAIN_U128=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_chain_f32.py tests/test_gpu_chain.py -m gpu -x -q -k "bitwise or f32" --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
val() { python -c "import json;d=json.loads(open('$1').read().strip().splitlines()[-1]);print(d['value'])"; }
for rep in 1 2; do
  for u in 0 1; do
    GPK_CHAIN_U128=$u GPK_BENCH_PERSIST_F32=1 timeout -k 10 300 python bench.py --config C3 --steps 40 --warmup 5 --no-cpu-baseline > $O/c3_u$u.json 2> $O/e.err || { tail -5 $O/e.err; exit 1; }
    GPK_CHAIN_U128=$u timeout -k 10 300 python bench.py --config C2 --steps 200 --warmup 20 --no-cpu-baseline > $O/c2_u$u.json 2> $O/e.err || { tail -5 $O/e.err; exit 1; }
    GPK_CHAIN_U128=$u timeout -k 10 200 python tools/bench_api_latency.py 4096 8192 > $O/api_u$u.jsonl 2>&1 || { tail -5 $O/api_u$u.jsonl; exit 1; }
    echo "rep $rep u128=$u: C3 f32 chain $(val $O/c3_u$u.json) C2 $(val $O/c2_u$u.json) api $(grep '^{' $O/api_u$u.jsonl | python -c "
import json,sys
print(' '.join('%d: %.3f / %.3f' % (d['n'], d['get_metric_ms'], d['get_metric_and_gradient_ms']) for d in map(json.loads, sys.stdin)))")"
  done
done
exit 0
