# round 6: chain_group_near (near-diagonal tile updates in sub-groups) -- tests under it, C3 f32 persistent / C2 / API
set -o pipefail
O=${O:-gpurun_out/r6p}; mkdir -p $O
GPK_CHAIN_GROUP_NEAR=2 timeout -k 10 600 python -u -m pytest tests/test_gpu_chain_f32.py tests/test_gpu_chain.py -m gpu -x -q -k "bitwise or f32" --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
val() { python -c "import json;d=json.loads(open('$1').read().strip().splitlines()[-1]);print(d['value'])"; }
for rep in 1 2; do
  for nn in 1 2 4; do
    GPK_CHAIN_GROUP_NEAR=$nn GPK_BENCH_PERSIST_F32=1 timeout -k 10 300 python bench.py --config C3 --steps 40 --warmup 5 --no-cpu-baseline > $O/c3_n$nn.json 2> $O/e.err || { tail -5 $O/e.err; exit 1; }
    echo "rep $rep C3 f32 chain near=$nn: $(val $O/c3_n$nn.json)"
  done
done
for rep in 1 2; do
  for nn in 1 2; do
    GPK_CHAIN_GROUP_NEAR=$nn timeout -k 10 300 python bench.py --config C2 --steps 200 --warmup 20 --no-cpu-baseline > $O/c2_n$nn.json 2> $O/e.err || { tail -5 $O/e.err; exit 1; }
    echo "rep $rep C2 near=$nn: $(val $O/c2_n$nn.json)"
    GPK_CHAIN_GROUP_NEAR=$nn timeout -k 10 200 python tools/bench_api_latency.py 4096 8192 > $O/api_n$nn.jsonl 2>&1 || { tail -5 $O/api_n$nn.jsonl; exit 1; }
    echo "   api near=$nn: $(grep '^{' $O/api_n$nn.jsonl | tr '\n' ' ')"
  done
done
exit 0
