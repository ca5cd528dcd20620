# round 6: defaults after chain_u128 auto -- chain GPU tests, C3 f32 persistent vs the launch path (alternating),
# f32 depth variants, C2, API latency
set -o pipefail
O=${O:-gpurun_out/r6s}; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_chain_f32.py tests/test_gpu_chain.py tests/test_gpu_grad*.py -m gpu -x -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
val() { python -c "import json;d=json.loads(open('$1').read().strip().splitlines()[-1]);print(d['value'])"; }
for rep in 1 2; do
  GPK_BENCH_PERSIST_F32=1 timeout -k 10 300 python bench.py --config C3 --steps 60 --warmup 10 --no-cpu-baseline > $O/c3_chain.json 2> $O/e.err || { tail -5 $O/e.err; exit 1; }
  timeout -k 10 300 python bench.py --config C3 --steps 60 --warmup 10 --no-cpu-baseline > $O/c3_launch.json 2> $O/e.err || { tail -5 $O/e.err; exit 1; }
  GPK_CHAIN_GROUP=12 GPK_CHAIN_GROUP_NEAR=4 GPK_BENCH_PERSIST_F32=1 timeout -k 10 300 python bench.py --config C3 --steps 60 --warmup 10 --no-cpu-baseline > $O/c3_chain_g12.json 2> $O/e.err || { tail -5 $O/e.err; exit 1; }
  GPK_BENCH_PERSIST_F32=1 GPK_BENCH_PERSIST_P=6 GPK_BENCH_PERSIST_SHARE=3 timeout -k 10 300 python bench.py --config C3 --steps 60 --warmup 10 --no-cpu-baseline > $O/c3_chain_p6s3.json 2> $O/e.err || { tail -5 $O/e.err; exit 1; }
  echo "rep $rep C3: f32 chain $(val $O/c3_chain.json) launch $(val $O/c3_launch.json) chain g12n4 $(val $O/c3_chain_g12.json) chain p6s3 $(val $O/c3_chain_p6s3.json)"
done
timeout -k 10 300 python bench.py --config C2 --steps 300 --warmup 30 --no-cpu-baseline > $O/c2.json 2> $O/e.err || { tail -5 $O/e.err; exit 1; }
echo "C2 $(val $O/c2.json)"
timeout -k 10 200 python tools/bench_api_latency.py 1024 2048 4096 6144 8192 > $O/api.jsonl 2>&1 || { tail -5 $O/api.jsonl; exit 1; }
grep '^{' $O/api.jsonl
exit 0
