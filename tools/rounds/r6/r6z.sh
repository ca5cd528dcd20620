# round 6 last tree (after s128 auto for identity-augmented plans): full GPU suite + smoke, API latency, --mode grad
set -o pipefail
O=${O:-gpurun_out/r6z}; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
grep smoke: $O/smoke.log
timeout -k 10 300 python tools/bench_api_latency.py 256 1024 2048 4096 6144 8192 > $O/api.log 2>&1 || exit 1
grep '^{' $O/api.log > $O/api_latency.jsonl; cat $O/api_latency.jsonl
timeout -k 10 300 python bench.py --mode grad --steps 6 --warmup 2 --no-cpu-baseline > $O/grad.log 2>&1 || exit 1
grep '^{' $O/grad.log | cut -c1-200
exit 0
