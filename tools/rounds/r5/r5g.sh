# round 5: SQ tasks (chain_uq 2: panel solve + quarter updates of the next diagonal block in one task) -- tests, spans, profile
set -o pipefail
O=gpurun_out/r5g; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_chain.py -m gpu > $O/tests.log 2>&1 || { tail -15 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for u in 1 2 1 2; do
  GPK_CHAIN_UQ=$u SETS='{"chain":1}' timeout -k 10 300 python tools/single_sched.py 1024 2048 4096 8192 >> $O/ab_uq$u.jsonl 2>&1 || exit 1
done
grep -h "^{" $O/ab_uq1.jsonl $O/ab_uq2.jsonl | cut -c1-100
GPK_CHAIN_UQ=2 timeout -k 10 120 python tools/chain_prof.py 4096 > $O/prof_uq2.txt 2>&1 || exit 1
tail -2 $O/prof_uq2.txt
GPK_CHAIN_UQ=2 timeout -k 10 200 python tools/bench_api_latency.py 4096 8192 > $O/api_uq2.log 2>&1 || exit 1
grep -h "^{" $O/api_uq2.log
