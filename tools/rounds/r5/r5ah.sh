# round 5: pinned asynchronous H2D of hyperparameters / noise -- full GPU suite, API latency A/B
set -o pipefail
O=gpurun_out/r5ah; mkdir -p $O; : > $O/api.jsonl
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -ne 0 ] && { grep FAILED $O/tests.log | head; exit $rc; }
for v in 1 0 1 0; do
  GPK_PINNED_H2D=$v timeout -k 10 300 python tools/bench_api_latency.py 256 1024 4096 > $O/api_$v.log 2>&1 || { tail -3 $O/api_$v.log; exit 1; }
  grep '^{' $O/api_$v.log | sed "s/^{/{\"pinned\": $v, /" | tee -a $O/api.jsonl
done
