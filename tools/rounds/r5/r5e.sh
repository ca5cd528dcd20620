# round 5: corner-tile grouping of the identity-augmented persistent launch (GPK_CHAIN_GROUP_CORNER / _TAIL)
set -o pipefail
O=gpurun_out/r5e; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_chain.py -m gpu -k "eye" > $O/tests.log 2>&1 || { tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for gc in 4 8 16; do
  for t in 4 8 16; do
    GPK_CHAIN_GROUP_CORNER=$gc GPK_CHAIN_CORNER_TAIL=$t timeout -k 10 200 python tools/bench_api_latency.py 4096 8192 > $O/api_${gc}_${t}.log 2>&1 || { tail -5 $O/api_${gc}_${t}.log; exit 1; }
    echo "gc=$gc tail=$t $(grep -h '^{' $O/api_${gc}_${t}.log | sed 's/"get_metric_ms"[^,]*,//; s/"last_nlml".*//' | tr '\n' ' ')"
  done
done
