# round 5: deferred-update depth (chain_group) and look-ahead distance for the identity-augmented persistent launch
set -o pipefail
O=gpurun_out/r5d; mkdir -p $O
for g in 2 4 8 16; do
  for la in 2 3; do
    GPK_CHAIN_GROUP=$g GPK_CHAIN_GROUP_LA=$la timeout -k 10 200 python tools/bench_api_latency.py 4096 8192 > $O/api_g${g}_la${la}.log 2>&1 || { tail -5 $O/api_g${g}_la${la}.log; exit 1; }
    echo "g=$g la=$la $(grep -h '^{' $O/api_g${g}_la${la}.log | cut -c1-90 | tr '\n' ' ')"
  done
done
