# round 5: small-N API latency, persistent launch vs launch path
set -o pipefail
O=gpurun_out/r5ak; mkdir -p $O; : > $O/api.jsonl
for c in 1 0 1 0; do
  GPK_CHAIN=$c timeout -k 10 300 python tools/bench_api_latency.py 128 256 384 512 768 1024 > $O/api_$c.log 2>&1 || { tail -3 $O/api_$c.log; exit 1; }
  grep '^{' $O/api_$c.log | sed "s/^{/{\"chain\": $c, /" | tee -a $O/api.jsonl
done
