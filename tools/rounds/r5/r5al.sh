# round 5: value + gradient latency around N = 1024 .. 3072, persistent launch (forced) vs launch path, then the
# auto mode with the new minimum sizes (chain_min_p 768, chain_min_p_eye 2304)
set -o pipefail
O=gpurun_out/r5al; mkdir -p $O; : > $O/api.jsonl
for c in 2 0 2 0 1; do
  GPK_CHAIN=$c timeout -k 10 300 python tools/bench_api_latency.py 256 512 768 1024 1280 1536 2048 3072 > $O/api_$c.log 2>&1 || { tail -3 $O/api_$c.log; exit 1; }
  grep '^{' $O/api_$c.log | sed "s/^{/{\"chain\": $c, /" | tee -a $O/api.jsonl
done
