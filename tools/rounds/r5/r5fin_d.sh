# round 5 final tree (4/4): drop-in API latency after the pinned-copy change
set -o pipefail
O=gpurun_out/r05fin; mkdir -p $O
timeout -k 10 300 python tools/bench_api_latency.py 256 1024 2048 4096 6144 8192 > $O/api2.log 2>&1 || { tail -3 $O/api2.log; exit 1; }
grep '^{' $O/api2.log > $O/api_latency.jsonl; cat $O/api_latency.jsonl
