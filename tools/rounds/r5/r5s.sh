# round 5: C2 pipelined throughput, round-4 protocol (100 steps, 10 warmup, no CPU baseline) vs the r5cfg one
set -o pipefail
O=gpurun_out/r5s; mkdir -p $O; : > $O/c2.jsonl
for a in "--warmup 10 --no-cpu-baseline --no-check" "--warmup 3 --cpu-seconds 10" "--warmup 10 --no-cpu-baseline --no-check" "--warmup 3 --no-cpu-baseline --no-check"; do
  timeout -k 10 200 python bench.py --config C2 --steps 100 $a > $O/c2.log 2>&1 || { tail -3 $O/c2.log; exit 1; }
  echo "$a $(grep '^{' $O/c2.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" | tee -a $O/c2.txt
done
