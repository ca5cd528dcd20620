# C2 (N = 4096 fp64, SE) throughput by candidates per launch and launches in flight; API latency
set -o pipefail
O=${R4O_OUT:-gpurun_out/r4o}; mkdir -p $O
for bp in "1 4" "1 1" "4 1" "4 2" "8 1" "8 2" "16 2"; do
  set -- $bp
  timeout -k 10 200 python bench.py --config C2 --batch $1 --pipeline $2 --steps 100 --warmup 10 --no-cpu-baseline --no-check > $O/c2_b$1_p$2.log 2>&1 || exit 1
  grep '^{' $O/c2_b$1_p$2.log | cut -c1-160
done
timeout -k 10 300 python tools/bench_api_latency.py 1024 2048 4096 6144 8192 > $O/api.log 2>&1 || exit 1
grep '^{' $O/api.log
