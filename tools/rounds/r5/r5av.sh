# round 5: bench after the per-slot priming pass: C2 with the default 3 warm-up steps, then the default metric line
set -o pipefail
O=gpurun_out/r5av; mkdir -p $O
timeout -k 10 300 python bench.py --config C2 --no-cpu-baseline > $O/c2.log 2>&1 || { tail -3 $O/c2.log; exit 1; }
grep '^{' $O/c2.log | cut -c1-200
timeout -k 10 300 python bench.py --config C2 --steps 300 --warmup 30 --no-cpu-baseline > $O/c2_300.log 2>&1 || { tail -3 $O/c2_300.log; exit 1; }
grep '^{' $O/c2_300.log | cut -c1-200
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/metric.log 2>&1 || { tail -3 $O/metric.log; exit 1; }
grep '^{' $O/metric.log | cut -c1-200
