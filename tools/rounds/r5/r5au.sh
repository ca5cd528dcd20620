# round 5: bench lines after the host-path change (metric default, C2 persistent side by side, --mode grad)
set -o pipefail
O=gpurun_out/r5au; mkdir -p $O
true
true
timeout -k 10 300 python bench.py --config C2 --steps 300 --warmup 30 --no-cpu-baseline > $O/c2.log 2>&1 || { tail -3 $O/c2.log; exit 1; }
grep '^{' $O/c2.log | cut -c1-200
timeout -k 10 300 python bench.py --mode grad --steps 5 --warmup 2 --no-cpu-baseline > $O/grad.log 2>&1 || { tail -3 $O/grad.log; exit 1; }
grep '^{' $O/grad.log | cut -c1-200
