# round 5: utilisation of the persistent launch (value / value + gradient) and the gradient call's kernels
set -o pipefail
O=gpurun_out/r5f; mkdir -p $O
for a in "4096" "4096 eye" "8192" "8192 eye"; do
  timeout -k 10 120 python tools/chain_util.py $a > "$O/util_${a// /_}.txt" 2>&1 || { tail -5 "$O/util_${a// /_}.txt"; exit 1; }
  cat "$O/util_${a// /_}.txt"
done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o grad -- python tools/bench_api_latency.py 8192 > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
find $O/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $O/grad8192_kernel_stats.csv
cut -d, -f1-8 $O/grad8192_kernel_stats.csv | head -14
