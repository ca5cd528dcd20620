# A/B of the chain's list-scheduling durations: old (28,7,7,18) vs the measured defaults
set -o pipefail
for rep in 1 2; do
  for d in "28,7,7,18" ""; do
    GPK_CHAIN_DUR=$d SETS='{"chain":1}' timeout -k 10 200 python tools/single_sched.py 1024 4096 6144 > gpurun_out/dur.log 2>&1 || { tail -5 gpurun_out/dur.log; exit 1; }
    grep '^{' gpurun_out/dur.log | sed "s/^/dur=${d:-measured} /"
  done
done
