# list-scheduling durations of the persistent factorisation's planner (GPK_CHAIN_DUR = D,S,U32,BLK us)
set -o pipefail
O=gpurun_out/r4y; mkdir -p $O
for rep in 1 2; do for d in "32,7,10,24" "28,6.5,12,22.5" "28,6.5,10,22.5" "28,6.5,12,28"; do
  GPK_CHAIN_DUR=$d SETS='{"chain":1}' timeout -k 10 300 python tools/single_sched.py 4096 6144 8192 > $O/tmp.jsonl 2>&1 || exit 1
  grep '^{' $O/tmp.jsonl | sed "s/^{/{\"dur\": \"$d\", /" >> $O/ab.jsonl
done; done
