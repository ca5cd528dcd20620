# round 5: C2 persistent launches in flight -- sweep of launches in flight x workgroups per launch
set -o pipefail
O=gpurun_out/r5v; mkdir -p $O; : > $O/c2.txt
for pg in "6 42" "8 32" "8 40" "8 48" "12 21" "16 16" "10 25" "8 32"; do
  set -- $pg
  GPK_CHAIN_GRID=$2 timeout -k 10 200 python bench.py --config C2 --pipeline $1 --chain 2 --steps 300 --warmup 30 --no-cpu-baseline --no-check > $O/c2.log 2>&1 || { tail -3 $O/c2.log; exit 1; }
  echo "P=$1 grid=$2 $(grep '^{' $O/c2.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" | tee -a $O/c2.txt
done
